"""CPU restatement of simple_reporter's tile stage — TEST INFRASTRUCTURE ONLY.

rows_from_reports: simple_reporter.py:176-196 (filter, duration/start/end, hour
    buckets) as binary rows, trace by trace in report order (the order the device K9
    stage writes them).
lines_of: simple_reporter.py:188-195 row text.
sort_and_cull: simple_reporter.py:216-239 — whole-line string sort and the reference's
    cull loop, restated line for line (pinned by tests/golden/cull_cases.json).
stream_rows_from_reports / stream_tiles: the Java streaming path — BatchingProcessor.java:
    108-141 (Segment.valid), TimeQuantisedTile.java:26-35, Collections.sort by
    Segment.compareTo (Segment.java:50-53, stable), AnonymisingProcessor.clean (:155-175,
    the same loop), Segment.appendToStringBuffer (Segment.java:59-74).
"""
import math

import numpy as np

TILE_ROW = np.dtype([('file', '<u8'), ('id', '<u8'), ('next_id', '<u8'), ('start', '<i8'), ('end', '<i8'),
                     ('duration', '<i4'), ('length', '<i4'), ('queue_length', '<i4'), ('speed_bin', '<i4')])
INVALID_SEGMENT_ID = 0x3fffffffffff
NO_ID = 0xFFFFFFFFFFFFFFFF


def _py2_round_int(x):
    f = math.floor(x)
    return int(f + 1 if x - f >= 0.5 else f) if x >= 0 else -_py2_round_int(-x)


def speed_bin(length, t0, t1):
    """The report's 20 km/h speed bin (0..7) carried by the rows (otr_tile_row.speed_bin)."""
    kmh = (length / (t1 - t0)) * 3.6
    return min(max(int(kmh / 20.0), 0), 7)


def rows_from_reports(res, first_time, last_time, q=3600):
    out = []
    off = res['trace_rep_off']
    for t in range(len(off) - 1):
        buckets = (int(last_time[t]) - int(first_time[t])) // q + 1          # :176 (py2 int /)
        for k in range(off[t], off[t + 1]):
            t0, t1 = float(res['rep_t0'][k]), float(res['rep_t1'][k])
            ln, qu = int(res['rep_length'][k]), int(res['rep_queue'][k])
            if not (t0 > 0 and t1 > 0 and t1 - t0 > .5 and ln > 0 and qu >= 0):  # :177
                continue
            duration = _py2_round_int(t1 - t0)                                # :179
            start, end = int(math.floor(t0)), int(math.ceil(t1))              # :180-181
            mn, mx = start // q, end // q                                     # :182-183
            if mx - mn > buckets:                                             # :184-187
                continue
            sid = int(res['rep_id'][k])
            nx = int(res['rep_next'][k])
            nx = INVALID_SEGMENT_ID if nx == NO_ID else nx                    # :193
            sb = speed_bin(ln, t0, t1)
            for b in range(mn, mx + 1):                                       # :188
                f = (b << 25) | ((sid & 7) << 22) | ((sid >> 3) & 0x3FFFFF)    # :189-191
                out.append((f, sid, nx, start, end, duration, ln, qu, sb))
    return np.array(out, dtype=TILE_ROW) if out else np.zeros(0, TILE_ROW)


def file_name(f, q=3600):
    b = int(f) >> 25
    return '%d_%d/%d/%d' % (b * q, (b + 1) * q - 1, (int(f) >> 22) & 7, int(f) & 0x3FFFFF)


def lines_of(rows, source='smpl_rprt', mode='auto'):
    return ['%d,%d,%d,1,%d,%d,%d,%d,%s,%s\n' % (int(r['id']), int(r['next_id']), int(r['duration']),
                                                int(r['length']), int(r['queue_length']), int(r['start']),
                                                int(r['end']), source, mode.upper()) for r in rows]


def sort_and_cull(lines, privacy):
    segments = sorted(lines)                        # :218
    start = 0
    i = 0
    while i < len(segments):                        # :221-239
        s = segments[start].split(',')
        e = segments[i].split(',')
        if s[0] != e[0] or s[1] != e[1] or i == len(segments) - 1:
            if i == len(segments) - 1:
                i += 1
            if i - start < privacy:
                segments[start:i] = []
                i = start
            else:
                start = i
        i += 1
    return segments


def tiles(rows, privacy, q=3600, source='smpl_rprt', mode='auto'):
    """{file name: kept lines} for rows of any order (files built as :188-196 appends)."""
    by_file = {}
    for r, line in zip(rows, lines_of(rows, source, mode)):
        by_file.setdefault(file_name(r['file'], q), []).append(line)
    out = {}
    for k, v in by_file.items():
        kept = sort_and_cull(v, privacy)
        if kept:                                    # :242-244
            out[k] = kept
    return out


def _java_round(x):
    """Math.round(double): closest long, ties toward positive infinity."""
    f = math.floor(x)
    return int(f + 1 if x - f >= 0.5 else f)


def stream_rows_from_reports(res, q=3600):
    out = []
    off = res['trace_rep_off']
    for t in range(len(off) - 1):
        for k in range(off[t], off[t + 1]):
            t0, t1 = float(res['rep_t0'][k]), float(res['rep_t1'][k])
            ln, qu = int(res['rep_length'][k]), int(res['rep_queue'][k])
            if not (t0 > 0 and t1 > 0 and t1 > t0 and ln > 0 and qu >= 0):   # Segment.valid
                continue
            sid = int(res['rep_id'][k])
            nx = int(res['rep_next'][k])
            nx = INVALID_SEGMENT_ID if nx == NO_ID else nx                    # Segment.java:26
            for b in range(int(t0) // q, int(t1) // q + 1):                   # getTiles: (long) casts
                f = (b << 25) | ((sid & 7) << 22) | ((sid >> 3) & 0x3FFFFF)
                out.append((f, sid, nx, int(math.floor(t0)), int(math.ceil(t1)), _java_round(t1 - t0), ln, qu,
                            speed_bin(ln, t0, t1)))
    return np.array(out, dtype=TILE_ROW) if out else np.zeros(0, TILE_ROW)


def java_clean(rows, privacy):
    """AnonymisingProcessor.clean over rows already in Segment.compareTo order."""
    segs = list(rows)
    start = 0
    i = 0
    while i < len(segs):
        s, e = segs[start], segs[i]
        if s['id'] != e['id'] or s['next_id'] != e['next_id'] or i == len(segs) - 1:
            if i == len(segs) - 1:
                i += 1
            if i - start < privacy:
                del segs[start:i]
                i = start
            else:
                start = i
        i += 1
    return segs


def java_line(r, source, mode):
    nx = '' if int(r['next_id']) == INVALID_SEGMENT_ID else str(int(r['next_id']))
    return '\n%d,%s,%d,1,%d,%d,%d,%d,%s,%s' % (int(r['id']), nx, int(r['duration']), int(r['length']),
                                              int(r['queue_length']), int(r['start']), int(r['end']), source,
                                              mode.upper())


def stream_tiles(rows, privacy, q=3600, source='reporter', mode='auto'):
    """{file name: lines} of the streaming path for rows in arrival order."""
    by_file = {}
    for r in rows:
        by_file.setdefault(file_name(r['file'], q), []).append(r)
    out = {}
    for k, v in by_file.items():
        v = sorted(v, key=lambda r: (int(r['id']), int(r['next_id'])))  # stable, as Collections.sort
        kept = java_clean(v, privacy)
        if kept:
            out[k] = [java_line(r, source, mode) for r in kept]
    return out
