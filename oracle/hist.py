"""CPU restatement of the device histogram stages — TEST INFRASTRUCTURE ONLY.

histogram(): the dense K8 stage — simple_reporter.py:176-187 filter + hour buckets,
accumulated into the [hour][segment][speed bin] count histogram of OTR batches.

Keyed speed histogram: the per-GPU histogram is simple_reporter's tile
rows (oracle/tiles.rows_from_reports, simple_reporter.py:176-196) counted by (hour-tile
file, segment id, next id, speed bin): one entry per key with its number of
observations.  The keyed exchange sends each entry to the rank owning its file
(reporter_amd.simple_reporter.file_owner, the (hour, tile) partition of §8e); the owner
sums the counts of equal keys it received and applies the privacy threshold to whole
segment pairs exactly as the reference loop does on the file's lines
(simple_reporter.py:218-239): a pair's run length is its total count over all speed bins
(one line per tile row); the lines are sorted as strings, so the runs come in the string
order of (id, next_id); every run is judged alone (kept iff >= privacy) except that a
trailing run of one line is judged together with the run before it (both kept iff that
run's length + 1 >= privacy).  Checker for otr_hist_reduce (include/otr.h)
and simple_reporter.exchange_hist; oracle/tiles.sort_and_cull is the same rule on lines.
"""
import math

import numpy as np

BINS = 8


def _py2_round_int(x):
    f = math.floor(x)
    return int(f + 1 if x - f >= 0.5 else f)


def histogram(res, first_time, last_time, seg_index_of_id, n_segments, base_time, hours, q=3600):
    """res: oracle/HIP result dict; first/last_time: per trace; seg_index_of_id: dict."""
    h = np.zeros((hours, n_segments, BINS), np.int64)
    rows = 0
    off = res['trace_rep_off']
    for t in range(len(off) - 1):
        buckets = (int(last_time[t]) - int(first_time[t])) // q + 1
        for k in range(off[t], off[t + 1]):
            t0, t1 = float(res['rep_t0'][k]), float(res['rep_t1'][k])
            ln, qu = int(res['rep_length'][k]), int(res['rep_queue'][k])
            if not (t0 > 0 and t1 > 0 and t1 - t0 > .5 and ln > 0 and qu >= 0):
                continue
            start, end = int(math.floor(t0)), int(math.ceil(t1))
            mn, mx = start // q, end // q
            if mx - mn > buckets:
                continue
            kmh = (ln / (t1 - t0)) * 3.6
            b = min(max(int(kmh / 20.0), 0), BINS - 1)
            seg = seg_index_of_id[int(res['rep_id'][k])]
            for bk in range(mn, mx + 1):
                rows += 1
                hh = (bk * q - base_time) // q
                if 0 <= hh < hours:
                    h[hh, seg, b] += 1
    return h, rows


HIST_ENTRY = np.dtype([('file', '<u8'), ('id', '<u8'), ('next_id', '<u8'), ('speed_bin', '<u4'), ('count', '<u4')])


def entries_from_rows(rows):
    """Tile rows -> unreduced entries, count 1 each (rows keep their order)."""
    e = np.zeros(len(rows), HIST_ENTRY)
    for k in ('file', 'id', 'next_id'):
        e[k] = rows[k]
    e['speed_bin'] = rows['speed_bin'].astype(np.uint32)
    e['count'] = 1
    return e


def reduce(entries, privacy=1):
    """Sum the counts of equal (file, id, next_id, speed_bin) keys, in key order; with
    privacy > 1 drop the pairs whose total count is below privacy.  Counts saturate at
    2^32 - 1 as the device's u32 field does."""
    if len(entries) == 0:
        return np.zeros(0, HIST_ENTRY)
    acc = {}
    for f, i, n, b, c in zip(entries['file'].tolist(), entries['id'].tolist(), entries['next_id'].tolist(),
                             entries['speed_bin'].tolist(), entries['count'].tolist()):
        acc[(f, i, n, b)] = acc.get((f, i, n, b), 0) + c
    keys = sorted(acc)
    pair_tot = {}
    for k in keys:
        pair_tot[k[:3]] = pair_tot.get(k[:3], 0) + acc[k]
    keep = {p: t >= privacy for p, t in pair_tot.items()}
    if privacy > 1:  # the reference loop's trailing run (simple_reporter.py:221-239)
        files = {}
        for f, i, nx in pair_tot:
            files.setdefault(f, []).append((str(i) + ',', str(nx) + ',', i, nx))
        for f, prs in files.items():
            prs.sort()  # the string order of the lines' (id, next_id) prefix
            if len(prs) >= 2 and pair_tot[(f, prs[-1][2], prs[-1][3])] == 1:
                prev = (f, prs[-2][2], prs[-2][3])
                k2 = pair_tot[prev] + 1 >= privacy
                keep[prev] = k2
                keep[(f, prs[-1][2], prs[-1][3])] = k2
    out = [(k[0], k[1], k[2], k[3], min(acc[k], 0xFFFFFFFF)) for k in keys
           if privacy <= 1 or keep[k[:3]]]
    return np.array(out, dtype=HIST_ENTRY) if out else np.zeros(0, HIST_ENTRY)


def owner_of(files, world):
    """The (hour, tile) owner rank: the same fixed mix as simple_reporter.file_owner."""
    files = np.asarray(files, dtype=np.uint64).astype(np.int64)
    return ((files >> 25) * 40503 + (files & 0x1FFFFFF)) % world


def keyed_exchange(per_rank_entries, world, privacy):
    """The whole exchange on one host: every rank's entries reduced locally, routed to
    their owners, and reduced + culled there.  Returns the owners' results by rank."""
    inbox = [[] for _ in range(world)]
    for e in per_rank_entries:
        r = reduce(e, 1)
        own = owner_of(r['file'], world) if len(r) else np.zeros(0, np.int64)
        for q in range(world):
            inbox[q].append(r[own == q])
    return [reduce(np.concatenate(b) if b else np.zeros(0, HIST_ENTRY), privacy) for b in inbox]
