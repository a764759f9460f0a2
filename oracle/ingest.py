"""CPU restatement of the reference's probe ingest — TEST INFRASTRUCTURE ONLY.

shard_traces: simple_reporter.match() reading a shard file (simple_reporter.py:136-160):
    line.strip().split(',') into uuid, time, lat, lon, acc; float()/int(); traces grouped
    per uuid (dict in first-appearance order: the reference's py2 dict order is arbitrary,
    so tests compare in this order); sort by time (stable); windows split at gaps
    > inactivity; windows of fewer than 2 points skipped.
raw_to_shard_text: simple_reporter.download() (:99-111) for the default valuer
    (:352, fields c[1], c[0], c[9], c[10], c[5] of l.split("|")) or any field indices:
    bbox skip, fast "%Y-%m-%d %H:%M:%S" time (:106-107) + calendar.timegm,
    min(int(math.ceil(float(acc))), 1000), serialised with Python 2 str() (12 significant
    digits for floats).  One text in input order stands for the sha1-keyed shard files
    (grouping per uuid is the same either way).
java_sv_points: Formatter.formatSV (Formatter.java:103-114): String.split (trailing empty
    fields dropped), float32 coordinates, Long.parseLong or yyyy-MM-dd HH:mm:ss, (int)ceil.
Python 3 runs these; the Python 2 semantics that differ are restated explicitly
(no '_' digit separators in float()/int(), str(float) = 12 significant digits).  Text
is decoded as latin-1; tests keep to ASCII whitespace, where Python 2 byte strings and
Python 3 str agree.
"""
import calendar
import math
import time as _time

import numpy as np


class IngestError(ValueError):
    def __init__(self, line, reason):
        super().__init__('line %d: %s' % (line, reason))
        self.line = line
        self.reason = reason


def _py2_float(s, overflow_ok=False):
    """float() without '_' separators and without inf/nan literals (refused: a divergence
    the device path keeps); decimal overflow to inf passes only where the caller filters
    it (download()'s bbox)."""
    if '_' in s:
        raise ValueError(s)
    v = float(s)
    if math.isnan(v) or (math.isinf(v) and (not overflow_ok or 'n' in s.lower())):
        raise ValueError(s)
    return v


def _py2_int(s):
    if '_' in s:
        raise ValueError(s)
    return int(s)


def py2_str_float(x):
    """Python 2.7 str(float): 12 significant digits ('%.12g'), '.0' added to integers."""
    s = '%.12g' % x
    return s + '.0' if s.lstrip('-').isdigit() else s


def _lines(text):
    """Python file iteration over bytes: split after every '\\n'; a final fragment counts."""
    parts = text.split(b'\n')
    if parts and parts[-1] == b'':
        parts.pop()
    return [p.decode('latin-1') for p in parts]


def _windows(points, inactivity):
    starts = [i for i, p in enumerate(points) if i == 0 or p[2] - points[i - 1][2] > inactivity]
    out = []
    for k, i in enumerate(starts):
        j = starts[k + 1] if k + 1 < len(starts) else len(points)
        if j - i >= 2:
            out.append(points[i:j])
    return out


def group_windows(recs, inactivity):
    """recs: [(uuid, (lat, lon, time, acc))] in line order → [(uuid, [points])] windows."""
    traces = {}
    for uuid, p in recs:
        traces.setdefault(uuid, []).append(p)
    out = []
    for uuid, pts in traces.items():
        pts.sort(key=lambda v: v[2])  # :146 stable
        for w in _windows(pts, inactivity):
            out.append((uuid, w))
    return out


def shard_records(text):
    recs = []
    for n, line in enumerate(_lines(text)):
        parts = line.strip().split(',')
        if len(parts) != 5:
            raise IngestError(n, 'fields')
        uuid, tm, lat, lon, acc = parts
        try:
            la, lo = _py2_float(lat), _py2_float(lon)
        except ValueError:
            raise IngestError(n, 'float')
        try:
            t, a = _py2_int(tm), _py2_int(acc)
        except ValueError:
            raise IngestError(n, 'int')
        if abs(a) > 1 << 24:
            raise IngestError(n, 'accuracy')
        recs.append((uuid, (la, lo, t, a)))
    return recs


def shard_traces(text, inactivity=120):
    return group_windows(shard_records(text), inactivity)


def _fast_time(tm):
    """:106-107 — int() of fixed slices, then calendar.timegm (datetime.date checks y, m)."""
    try:
        st = (_py2_int(tm[0:4]), _py2_int(tm[5:7]), _py2_int(tm[8:10]), _py2_int(tm[11:13]),
              _py2_int(tm[14:16]), _py2_int(tm[17:19]))
    except ValueError:
        return None, 'int'
    try:
        return calendar.timegm(_time.struct_time(st + (0, 0, 0))), None
    except (ValueError, OverflowError):
        return None, 'time'


def raw_to_shard_text(text, idx=(1, 0, 9, 10, 5), sep='|', bbox=None, time_format='ymdhms'):
    """download() → the shard lines match() reads (one text, input order)."""
    out = []
    for n, message in enumerate(_lines(text)):
        c = message.split(sep)
        try:
            uuid, tm, lat, lon, acc = [c[i] for i in idx]
        except IndexError:
            raise IngestError(n, 'fields')
        try:
            lat, lon = _py2_float(lat, True), _py2_float(lon, True)
        except ValueError:
            raise IngestError(n, 'float')
        if bbox is not None and (lat < bbox[0] or lat > bbox[2] or lon < bbox[1] or lon > bbox[3]):
            continue
        if not (math.isfinite(lat) and math.isfinite(lon)):
            raise IngestError(n, 'float')
        if time_format == 'ymdhms':
            tm, why = _fast_time(tm)
            if why:
                raise IngestError(n, why)
        else:
            try:
                tm = _py2_int(tm)
            except ValueError:
                raise IngestError(n, 'int')
        try:
            acc = min(int(math.ceil(_py2_float(acc))), 1000)
        except (ValueError, OverflowError):
            raise IngestError(n, 'accuracy')
        if acc < -(1 << 24):
            raise IngestError(n, 'accuracy')
        if ',' in uuid.lstrip():
            raise IngestError(n, 'uuid')  # match() would see more than 5 fields
        out.append(','.join([uuid, str(tm), py2_str_float(lat), py2_str_float(lon), str(acc)]) + '\n')
    return ''.join(out).encode('latin-1')


def raw_traces(text, inactivity=120, **kw):
    return shard_traces(raw_to_shard_text(text, **kw), inactivity)


def _java_split(s, sep):
    parts = s.split(sep)
    while parts and parts[-1] == '':
        parts.pop()
    return parts


def _java_time(s, time_format):
    if time_format == 'ymdhms':
        return _fast_time(s)
    body = s[1:] if s[:1] in ('+', '-') else s  # Long.parseLong: sign, digits, nothing else
    if not body or any(ch not in '0123456789' for ch in body):
        return None, 'int'
    v = int(s)
    if not -2 ** 63 <= v < 2 ** 63:
        return None, 'int'
    return v, None


def java_sv_records(text, idx=(1, 0, 9, 10, 5), sep='|', time_format='ymdhms'):
    recs = []
    for n, message in enumerate(_lines(text)):
        c = _java_split(message, sep)
        try:
            uuid, tm, lat, lon, acc = [c[i] for i in idx]
        except IndexError:
            raise IngestError(n, 'fields')
        try:
            la = float(np.float32(_py2_float(lat)))
            lo = float(np.float32(_py2_float(lon)))
        except ValueError:
            raise IngestError(n, 'float')
        t, why = _java_time(tm, time_format)
        if why:
            raise IngestError(n, why)
        try:
            af = float(np.float32(_py2_float(acc)))
        except ValueError:
            raise IngestError(n, 'accuracy')
        a = math.ceil(af)
        a = max(min(a, 2 ** 31 - 1), -2 ** 31)
        if abs(a) > 1 << 24:
            raise IngestError(n, 'accuracy')
        recs.append((uuid, (la, lo, t, a)))
    return recs


def java_sv_traces(text, inactivity=120, **kw):
    return group_windows(java_sv_records(text, **kw), inactivity)


def to_soa(windows):
    """[(uuid, points)] → (uuids, offsets, lat, lon, time, acc) numpy arrays."""
    offs = [0]
    lat, lon, tm, acc = [], [], [], []
    for _, pts in windows:
        for p in pts:
            lat.append(p[0])
            lon.append(p[1])
            tm.append(p[2])
            acc.append(p[3])
        offs.append(len(lat))
    return ([u for u, _ in windows], np.asarray(offs, np.int64), np.asarray(lat, np.float64),
            np.asarray(lon, np.float64), np.asarray(tm, np.int64), np.asarray(acc, np.float32))
