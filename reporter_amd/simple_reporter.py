"""Batch driver mirroring py/simple_reporter.py's match → bucket → cull stages over the
batched HIP API.  S3 download/upload (simple_reporter.py:51-129, 247-254) is out of
scope (network); inputs and outputs are local files.

The product path (every stage on the device):
  report(m, traces, privacy, ...)  windows → one batch → K9 tile rows → K10 sort + cull in HBM
                                   → CSV lines per tile (= report_tiles_device)
  text_tiles_device(m, text, p)    shard / raw probe text → tiles, every stage in HBM
                                   (K11 ingest :99-111,136-160 → K1-K10)
  stream_tiles_device(m, tr, p)    the Java streaming output stage (AnonymisingProcessor)
  shard_key(uuid)                  sha1(uuid)[0:3]                (:116)
  windows(times, inactivity)       inactivity windows             (:150-160)

The host mirror of the reference's loops (small inputs, and the goldens that pin K9/K10:
tests/test_golden_tiles.py, tests/test_gpu_tiles.py compares the two paths):
  bucket(first, last, reports, q, mode, source)
                                   filter + hour buckets → rows   (:176-196)
  cull(lines, privacy)             privacy cull incl. the trailing-singleton merge (:218-239)
  match_traces(traces, ...)        windows → otr_match_batch → rows per tile (host bucketing)
  report_tiles(tiles, privacy)     sort + cull                    (:211-245)
"""
import hashlib
import math
import os

import numpy as np

LEVEL_BITS = 3
TILE_INDEX_BITS = 22
SEGMENT_INDEX_BITS = 21
LEVEL_MASK = (1 << LEVEL_BITS) - 1
TILE_INDEX_MASK = (1 << TILE_INDEX_BITS) - 1
SEGMENT_INDEX_MASK = (1 << SEGMENT_INDEX_BITS) - 1
INVALID_SEGMENT_ID = (SEGMENT_INDEX_MASK << (TILE_INDEX_BITS + LEVEL_BITS)) | \
    (TILE_INDEX_MASK << LEVEL_BITS) | LEVEL_MASK
COLUMNS = 'segment_id,next_segment_id,duration,count,length,queue_length,minimum_timestamp,maximum_timestamp,' \
          'source,vehicle_type'


def get_tile_level(segment_id):
    return segment_id & LEVEL_MASK


def get_tile_index(segment_id):
    return (segment_id >> LEVEL_BITS) & TILE_INDEX_MASK


def shard_key(uuid):
    return hashlib.sha1(uuid.encode() if isinstance(uuid, str) else uuid).hexdigest()[0:3]


def shard_of(uuid, n):
    """GPU (or worker) owning a vehicle: the simple_reporter hash prefix modulo n."""
    return int(shard_key(uuid), 16) % n


def windows(times, inactivity):
    """[i, j) index ranges split at gaps > inactivity, dropping ranges shorter than 2."""
    starts = [i for i in range(len(times)) if i == 0 or times[i] - times[i - 1] > inactivity]
    out = []
    for k, i in enumerate(starts):
        j = starts[k + 1] if k + 1 < len(starts) else len(times)
        if j - i >= 2:
            out.append((i, j))
    return out


def py2_round_int(x):
    """int(round(x)) with Python 2 half-away-from-zero on the exact binary value."""
    f = math.floor(x)
    return int(f + 1 if x - f >= 0.5 else f) if x >= 0 else -py2_round_int(-x)


def _str_num(v):
    if isinstance(v, float):  # Python 2 str(float): 12 significant digits
        s = '%.12g' % v
        if '.' not in s and 'e' not in s and 'n' not in s:
            s += '.0'
        return s
    return str(v)


def bucket(first_time, last_time, reports, quantisation, mode, source):
    """{tile_key: [row lines]} for one window's report() output (simple_reporter.py:176-196).
    tile_key = '{b*q}_{(b+1)*q-1}/{level}/{tile_index}'."""
    tiles = {}
    buckets = (last_time - first_time) // quantisation + 1
    for r in reports:
        if not (r['t0'] > 0 and r['t1'] > 0 and r['t1'] - r['t0'] > .5 and r['length'] > 0 and r['queue_length'] >= 0):
            continue
        duration = py2_round_int(r['t1'] - r['t0'])
        start = int(math.floor(r['t0']))
        end = int(math.ceil(r['t1']))
        min_b = start // quantisation
        max_b = end // quantisation
        if max_b - min_b > buckets:
            continue
        for b in range(min_b, max_b + 1):
            key = '%d_%d/%d/%d' % (b * quantisation, (b + 1) * quantisation - 1, get_tile_level(r['id']),
                                   get_tile_index(r['id']))
            row = [str(r['id']), str(r.get('next_id', INVALID_SEGMENT_ID)), str(duration), '1',
                   _str_num(r['length']), _str_num(r['queue_length']), str(start), str(end), source, mode.upper()]
            tiles.setdefault(key, []).append(','.join(row) + os.linesep)
    return tiles


def cull(lines, privacy):
    """Delete (id,next_id) runs seen fewer than `privacy` times, on lexicographically
    sorted lines.  Reproduces the reference loop exactly, including its quirk: a
    trailing run of length 1 is judged together with the run before it."""
    segs = list(lines)
    start = 0
    i = 0
    while i < len(segs):
        s = segs[start].split(',')
        e = segs[i].split(',')
        if s[0] != e[0] or s[1] != e[1] or i == len(segs) - 1:
            if i == len(segs) - 1:
                i += 1
            if i - start < privacy:
                del segs[start:i]
                i = start
            else:
                start = i
        i += 1
    return segs


def report_tiles(tiles, privacy):
    """Sort (string order, :218) and cull each tile; drop empty tiles (:242-244)."""
    out = {}
    for key, lines in tiles.items():
        kept = cull(sorted(lines), privacy)
        if kept:
            out[key] = kept
    return out


def match_traces(matcher, traces, mode='auto', report_levels=(0, 1), transition_levels=(0, 1),
                 quantisation=3600, inactivity=120, source='smpl_rprt', threshold_sec=15):
    """simple_reporter.match() over a batch: split each trace at inactivity gaps, match
    all windows in ONE otr_match_batch call, bucket every window's reports."""
    from .tools.gen import Traces
    idx_lat, idx_lon, idx_time, offs, modes = [], [], [], [0], []
    win_src = []
    for t in range(traces.n_traces):
        a, b = int(traces.offsets[t]), int(traces.offsets[t + 1])
        order = np.argsort(traces.time[a:b], kind='stable') + a  # :146 sort by time
        tm = traces.time[order]
        for i, j in windows(tm.tolist(), inactivity):
            sel = order[i:j]
            idx_lat.append(traces.lat[sel])
            idx_lon.append(traces.lon[sel])
            idx_time.append(traces.time[sel])
            offs.append(offs[-1] + len(sel))
            modes.append(traces.mode[t])
            win_src.append(t)
    if not win_src:
        return {}
    batch = Traces(np.concatenate(idx_lat), np.concatenate(idx_lon), np.concatenate(idx_time),
                   np.asarray(offs, np.int64), np.asarray(modes, np.uint8))
    r = matcher.match_batch_numpy(batch, report_levels=report_levels, transition_levels=transition_levels,
                                  threshold_sec=threshold_sec, quantisation=quantisation)
    tiles = {}
    for w in range(batch.n_traces):
        lo, hi = r['trace_rep_off'][w], r['trace_rep_off'][w + 1]
        reps = []
        for k in range(lo, hi):
            d = {'id': int(r['rep_id'][k]), 't0': float(r['rep_t0'][k]), 't1': float(r['rep_t1'][k]),
                 'length': int(r['rep_length'][k]), 'queue_length': int(r['rep_queue'][k])}
            if int(r['rep_next'][k]) != 0xFFFFFFFFFFFFFFFF:
                d['next_id'] = int(r['rep_next'][k])
            reps.append(d)
        first, last = int(batch.time[batch.offsets[w]]), int(batch.time[batch.offsets[w + 1] - 1])
        for key, rows in bucket(first, last, reps, quantisation, mode, source).items():
            tiles.setdefault(key, []).extend(rows)
    return tiles


def write_tiles(tiles, dest_dir):
    """Tile files with the reference's CSV header (simple_reporter.py:252)."""
    for key, lines in tiles.items():
        path = os.path.join(dest_dir, key)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, 'w') as f:
            f.write(COLUMNS + os.linesep)
            f.write(''.join(lines))


# ---------------------------------------------------------------------------------
# Device tile stage: rows (K9) → sort + cull (K10) → CSV lines, and the multi-GPU
# exchange that routes every row to the GPU owning its (hour, tile) file.
# ---------------------------------------------------------------------------------
def file_key(file, quantisation=3600):
    """'{b*q}_{(b+1)*q-1}/{level}/{tile_index}' of an otr_tile_row.file (simple_reporter.py:189)."""
    b, level, tile = int(file) >> 25, (int(file) >> 22) & LEVEL_MASK, int(file) & TILE_INDEX_MASK
    return '%d_%d/%d/%d' % (b * quantisation, (b + 1) * quantisation - 1, level, tile)


def file_owner(files, world):
    """Rank owning each (hour, tile) file: a fixed mix of bucket and tile, modulo world
    (numpy or torch int64 arrays)."""
    return ((files >> 25) * 40503 + (files & 0x1FFFFFF)) % world


def cull_rows(matcher, rows, privacy, device_ptr=None, n=None, rules=0):
    """otr_tiles_cull: host numpy TILE_ROW rows, or (device_ptr, n) rows in HBM →
    kept rows (numpy, sorted per file in simple_reporter's line order, or with
    rules=OTR_TILE_RULES_STREAM in Segment.compareTo order)."""
    import ctypes
    from . import _lib
    L = _lib.lib()
    out, nout = ctypes.c_void_p(), ctypes.c_int64()
    if device_ptr is not None:
        rc = L.otr_tiles_cull(matcher._h, device_ptr, int(n), _lib.OTR_MEM_DEVICE, int(privacy), int(rules),
                              ctypes.byref(out), ctypes.byref(nout))
    else:
        rows = np.ascontiguousarray(rows, dtype=_lib.TILE_ROW)
        rc = L.otr_tiles_cull(matcher._h, rows.ctypes.data if len(rows) else None, len(rows), _lib.OTR_MEM_HOST,
                              int(privacy), int(rules), ctypes.byref(out), ctypes.byref(nout))
    if rc != 0:
        raise RuntimeError('otr_tiles_cull failed (%d): %s' % (rc, _lib.last_error()))
    k = nout.value
    if k == 0:
        return np.zeros(0, _lib.TILE_ROW)
    buf = (ctypes.c_char * (k * _lib.TILE_ROW.itemsize)).from_address(out.value)
    return np.frombuffer(bytes(buf), dtype=_lib.TILE_ROW)


def rows_to_tiles(rows, quantisation=3600, mode='auto', source='smpl_rprt', rules=0):
    """{tile_key: [lines]} from rows grouped by file (otr_tiles_format writes the lines;
    with rules=OTR_TILE_RULES_STREAM each line is '\n' + fields as Segment.java:59-74)."""
    import ctypes
    from . import _lib
    rows = np.ascontiguousarray(rows, dtype=_lib.TILE_ROW)
    if len(rows) == 0:
        return {}
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = _lib.lib().otr_tiles_format(rows.ctypes.data, len(rows), source.encode(), mode.encode(), int(rules),
                                     ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError('otr_tiles_format failed: %s' % _lib.last_error())
    text = _lib.take_string(out, n)
    if rules == _lib.OTR_TILE_RULES_STREAM:
        lines = ['\n' + l for l in text.split('\n')[1:]]
    else:
        lines = text.splitlines(True)
    tiles = {}
    cuts = np.flatnonzero(np.diff(rows['file'].astype(np.int64))) + 1
    for a, b in zip(np.concatenate([[0], cuts]), np.concatenate([cuts, [len(rows)]])):
        tiles[file_key(rows['file'][a], quantisation)] = lines[a:b]
    return tiles


def _window_batch(traces, inactivity):
    from .tools.gen import Traces
    idx_lat, idx_lon, idx_time, offs, modes = [], [], [], [0], []
    for t in range(traces.n_traces):
        a, b = int(traces.offsets[t]), int(traces.offsets[t + 1])
        order = np.argsort(traces.time[a:b], kind='stable') + a  # :146 sort by time
        tm = traces.time[order]
        for i, j in windows(tm.tolist(), inactivity):
            sel = order[i:j]
            idx_lat.append(traces.lat[sel])
            idx_lon.append(traces.lon[sel])
            idx_time.append(traces.time[sel])
            offs.append(offs[-1] + len(sel))
            modes.append(traces.mode[t])
    if len(offs) == 1:
        return None
    return Traces(np.concatenate(idx_lat), np.concatenate(idx_lon), np.concatenate(idx_time),
                  np.asarray(offs, np.int64), np.asarray(modes, np.uint8))


def report_tiles_device(matcher, traces, privacy, mode='auto', report_levels=(0, 1), transition_levels=(0, 1),
                        quantisation=3600, inactivity=120, source='smpl_rprt', threshold_sec=15):
    """simple_reporter match() + report() with the tile stage on device: windows → one
    batch emitting tile rows in HBM (K9) → sort + cull in HBM (K10) → CSV lines.
    Equals report_tiles(match_traces(...), privacy)."""
    from . import _lib
    batch = _window_batch(traces, inactivity)
    if batch is None:
        return {}
    r = matcher.match_batch(batch, report_levels=report_levels, transition_levels=transition_levels,
                            threshold_sec=threshold_sec, quantisation=quantisation, copy_out=False, tile_rows=True)
    kept = cull_rows(matcher, None, privacy, device_ptr=r.d_rows, n=r.n_rows)
    return rows_to_tiles(kept, quantisation, mode, source)


def report(matcher, traces, privacy, **kw):
    """simple_reporter's match() + report() + cull for a batch of traces, the product path:
    every stage on the device (report_tiles_device).  The host functions bucket / cull /
    match_traces / report_tiles give the same tiles (tests/test_gpu_tiles.py)."""
    return report_tiles_device(matcher, traces, privacy, **kw)


def text_tiles_device(matcher, text, privacy, rules=0, mode='auto', report_levels=(0, 1), transition_levels=(0, 1),
                      quantisation=3600, inactivity=120, source='smpl_rprt', threshold_sec=15, **fmt):
    """simple_reporter from probe text to tiles with every stage in HBM: the shard lines
    match() reads (rules OTR_INGEST_SHARD, :136-160) or the raw feed download() reads
    (OTR_INGEST_RAW, :99-111; fmt: separator, field indices, bbox) → K11 ingest → K1-K8
    → K9 tile rows → K10 sort + cull → CSV lines."""
    r, batch = matcher.ingest(text, rules=rules, inactivity=inactivity, mode=mode, **fmt)
    if r.n_traces == 0:
        return {}
    res = matcher.match_batch(batch, report_levels=report_levels, transition_levels=transition_levels,
                              threshold_sec=threshold_sec, quantisation=quantisation, copy_out=False,
                              tile_rows=True, device_arrays=batch.arrays)
    kept = cull_rows(matcher, None, privacy, device_ptr=res.d_rows, n=res.n_rows)
    return rows_to_tiles(kept, quantisation, mode, source)


def stream_tiles_device(matcher, traces, privacy, mode='auto', report_levels=(0, 1), transition_levels=(0, 1),
                        quantisation=3600, source='reporter', threshold_sec=15):
    """The Java streaming path's output stage on device: report() reports → Segment
    (BatchingProcessor.java:108-141) → TimeQuantisedTile buckets → Collections.sort +
    clean (AnonymisingProcessor.java:155-175, 223-266) → Segment lines.  Returns
    {"{start}_{start+q-1}/{level}/{tile}": [lines]} (AnonymisingProcessor.store names the
    file under that directory source.UUID, :185-188)."""
    from . import _lib
    r = matcher.match_batch(traces, report_levels=report_levels, transition_levels=transition_levels,
                            threshold_sec=threshold_sec, quantisation=quantisation, copy_out=False, tile_rows=True,
                            tile_rules=_lib.OTR_TILE_RULES_STREAM)
    kept = cull_rows(matcher, None, privacy, device_ptr=r.d_rows, n=r.n_rows, rules=_lib.OTR_TILE_RULES_STREAM)
    return rows_to_tiles(kept, quantisation, mode, source, rules=_lib.OTR_TILE_RULES_STREAM)


def _exchange_by_file_owner(buf, itemsize, world, group=None):
    """All-to-all of fixed-size records whose first 8 bytes are their (hour, tile) file:
    each record goes to file_owner(file); returns the records this rank received (uint8
    tensor, grouped by sender rank)."""
    import torch
    import torch.distributed as dist
    r8 = buf.view(-1, itemsize)
    files = r8[:, 0:8].contiguous().view(torch.int64).reshape(-1)
    owner = file_owner(files, world)
    order = torch.argsort(owner, stable=True)
    send = r8[order].contiguous().reshape(-1)
    counts = torch.bincount(owner, minlength=world).to(torch.int64)
    recv = torch.empty_like(counts)
    dist.all_to_all_single(recv, counts, group=group)
    out = torch.empty(int(recv.sum().item()) * itemsize, dtype=torch.uint8, device=buf.device)
    dist.all_to_all_single(out, send, output_split_sizes=[int(x) * itemsize for x in recv.tolist()],
                           input_split_sizes=[int(x) * itemsize for x in counts.tolist()], group=group)
    return out


def exchange_rows(rows, world, group=None):
    """Route every row to the rank owning its file (all-to-all, one exchange step):
    rows is a uint8 tensor of n*56 bytes (device for RCCL, host for gloo); returns the
    rows this rank owns (uint8 tensor).  Owners then cull complete files locally."""
    from . import _lib
    return _exchange_by_file_owner(rows, _lib.TILE_ROW.itemsize, world, group)


def hist_reduce(matcher, src, n, privacy=1, rows_in=False, memory='device', out=None, out_memory=None):
    """otr_hist_reduce: n tile rows (rows_in) or histogram entries → entries summed per
    (file, id, next_id, speed_bin) in key order, pairs below `privacy` dropped.  src: a
    device pointer (memory='device') or a numpy array (memory='host').  out: a device
    pointer with room for n entries (returns their number), or None for a numpy array."""
    import ctypes
    from . import _lib
    L = _lib.lib()
    n = int(n)
    mem = _lib.OTR_MEM_DEVICE if memory == 'device' else _lib.OTR_MEM_HOST
    if memory != 'device':
        src = np.ascontiguousarray(src, dtype=_lib.TILE_ROW if rows_in else _lib.HIST_ENTRY)
        ptr = src.ctypes.data if n else None
    else:
        ptr = int(src) if n else None
    nout = ctypes.c_int64()
    if out is not None:
        rc = L.otr_hist_reduce(matcher._h, ptr, n, mem, int(bool(rows_in)), int(privacy), int(out), max(n, 1),
                               _lib.OTR_MEM_DEVICE if out_memory in (None, 'device') else _lib.OTR_MEM_HOST,
                               ctypes.byref(nout))
        if rc != 0:
            raise RuntimeError('otr_hist_reduce failed (%d): %s' % (rc, _lib.last_error()))
        return nout.value
    res = np.zeros(max(n, 1), _lib.HIST_ENTRY)
    rc = L.otr_hist_reduce(matcher._h, ptr, n, mem, int(bool(rows_in)), int(privacy), res.ctypes.data, max(n, 1),
                           _lib.OTR_MEM_HOST, ctypes.byref(nout))
    if rc != 0:
        raise RuntimeError('otr_hist_reduce failed (%d): %s' % (rc, _lib.last_error()))
    return res[:nout.value].copy()


def exchange_hist(entries, world, group=None):
    """The keyed histogram exchange: every 32-B histogram entry goes to
    the rank owning its (hour, tile) file (one all-to-all); returns the entries this rank
    received (uint8 tensor; device for RCCL, host for gloo).  The owner then reduces and
    culls them with hist_reduce(..., privacy)."""
    from . import _lib
    return _exchange_by_file_owner(entries, _lib.HIST_ENTRY.itemsize, world, group)
