"""ctypes wrappers for libotrgen.so: seeded synthetic graphs and traces.

Workload infrastructure for bench.py and the tests; the product never imports it.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

# named workloads: (graph args, trace args)  — SURVEY.md §8d / BASELINE.md table
GRAPHS = {
    # rows, cols, spacing_m, center_lat, center_lon, p_remove, seed, cell_deg
    'tiny': (24, 24, 60.0, 14.55, 121.03, 0.10, 11, 0.0005),
    'city': (200, 200, 50.0, 14.55, 121.03, 0.15, 1, 0.0005),
    'metro': (1024, 1024, 50.0, 14.55, 121.03, 0.15, 2, 0.0005),
    # C5: a country-scale grid, 7072 x 7072 = 50M nodes over ~700 x 700 km,
    # ~135M directed edges (minutes to generate; 12 GB file)
    'country': (7072, 7072, 100.0, 14.55, 121.03, 0.40, 5, 0.0005),
}
CONFIGS = {
    # graph, n_traces, points/trace, sample_rate s, sigma m, seed, frac_bicycle, frac_ped, search_radius
    'C1': ('city', 1000, 300, 1, 5.0, 1, 0.0, 0.0, 50.0),
    'C2': ('metro', 10000, 100, 15, 10.0, 2, 0.0, 0.0, 50.0),
    'C4': ('metro', 20000, 60, 60, 50.0, 4, 0.0, 0.0, 200.0),
}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, 'libotrgen.so')
        if not os.path.exists(path):
            raise RuntimeError('libotrgen.so not built: run python __graft_entry__.py build')
        L = ctypes.CDLL(path)
        L.otrgen_graph.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_uint64,
                                   ctypes.c_double]
        L.otrgen_graph.restype = ctypes.c_int
        P = ctypes.POINTER
        L.otrgen_traces.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_uint64, ctypes.c_double, ctypes.c_double, P(ctypes.c_double),
                                    P(ctypes.c_double), P(ctypes.c_int64), P(ctypes.c_uint8),
                                    P(ctypes.c_uint32), ctypes.c_int64, ctypes.c_int64]
        L.otrgen_traces.restype = ctypes.c_int
        L.otrgen_traces_ids.argtypes = [ctypes.c_char_p, ctypes.c_int, P(ctypes.c_int64), ctypes.c_int, ctypes.c_int,
                                        ctypes.c_double, ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                        P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int64),
                                        P(ctypes.c_uint8), P(ctypes.c_uint32), ctypes.c_int64, ctypes.c_int64]
        L.otrgen_traces_ids.restype = ctypes.c_int
        _LIB = L
    return _LIB


def graph_path(name, cache_dir=None):
    """Return the path of graph `name`, generating it once into cache_dir."""
    cache_dir = cache_dir or os.environ.get('OTR_CACHE', os.path.join(_HERE, '..', '..', 'build', 'graphs'))
    os.makedirs(cache_dir, exist_ok=True)
    path = os.path.abspath(os.path.join(cache_dir, name + '.otrg'))
    if not os.path.exists(path):
        args = GRAPHS[name]
        tmp = path + '.tmp%d' % os.getpid()
        rc = lib().otrgen_graph(tmp.encode(), *args)
        if rc != 0:
            raise RuntimeError('otrgen_graph failed: %d' % rc)
        os.replace(tmp, path)
    return path


class Traces:
    """SoA batch of traces: offsets, lat, lon, time, accuracy, mode, uuids."""

    def __init__(self, lat, lon, time, offsets, mode, accuracy=None, truth=None, uuids=None):
        self.lat, self.lon, self.time, self.offsets, self.mode = lat, lon, time, offsets, mode
        self.accuracy = accuracy
        self.truth = truth
        self.uuids = uuids

    @property
    def n_traces(self):
        return len(self.offsets) - 1

    @property
    def n_probes(self):
        return int(self.offsets[-1])

    def slice(self, a, b):
        """The contiguous traces a..b-1 (views where possible)."""
        q0, q1 = int(self.offsets[a]), int(self.offsets[b])
        off = self.offsets[a:b + 1] - q0
        acc = None if self.accuracy is None else self.accuracy[q0:q1]
        tr = None if self.truth is None else self.truth[q0:q1]
        uu = None if self.uuids is None else self.uuids[a:b]
        return Traces(self.lat[q0:q1], self.lon[q0:q1], self.time[q0:q1], off, self.mode[a:b], acc, tr, uu)

    def subset(self, idx):
        idx = np.asarray(idx, dtype=np.int64)
        parts = [np.arange(self.offsets[i], self.offsets[i + 1]) for i in idx]
        sel = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        lens = np.array([self.offsets[i + 1] - self.offsets[i] for i in idx], dtype=np.int64)
        off = np.zeros(len(idx) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        acc = None if self.accuracy is None else self.accuracy[sel]
        tr = None if self.truth is None else self.truth[sel]
        uu = None if self.uuids is None else [self.uuids[i] for i in idx]
        return Traces(self.lat[sel].copy(), self.lon[sel].copy(), self.time[sel].copy(), off,
                      self.mode[idx].copy(), acc, tr, uu)


T_BEGIN = 1483228800  # 2017-01-01T00:00:00Z


def make_traces(graph, n_traces, n_points, sample_rate, sigma, seed, frac_bicycle=0.0, frac_ped=0.0,
                point_accuracy=None, uuid_base=0, t_begin=T_BEGIN, t_spread=86400 * 7):
    n = n_traces * n_points
    lat = np.zeros(n, np.float64)
    lon = np.zeros(n, np.float64)
    tm = np.zeros(n, np.int64)
    mode = np.zeros(n_traces, np.uint8)
    truth = np.zeros(n, np.uint32)
    P = ctypes.POINTER
    rc = lib().otrgen_traces(graph.encode(), n_traces, n_points, sample_rate, sigma, seed, frac_bicycle,
                             frac_ped, lat.ctypes.data_as(P(ctypes.c_double)),
                             lon.ctypes.data_as(P(ctypes.c_double)), tm.ctypes.data_as(P(ctypes.c_int64)),
                             mode.ctypes.data_as(P(ctypes.c_uint8)), truth.ctypes.data_as(P(ctypes.c_uint32)),
                             int(t_begin), int(t_spread))
    if rc != 0:
        raise RuntimeError('otrgen_traces failed: %d' % rc)
    off = np.arange(n_traces + 1, dtype=np.int64) * n_points
    acc = None
    if point_accuracy is not None:
        acc = np.full(n, float(point_accuracy), np.float32)
    uuids = ['veh%07d' % (uuid_base + i) for i in range(n_traces)]
    return Traces(lat, lon, tm, off, mode, acc, truth, uuids)


def make_traces_ids(graph, ids, n_points, sample_rate, sigma, seed, frac_bicycle=0.0, frac_ped=0.0,
                    point_accuracy=None, t_begin=T_BEGIN, t_spread=86400 * 7, threads=1):
    """Traces of the vehicles numbered `ids` ("veh%07d" uuids), each drawn from its own
    generator (seed, id): a uuid shard of a fleet is generated without the rest (C3).
    threads > 1: slices of `ids` generated concurrently (the same traces: per-id seeds)."""
    ids = np.ascontiguousarray(ids, np.int64)
    n_traces = len(ids)
    n = n_traces * n_points
    lat = np.zeros(n, np.float64)
    lon = np.zeros(n, np.float64)
    tm = np.zeros(n, np.int64)
    mode = np.zeros(n_traces, np.uint8)
    truth = np.zeros(n, np.uint32)
    P = ctypes.POINTER

    def run(a, b):
        if b <= a:
            return 0
        q = a * n_points
        return lib().otrgen_traces_ids(graph.encode(), b - a, ids[a:].ctypes.data_as(P(ctypes.c_int64)), n_points,
                                       sample_rate, sigma, seed, frac_bicycle, frac_ped,
                                       lat[q:].ctypes.data_as(P(ctypes.c_double)),
                                       lon[q:].ctypes.data_as(P(ctypes.c_double)),
                                       tm[q:].ctypes.data_as(P(ctypes.c_int64)),
                                       mode[a:].ctypes.data_as(P(ctypes.c_uint8)),
                                       truth[q:].ctypes.data_as(P(ctypes.c_uint32)), int(t_begin), int(t_spread))
    nt = max(1, min(int(threads), n_traces // 1000 + 1))
    cuts = np.linspace(0, n_traces, nt + 1).astype(np.int64)
    if nt == 1:
        rcs = [run(0, n_traces)]
    else:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=nt) as ex:
            rcs = list(ex.map(run, cuts[:-1].tolist(), cuts[1:].tolist()))
    if any(rc != 0 for rc in rcs):
        raise RuntimeError('otrgen_traces_ids failed: %s' % rcs)
    off = np.arange(n_traces + 1, dtype=np.int64) * n_points
    acc = None if point_accuracy is None else np.full(n, float(point_accuracy), np.float32)
    return Traces(lat, lon, tm, off, mode, acc, truth, ['veh%07d' % int(i) for i in ids])


def config_traces(name, n_traces=None, graph_cache=None):
    g, nt, npnt, sr, sig, seed, fb, fp, radius = CONFIGS[name]
    path = graph_path(g, graph_cache)
    acc = 50.0 if name == 'C4' else None
    return path, make_traces(path, n_traces or nt, npnt, sr, sig, seed, fb, fp, acc)


def _coord_text(x, style, rng):
    if style == 0:
        return repr(float(x))                      # shortest round trip (≤ 17 digits)
    if style == 1:
        return '%.6f' % x                          # a fixed-point feed (Point.java:49 prints ≤ 6)
    if style == 2:
        return '%.*f' % (int(rng.integers(0, 15)), x)
    return '%.15e' % x                             # exponent form


def probe_text(traces, kind='shard', seed=0, shuffle=0.3, styles=(0, 1, 2, 3), split_gap=None, crlf=False,
               uuids=None):
    """Probe lines for the ingest path (bench/test workload): kind 'shard' =
    "uuid,time,lat,lon,acc" (simple_reporter match() input), 'raw' = the '|' feed of the
    default valuer (c[0] time string, c[1] uuid, c[5] accuracy, c[9] lat, c[10] lon).
    A fraction `shuffle` of lines is moved to random positions (files are appended by
    competing processes); split_gap inserts a pause longer than the inactivity window
    into each trace.  Returns bytes."""
    import datetime
    rng = np.random.default_rng(seed)
    lines = []
    nl = '\r\n' if crlf else '\n'
    for t in range(traces.n_traces):
        u = uuids[t] if uuids is not None else 'veh%07d' % t
        a, b = int(traces.offsets[t]), int(traces.offsets[t + 1])
        shift = 0
        for k in range(a, b):
            if split_gap and k == (a + b) // 2:
                shift = split_gap
            tm = int(traces.time[k]) + shift
            acc = 5 + int(rng.integers(0, 20))
            st = styles[int(rng.integers(0, len(styles)))]
            la = _coord_text(traces.lat[k], st, rng)
            lo = _coord_text(traces.lon[k], st, rng)
            if kind == 'shard':
                lines.append('%s,%d,%s,%s,%d%s' % (u, tm, la, lo, acc, nl))
            else:
                ts = datetime.datetime.fromtimestamp(tm, datetime.timezone.utc).strftime('%Y-%m-%d %H:%M:%S')
                accs = '%.1f' % (acc - rng.random())
                lines.append('%s|%s|x|y|z|%s|a|b|c|%s|%s%s' % (ts, u, accs, la, lo, nl))
    n = len(lines)
    m = int(n * shuffle)
    if m:
        src = rng.choice(n, m, replace=False)
        moved = [lines[i] for i in src]
        keep = np.ones(n, bool)
        keep[src] = False
        rest = [lines[i] for i in np.flatnonzero(keep)]
        for ln in moved:
            rest.insert(int(rng.integers(0, len(rest) + 1)), ln)
        lines = rest
    return ''.join(lines).encode()
