"""ctypes bindings for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (reporter_amd) never does.  See oracle.h for provenance.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
KMAX = 64
NO_ID = 0xFFFFFFFFFFFFFFFF
P = ctypes.POINTER


class Params(ctypes.Structure):
    _fields_ = [('sigma_z', ctypes.c_double), ('beta', ctypes.c_double),
                ('max_route_distance_factor', ctypes.c_double), ('max_route_time_factor', ctypes.c_double),
                ('breakage_distance', ctypes.c_double), ('interpolation_distance', ctypes.c_double),
                ('search_radius', ctypes.c_double), ('max_search_radius', ctypes.c_double),
                ('gps_accuracy', ctypes.c_double), ('turn_penalty_factor', ctypes.c_double),
                ('speed_kph', ctypes.c_double), ('queue_kph', ctypes.c_double),
                ('max_candidates', ctypes.c_int32), ('threshold_sec', ctypes.c_int32)]


MODES = ('auto', 'bicycle', 'pedestrian')
# Restated valhalla_build_config meili section (UPSTREAM 2.3.x) with the
# reference deployment's overrides (Dockerfile:14-17,42-49: sigma_z 4.07, beta 3,
# max_route_distance_factor 5, max_route_time_factor 2), plus this build's per-mode route
# speeds and queue thresholds.
DEFAULTS = dict(sigma_z=4.07, beta=3.0, max_route_distance_factor=5.0, max_route_time_factor=2.0,
                breakage_distance=2000.0, interpolation_distance=10.0, search_radius=50.0,
                max_search_radius=100.0, gps_accuracy=5.0, turn_penalty_factor=0.0, speed_kph=0.0,
                queue_kph=10.0, max_candidates=32, threshold_sec=15)
MODE_DEFAULTS = {'auto': dict(turn_penalty_factor=200.0, search_radius=50.0),
                 'bicycle': dict(turn_penalty_factor=140.0, speed_kph=18.0, queue_kph=5.0),
                 'pedestrian': dict(turn_penalty_factor=100.0, search_radius=50.0, speed_kph=5.1, queue_kph=2.0)}


def params(modes=None, **kw):
    """Per-mode parameter array (ORC_MODES): DEFAULTS, then MODE_DEFAULTS[mode], then
    modes[mode] (config sections), then kw applied to every mode — as a request's
    match_options override the configured values (reporter_amd.matcher.default_config
    builds the same configuration for the engine)."""
    arr = (Params * 3)()
    for i, m in enumerate(MODES):
        d = dict(DEFAULTS)
        d.update(MODE_DEFAULTS[m])
        d.update((modes or {}).get(m, {}))
        d.update(kw)
        d['max_candidates'] = int(d['max_candidates'])
        d['threshold_sec'] = int(d['threshold_sec'])
        arr[i] = Params(**{k: d[k] for k, _ in Params._fields_})
    return arr


class Result(ctypes.Structure):
    _fields_ = [('n_traces', ctypes.c_int32), ('n_states', ctypes.c_int64),
                ('trace_state_off', P(ctypes.c_int64)), ('state_probe', P(ctypes.c_int64)),
                ('cand_count', P(ctypes.c_int32)), ('cand_edge', P(ctypes.c_uint32)),
                ('cand_p', P(ctypes.c_double)), ('cand_sqd', P(ctypes.c_double)),
                ('winner', P(ctypes.c_int32)), ('subpath', P(ctypes.c_int32)),
                ('trace_route_off', P(ctypes.c_int64)), ('route_edge', P(ctypes.c_uint32)),
                ('n_route', ctypes.c_int64), ('trace_seg_off', P(ctypes.c_int64)), ('n_seg', ctypes.c_int64),
                ('seg_id', P(ctypes.c_uint64)), ('seg_start', P(ctypes.c_double)),
                ('seg_end', P(ctypes.c_double)), ('seg_length', P(ctypes.c_int32)),
                ('seg_queue', P(ctypes.c_int32)), ('seg_internal', P(ctypes.c_uint8)),
                ('seg_begin_shape', P(ctypes.c_int32)), ('seg_end_shape', P(ctypes.c_int32)),
                ('seg_way_off', P(ctypes.c_int64)), ('seg_way', P(ctypes.c_uint32)),
                ('trace_rep_off', P(ctypes.c_int64)), ('n_rep', ctypes.c_int64),
                ('rep_id', P(ctypes.c_uint64)), ('rep_next', P(ctypes.c_uint64)),
                ('rep_t0', P(ctypes.c_double)), ('rep_t1', P(ctypes.c_double)),
                ('rep_length', P(ctypes.c_int32)), ('rep_queue', P(ctypes.c_int32)),
                ('shape_used', P(ctypes.c_int32)), ('stats', P(ctypes.c_int32)),
                ('stats_len', P(ctypes.c_double))]


class ReportOut(ctypes.Structure):
    _fields_ = [('n_rep', ctypes.c_int32), ('shape_used', ctypes.c_int32), ('counts', ctypes.c_int32 * 6),
                ('lengths', ctypes.c_double * 2), ('length_set', ctypes.c_int32 * 2)]


_L = None


def lib():
    global _L
    if _L is None:
        path = os.path.join(_HERE, 'liboracle.so')
        if not os.path.exists(path):
            raise RuntimeError('oracle/liboracle.so not built (make -C oracle)')
        L = ctypes.CDLL(path)
        L.orc_graph_load.argtypes = [ctypes.c_char_p]
        L.orc_graph_load.restype = ctypes.c_void_p
        L.orc_graph_free.argtypes = [ctypes.c_void_p]
        L.orc_match_batch.argtypes = [ctypes.c_void_p, P(Params), ctypes.c_int32, P(ctypes.c_int64),
                                      P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int64),
                                      P(ctypes.c_float), P(ctypes.c_uint8), ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_int32, P(Result)]
        L.orc_result_free.argtypes = [P(Result)]
        L.orc_report.argtypes = [ctypes.c_int32, P(ctypes.c_uint8), P(ctypes.c_uint64), P(ctypes.c_double),
                                 P(ctypes.c_double), P(ctypes.c_uint8), P(ctypes.c_int32), P(ctypes.c_uint8),
                                 P(ctypes.c_int32), P(ctypes.c_int32), ctypes.c_int64, ctypes.c_double,
                                 ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint64), P(ctypes.c_uint64),
                                 P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_int32),
                                 P(ReportOut)]
        L.orc_route.argtypes = [ctypes.c_void_p, P(Params), ctypes.c_int, ctypes.c_uint32, ctypes.c_double,
                                ctypes.c_uint32, ctypes.c_double, ctypes.c_double, ctypes.c_int64,
                                P(ctypes.c_double), P(ctypes.c_int64), P(ctypes.c_int64)]
        L.orc_route.restype = ctypes.c_int
        L.orc_edge_info.argtypes = [ctypes.c_void_p, P(Params), ctypes.c_uint32, P(ctypes.c_int32),
                                    P(ctypes.c_int32), P(ctypes.c_int64)]
        L.orc_turn_table.argtypes = [P(Params), P(ctypes.c_int32)]
        _L = L
    return _L


def _ptr(a, t):
    return a.ctypes.data_as(P(t)) if a is not None else None


def _arr(p, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)


class Graph:
    def __init__(self, path):
        self.h = lib().orc_graph_load(path.encode())
        if not self.h:
            raise RuntimeError('oracle failed to load graph %s' % path)

    def __del__(self):
        if getattr(self, 'h', None):
            lib().orc_graph_free(self.h)
            self.h = None

    def route(self, se, sp, de, dp, bound, dt_sec=0, prm=None, mode=0):
        """(length m, time 0.1 s, turn cost mm) of one transition's route, or None."""
        prm = prm if prm is not None else params()
        d, t, c = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
        ok = lib().orc_route(self.h, ctypes.byref(prm[mode]), mode, se, sp, de, dp, bound, int(dt_sec),
                             ctypes.byref(d), ctypes.byref(t), ctypes.byref(c))
        return (d.value, t.value, c.value) if ok else None

    def edge_info(self, e, prm=None, mode=0):
        """(begin heading, end heading, route time 0.1 s) of edge e."""
        prm = prm if prm is not None else params()
        hb, he, t = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        lib().orc_edge_info(self.h, ctypes.byref(prm[mode]), e, ctypes.byref(hb), ctypes.byref(he), ctypes.byref(t))
        return hb.value, he.value, t.value


def turn_table(prm, mode=0):
    tab = (ctypes.c_int32 * 181)()
    lib().orc_turn_table(ctypes.byref(prm[mode]), tab)
    return list(tab)


def levels_mask(levels):
    m = 0
    for l in levels:
        if 0 <= l < 32:
            m |= 1 << l
    return m


def match_batch(graph, traces, prm=None, report_levels=(0, 1), transition_levels=(0, 1), threads=1):
    """Run the oracle over a gen.Traces batch; returns a dict of numpy arrays."""
    prm = prm or params()
    r = Result()
    acc = traces.accuracy
    lib().orc_match_batch(graph.h, prm, traces.n_traces, _ptr(traces.offsets, ctypes.c_int64),
                          _ptr(traces.lat, ctypes.c_double), _ptr(traces.lon, ctypes.c_double),
                          _ptr(traces.time, ctypes.c_int64), _ptr(acc, ctypes.c_float),
                          _ptr(traces.mode, ctypes.c_uint8), levels_mask(report_levels),
                          levels_mask(transition_levels), threads, ctypes.byref(r))
    nt, ns, nseg, nrep = r.n_traces, r.n_states, r.n_seg, r.n_rep
    out = dict(
        trace_state_off=_arr(r.trace_state_off, nt + 1, np.int64),
        state_probe=_arr(r.state_probe, ns, np.int64),
        cand_count=_arr(r.cand_count, ns, np.int32),
        cand_edge=_arr(r.cand_edge, ns * KMAX, np.uint32).reshape(ns, KMAX),
        cand_p=_arr(r.cand_p, ns * KMAX, np.float64).reshape(ns, KMAX),
        cand_sqd=_arr(r.cand_sqd, ns * KMAX, np.float64).reshape(ns, KMAX),
        winner=_arr(r.winner, ns, np.int32), subpath=_arr(r.subpath, ns, np.int32),
        trace_route_off=_arr(r.trace_route_off, nt + 1, np.int64),
        route_edge=_arr(r.route_edge, r.n_route, np.uint32),
        trace_seg_off=_arr(r.trace_seg_off, nt + 1, np.int64),
        seg_id=_arr(r.seg_id, nseg, np.uint64), seg_start=_arr(r.seg_start, nseg, np.float64),
        seg_end=_arr(r.seg_end, nseg, np.float64), seg_length=_arr(r.seg_length, nseg, np.int32),
        seg_queue=_arr(r.seg_queue, nseg, np.int32), seg_internal=_arr(r.seg_internal, nseg, np.uint8),
        seg_begin_shape=_arr(r.seg_begin_shape, nseg, np.int32),
        seg_end_shape=_arr(r.seg_end_shape, nseg, np.int32),
        seg_way_off=_arr(r.seg_way_off, nseg + 1, np.int64),
        trace_rep_off=_arr(r.trace_rep_off, nt + 1, np.int64),
        rep_id=_arr(r.rep_id, nrep, np.uint64), rep_next=_arr(r.rep_next, nrep, np.uint64),
        rep_t0=_arr(r.rep_t0, nrep, np.float64), rep_t1=_arr(r.rep_t1, nrep, np.float64),
        rep_length=_arr(r.rep_length, nrep, np.int32), rep_queue=_arr(r.rep_queue, nrep, np.int32),
        shape_used=_arr(r.shape_used, nt, np.int32),
        stats=_arr(r.stats, nt * 7, np.int32).reshape(nt, 7),
        stats_len=_arr(r.stats_len, nt * 2, np.float64).reshape(nt, 2),
    )
    out['seg_way'] = _arr(r.seg_way, int(out['seg_way_off'][-1]) if nseg else 0, np.uint32)
    lib().orc_result_free(ctypes.byref(r))
    return out


def report_segments(segs, end_time, threshold, report_levels, transition_levels):
    """orc_report over a list of meili-style segment dicts; returns report() dict."""
    n = len(segs)
    has_id = np.array([('segment_id' in s and s['segment_id'] is not None) for s in segs] or [0], np.uint8)
    sid = np.array([int(s.get('segment_id') or 0) for s in segs] or [0], np.uint64)
    st = np.array([float(s['start_time']) for s in segs] or [0], np.float64)
    en = np.array([float(s['end_time']) for s in segs] or [0], np.float64)
    internal = np.array([bool(s.get('internal', False)) for s in segs] or [0], np.uint8)
    q = np.array([int(s.get('queue_length') or 0) for s in segs] or [0], np.int32)
    hl = np.array([s.get('length') is not None for s in segs] or [0], np.uint8)
    ln = np.array([int(s.get('length') or 0) for s in segs] or [0], np.int32)
    bs = np.array([int(s.get('begin_shape_index') or 0) for s in segs] or [0], np.int32)
    m = max(n, 1)
    rid = np.zeros(m, np.uint64)
    rnx = np.zeros(m, np.uint64)
    t0 = np.zeros(m)
    t1 = np.zeros(m)
    rl = np.zeros(m, np.int32)
    rq = np.zeros(m, np.int32)
    o = ReportOut()
    lib().orc_report(n, _ptr(has_id, ctypes.c_uint8), _ptr(sid, ctypes.c_uint64), _ptr(st, ctypes.c_double),
                     _ptr(en, ctypes.c_double), _ptr(internal, ctypes.c_uint8), _ptr(q, ctypes.c_int32),
                     _ptr(hl, ctypes.c_uint8), _ptr(ln, ctypes.c_int32), _ptr(bs, ctypes.c_int32), int(end_time),
                     float(threshold), levels_mask(report_levels), levels_mask(transition_levels),
                     _ptr(rid, ctypes.c_uint64), _ptr(rnx, ctypes.c_uint64), _ptr(t0, ctypes.c_double),
                     _ptr(t1, ctypes.c_double), _ptr(rl, ctypes.c_int32), _ptr(rq, ctypes.c_int32),
                     ctypes.byref(o))
    reports = []
    for i in range(o.n_rep):
        r = {'id': int(rid[i]), 't0': float(t0[i]), 't1': float(t1[i]), 'length': int(rl[i]),
             'queue_length': int(rq[i])}
        if int(rnx[i]) != NO_ID:
            r['next_id'] = int(rnx[i])
        reports.append(r)
    c = list(o.counts)
    res = {'datastore': {'mode': 'auto', 'reports': reports},
           'stats': {'successful_matches': {'count': c[0], 'length': o.lengths[0] if o.length_set[0] else 0},
                     'unreported_matches': {'count': c[1], 'length': o.lengths[1] if o.length_set[1] else 0},
                     'match_errors': {'discontinuities': c[2], 'invalid_speeds': c[3], 'invalid_times': c[4]},
                     'unassociated_segments': c[5]}}
    if o.shape_used >= 0:
        res['shape_used'] = o.shape_used
    return res
