#!/usr/bin/env python3
"""Design statistics of the deployed configuration's edge-state searches (CPU simulation of
the GPU's exact rounds, tools/edge_stats.c): table keys, settled states, rounds per search,
and the union of one step's sources.  Analysis tool, not a test.

  python tools/edge_stats.py [--traces 300] [--workload c2dep|c4dep]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from reporter_amd.tools import gen  # noqa: E402


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        'searches', 'keys', 'settled', 'rounds', 'rounds_tmin', 'settled_tmin', 'steps', 'union_keys', 'sum_keys',
        'sources', 'union_settle_events', 'sum_settle_events')] + [
        ('hist_keys', ctypes.c_int64 * 64), ('hist_union', ctypes.c_int64 * 64), ('hist_rounds', ctypes.c_int64 * 64),
        ('pend_max', ctypes.c_int64), ('max_rounds_sum', ctypes.c_int64), ('relaxed', ctypes.c_int64),
        ('groups', ctypes.c_int64), ('hist_bmm_keys', (ctypes.c_int64 * 24) * 24),
        ('settled_out', ctypes.c_int64), ('rounds_out', ctypes.c_int64), ('scans_tmin', ctypes.c_int64),
        ('scans_out', ctypes.c_int64), ('settled_tterm', ctypes.c_int64), ('rounds_tterm', ctypes.c_int64),
        ('settled_ast', ctypes.c_int64), ('rounds_ast', ctypes.c_int64), ('settled_ast1', ctypes.c_int64),
        ('rounds_ast1', ctypes.c_int64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--traces', type=int, default=300)
    ap.add_argument('--group', type=int, default=0, help='sources per multi-source group (0: the whole step)')
    ap.add_argument('--workload', default='c2dep', choices=['c2dep'])
    args = ap.parse_args()
    so = os.path.join(ROOT, 'tools', 'libedgestats.so')
    src = os.path.join(ROOT, 'tools', 'edge_stats.c')
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(['gcc', '-O2', '-std=gnu11', '-shared', '-fPIC', '-ffp-contract=off', '-o', so, src,
                               '-lm', '-lpthread'])
    L = ctypes.CDLL(so)
    gpath = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gpath, args.traces, 100, 15, 10.0, 2, 0.0, 0.0, None, t_begin=1483228800, t_spread=1800)
    g = po.Graph(gpath)
    prm = po.params()
    S = Stats()
    P = ctypes.POINTER
    L.es_run.argtypes = [ctypes.c_void_p, P(po.Params), ctypes.c_int32, P(ctypes.c_int64), P(ctypes.c_double),
                         P(ctypes.c_double), P(ctypes.c_int64), ctypes.c_int, P(Stats)]
    L.es_run(g.h, prm, tr.n_traces, tr.offsets.ctypes.data_as(P(ctypes.c_int64)),
             tr.lat.ctypes.data_as(P(ctypes.c_double)), tr.lon.ctypes.data_as(P(ctypes.c_double)),
             tr.time.ctypes.data_as(P(ctypes.c_int64)), args.group, ctypes.byref(S))
    n = max(S.searches, 1)
    st = max(S.groups, 1)
    hk = np.array(S.hist_keys[:], np.int64)
    cum = np.cumsum(hk) / n
    hu = np.array(S.hist_union[:], np.int64)
    cu = np.cumsum(hu) / st
    out = {
        'traces': args.traces, 'searches': S.searches, 'steps': S.steps,
        'keys_per_search': S.keys / n, 'settled_per_search': S.settled / n, 'relaxed_per_search': S.relaxed / n,
        'rounds_per_search': S.rounds / n,
        'settled_per_search_tmin': S.settled_tmin / n, 'rounds_per_search_tmin': S.rounds_tmin / n,
        'settled_per_search_out': S.settled_out / n, 'rounds_per_search_out': S.rounds_out / n,
        'settled_per_search_tterm': S.settled_tterm / n, 'rounds_per_search_tterm': S.rounds_tterm / n,
        'settled_per_search_astar': S.settled_ast / n, 'rounds_per_search_astar': S.rounds_ast / n,
        'settled_per_search_astar1': S.settled_ast1 / n, 'rounds_per_search_astar1': S.rounds_ast1 / n,
        'pending_scanned_per_search_tmin': S.scans_tmin / n, 'pending_scanned_per_search_out': S.scans_out / n,
        'groups': S.groups, 'sources_per_group': S.sources / st, 'sum_keys_per_step': S.sum_keys / st,
        'union_keys_per_step': S.union_keys / st, 'max_rounds_per_step': S.max_rounds_sum / st,
        'settle_events_separate_per_step': S.sum_settle_events / st,
        'settle_events_union_per_step': S.union_settle_events / st,
        'pend_max': S.pend_max,
        'keys_cdf_by_32': {str(32 * (i + 1)): round(float(cum[i]), 4) for i in range(24)},
        'union_cdf_by_64': {str(64 * (i + 1)): round(float(cu[i]), 4) for i in range(24)},
        'rounds_hist': {str(i): int(S.hist_rounds[i]) for i in range(64) if S.hist_rounds[i]},
    }
    print(json.dumps(out, indent=1))
    hb = np.array([[S.hist_bmm_keys[i][j] for j in range(24)] for i in range(24)])
    print('route bound (100 m) -> searches, mean keys, P(keys > 224), P(keys > 320), share of all keys > 320')
    over = hb[:, 10:].sum()
    for i in range(24):
        n_i = hb[i].sum()
        if n_i:
            mk = (hb[i] * (np.arange(24) * 32 + 16)).sum() / n_i
            print('  %4d m: %7d  %6.1f  %.3f  %.3f  %.3f' % (i * 100, n_i, mk, hb[i][7:].sum() / n_i, hb[i][10:].sum() / n_i,
                                                           hb[i][10:].sum() / max(over, 1)))


if __name__ == '__main__':
    main()
