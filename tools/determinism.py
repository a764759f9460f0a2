#!/usr/bin/env python3
"""Diagnostic: one device batch run R times through the library OTR_LIB names (route_work
alternating off / on, as bench.py's timed and instrumented steps), every per-trace output
compared with the first run.  Names the first differing traces, the fields that differ,
and for each which run the CPU oracle agrees with.  Prints one JSON line.

  python tools/determinism.py --workload c4 --runs 6 [--traces N]

Results must not depend on the run (reporter_service.py:240 returns one answer per trace):
the retry tiers' dump-slot claims, work-queue claims and hash-slot races must never show.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
WORK = {  # bench.py's workloads (points, rate, sigma, seed, bike, ped, acc, traces, options)
    'c2': (100, 15, 10.0, 2, 0.0, 0.0, None, 10000, dict(GTT, search_radius=50, gps_accuracy=16.45)),
    'c2dep': (100, 15, 10.0, 2, 0.0, 0.0, None, 10000, {}),
    'c4': (60, 60, 50.0, 4, 0.0, 0.0, 50.0, 20000,
           dict(GTT, search_radius=200, max_search_radius=200, gps_accuracy=82.24)),
}
PER_STATE = ('winner', 'subpath')
PER_ROUTE = ('route_edge',)
PER_SEG = ('seg_id', 'seg_start', 'seg_end', 'seg_length', 'seg_queue', 'seg_internal', 'seg_begin_shape',
           'seg_end_shape')
PER_REP = ('rep_id', 'rep_next', 'rep_t0', 'rep_t1', 'rep_length', 'rep_queue')


def trace_view(o, t):
    """Every output of trace t, as comparable arrays."""
    v = {}
    s0, s1 = o['trace_state_off'][t], o['trace_state_off'][t + 1]
    for k in PER_STATE:
        v[k] = o[k][s0:s1]
    r0, r1 = o['trace_route_off'][t], o['trace_route_off'][t + 1]
    for k in PER_ROUTE:
        v[k] = o[k][r0:r1]
    g0, g1 = o['trace_seg_off'][t], o['trace_seg_off'][t + 1]
    for k in PER_SEG:
        v[k] = o[k][g0:g1]
    p0, p1 = o['trace_rep_off'][t], o['trace_rep_off'][t + 1]
    for k in PER_REP:
        v[k] = o[k][p0:p1]
    return v


def diff_traces(a, b, n_traces):
    """Traces whose outputs differ between two results, with the differing fields."""
    keys = ('trace_state_off', 'trace_route_off', 'trace_seg_off', 'trace_rep_off') + PER_STATE + PER_ROUTE + \
        PER_SEG + PER_REP
    if all(a[k].shape == b[k].shape and np.array_equal(a[k], b[k]) for k in keys):
        return []
    out = []
    for t in range(n_traces):
        va, vb = trace_view(a, t), trace_view(b, t)
        bad = [k for k in va if va[k].shape != vb[k].shape or not np.array_equal(va[k], vb[k])]
        if bad:
            out.append((t, bad))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', choices=sorted(WORK), default='c4')
    ap.add_argument('--runs', type=int, default=6)
    ap.add_argument('--traces', type=int, default=None)
    ap.add_argument('--oracle', type=int, default=4, help='differing traces checked against the oracle')
    args = ap.parse_args()
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    pts, rate, sig, seed, bike, ped, acc, nt, opts = WORK[args.workload]
    nt = args.traces or nt
    gp = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gp, nt, pts, rate, sig, seed, bike, ped, acc, t_begin=1483228800, t_spread=1800)
    M.configure(M.default_config(gp, **opts))
    m = M.Matcher()
    runs, work = [], []
    for i in range(args.runs):
        t0 = time.time()
        r = m.match_batch(tr, copy_out=True, timing=True, tile_rows=True, route_work=bool(i & 1))
        if r.status != 0:
            raise SystemExit('run %d: status %d' % (i, r.status))
        o = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v)
             for k, v in _lib.result_to_numpy(r).items()}
        runs.append(o)
        c = [int(x) for x in r.counters]
        work.append({'run': i, 'route_work': bool(i & 1), 'ms': round(1e3 * (time.time() - t0), 1),
                     'segments': c[7], 'resumed': c[11], 'dumped': c[12]})
        print('run %d: %s' % (i, work[-1]), file=sys.stderr, flush=True)
    diffs = {}
    for i in range(1, args.runs):
        d = diff_traces(runs[0], runs[i], tr.n_traces)
        if d:
            diffs[i] = d
    report = {'workload': args.workload, 'traces': int(tr.n_traces), 'runs': work,
              'lib': os.environ.get('OTR_LIB', 'reporter_amd/libotr.so'),
              'env': {k: v for k, v in os.environ.items() if k.startswith('OTR_')},
              'differing_runs': {str(i): {'traces': len(d), 'first': [[t, f] for t, f in d[:8]]}
                                 for i, d in diffs.items()},
              'deterministic': not diffs}
    if diffs and args.oracle > 0:
        from oracle import pyoracle as po
        from oracle.compare import compare, subset
        ts = sorted({t for d in diffs.values() for t, _ in d})[:args.oracle]
        idx = np.array(ts)
        want = po.match_batch(po.Graph(gp), tr.subset(idx), po.params(**{k: float(v) for k, v in opts.items()}),
                              threads=8)
        agree = {}
        for i, o in enumerate(runs):
            errs, _ = compare(subset(o, idx, tr.offsets), want)
            agree[i] = not errs
        report['oracle_traces'] = ts
        report['oracle_agrees_with_run'] = agree
    print(json.dumps(report))


if __name__ == '__main__':
    main()
