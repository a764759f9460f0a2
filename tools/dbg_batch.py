#!/usr/bin/env python3
"""Diagnostic: one large device batch (the C3 N = 8 share by default) through the library
named by OTR_LIB; prints status, overflow traces and the per-tier work."""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    gp = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    ids = np.array([u for u in range(1000000) if int(hashlib.sha1(('veh%07d' % u).encode()).hexdigest()[:3], 16) % 8 == 0])[:n]
    tr = gen.make_traces_ids(gp, ids, 100, 15, 10.0, 3, 0.0, 0.0, None, t_begin=1483228800, t_spread=1800, threads=16)
    M.configure(M.default_config(gp, turn_penalty_factor=0, beta=3, sigma_z=4.07, breakage_distance=2000,
                                 search_radius=50, gps_accuracy=16.45))
    m = M.Matcher()
    t = time.time()
    r = m.match_batch(tr, copy_out=False, timing=True, route_work=True)
    print('traces', tr.n_traces, 'status', r.status, 'overflow traces', r.n_overflow_traces, 'ms', 1e3 * (time.time() - t))
    for k in range(len(r.route_tier_code)):
        if r.route_tier_code[k]:
            print(k, r.route_tier_code[k], round(r.route_tier_ms[k], 3), [int(x) for x in r.route_tier_work[k]])
    print('counters', [int(r.counters[k]) for k in range(24)])


if __name__ == '__main__':
    main()
