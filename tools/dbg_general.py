"""Debug helper: run the generalcheck build's cases (tests/test_gpu_tiers.py GENERAL_CHILD)
and print the per-tier work counters and the oracle comparison of each."""
import sys
sys.path.insert(0, '/root/repo')
from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import matcher as M
from reporter_amd import _lib
from reporter_amd.tools import gen
cases = [('city', 40, 100, 15, 10.0, 2, 0.0, 0.0, None, {'turn_penalty_factor': 0}),
         ('metro', 30, 60, 60, 50.0, 4, 0.0, 0.0, 50.0, {'search_radius': 200, 'max_search_radius': 200,
                                                      'turn_penalty_factor': 0}),
         ('metro', 40, 100, 15, 10.0, 5, 0.25, 0.15, None, {})]
for g, nt, npnt, sr, sig, seed, fb, fp, acc, over in cases:
    path = gen.graph_path(g, '/root/repo/build/graphs')
    M.configure(M.default_config(path, **over))
    tr = gen.make_traces(path, nt, npnt, sr, sig, seed, fb, fp, acc)
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=True, route_work=True)
    print(g, 'status', r.status, 'overflow traces', r.n_overflow_traces)
    print('counters', [int(r.counters[k]) for k in range(24)])
    for t in range(10):
        print('tier', t, int(r.route_tier_code[t]), [int(r.route_tier_work[t][k]) for k in range(4)])
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(**over), threads=8)
    errors, stats = compare(got, want)
    print('errors', errors[:3], flush=True)
