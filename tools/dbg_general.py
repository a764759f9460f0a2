import sys, os
sys.path.insert(0, '/root/repo')
from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import matcher as M
from reporter_amd import _lib
from reporter_amd.tools import gen
path = gen.graph_path('city', '/root/repo/build/graphs')
over = {'turn_penalty_factor': 0}
M.configure(M.default_config(path, **over))
tr = gen.make_traces(path, 40, 100, 15, 10.0, 2, 0.0, 0.0, None)
m = M.Matcher()
r = m.match_batch(tr, copy_out=True, route_work=True)
print('status', r.status, 'overflow traces', r.n_overflow_traces)
print('counters', [int(r.counters[k]) for k in range(24)])
for t in range(10):
    print('tier', t, int(r.route_tier_code[t]), [int(r.route_tier_work[t][k]) for k in range(4)])
got = _lib.result_to_numpy(r)
want = po.match_batch(po.Graph(path), tr, po.params(**over), threads=8)
errors, stats = compare(got, want)
print('errors', errors[:5])
