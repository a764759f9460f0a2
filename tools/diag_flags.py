"""Diagnostic: per-tier route work and the withdrawn-label / window flag count (counter 15)
of one C2 batch (route_work on).  Usage: python tools/diag_flags.py [c2|c2dep] [n_traces]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from reporter_amd import matcher as M  # noqa: E402
from reporter_amd.tools import gen  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else 'c2'
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
path = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
gtt = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000, 'search_radius': 50,
       'gps_accuracy': 16.45}
M.configure(M.default_config(path, **(gtt if wl == 'c2' else {})))
tr = gen.make_traces(path, nt, 100, 15, 10.0, 2)
m = M.Matcher()
r = m.match_batch(tr, copy_out=False, route_work=True)
print('status', r.status, 'counters', [int(r.counters[k]) for k in range(24)])
for t in range(10):
    print('tier', t, int(r.route_tier_code[t]), [int(x) for x in r.route_tier_work[t]])
