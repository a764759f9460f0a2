"""Debug helper: match a config on the GPU, find the oracle-sample traces that differ, and
re-match each alone (GPU and oracle) to see whether winners or paths differ.
Usage: python tools/debug_parity.py C4|C2 [n_sample]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from oracle.compare import compare, subset  # noqa: E402
from reporter_amd import _lib  # noqa: E402
from reporter_amd import matcher as M  # noqa: E402
from reporter_amd.tools import gen  # noqa: E402

GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
CFG = {'C2': (10000, 100, 15, 10.0, 2, None, dict(GTT, search_radius=50, gps_accuracy=16.45)),
       'C4': (20000, 60, 60, 50.0, 4, 50.0, dict(GTT, search_radius=200, max_search_radius=200,
                                                   gps_accuracy=82.24))}
name = sys.argv[1]
n_sample = int(sys.argv[2]) if len(sys.argv) > 2 else 120
nt, npnt, rate, sig, seed, acc, opts = CFG[name]
path = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
M.configure(M.default_config(path, **opts))
tr = gen.make_traces(path, nt, npnt, rate, sig, seed, 0.0, 0.0, acc, t_begin=gen.T_BEGIN, t_spread=1800)
got = _lib.result_to_numpy(M.Matcher().match_batch(tr, copy_out=True))
idx = np.linspace(0, nt - 1, n_sample).astype(np.int64)
prm = po.params(**{k: float(v) for k, v in opts.items()})
g = po.Graph(path)
bad = []
for t in idx:
    one = tr.subset(np.array([t]))
    e, _ = compare(subset(got, np.array([t]), tr.offsets), po.match_batch(g, one, prm))
    if e:
        bad.append(int(t))
print('mismatching traces in the sample:', bad)
for t in bad[:3]:
    one = tr.subset(np.array([t]))
    alone = _lib.result_to_numpy(M.Matcher().match_batch(one, copy_out=True))
    want = po.match_batch(g, one, prm)
    e_alone, _ = compare(alone, want)
    e_batch, _ = compare(subset(got, np.array([t]), tr.offsets), alone)
    print('trace', t, 'alone vs oracle:', e_alone[:3])
    print('   batch vs alone:', e_batch[:3])
    gb = subset(got, np.array([t]), tr.offsets)
    for k in ('winner', 'subpath'):
        d = np.flatnonzero(gb[k] != want[k])
        print('   %s differs at states %s: gpu %s oracle %s' % (k, d[:8], gb[k][d[:8]], want[k][d[:8]]))
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    np.savez(os.path.join(ROOT, 'gpurun_out', 'dbg_%s_%d.npz' % (name, t)),
             **{k: v for k, v in alone.items() if isinstance(v, np.ndarray)})
