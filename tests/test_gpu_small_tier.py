"""The small-search first tiers (k_route<80,4> and k_paths<80,4>: four searches per wave;
k_route<40,8>: eight; otr_kernels.h k_ntask, otr_engine.hip k_step_lists) give the
two-search tiers' results: the same batches with the tiers off (OTR_SMALL_KEYS=0,
OTR_SMALL_PATH_KEYS=0), at their default size limits, with every eligible step sent to
them (1e9: many of those searches outgrow their tables and go on to the retry tiers), and
with the tiny tier off and every eligible step in the small one, each equal to the oracle
field by field and to one another bit for bit.
Runs in a child process per setting (the knob is read once per process)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, pickle
sys.path.insert(0, %r)
import numpy as np
from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import matcher as M
from reporter_amd import _lib
from reporter_amd.tools import gen
# (graph, traces, points, sample s, sigma, seed, accuracy, options): 1 Hz and 15 s steps on
# the city graph (small searches), 15 s and 60 s steps on the metro graph
cases = [('city', 60, 120, 1, 5.0, 11, None, {'turn_penalty_factor': 0}),
         ('city', 40, 100, 15, 10.0, 12, None, {'turn_penalty_factor': 0}),
         ('metro', 40, 100, 15, 10.0, 13, None, {'turn_penalty_factor': 0}),
         ('metro', 20, 60, 60, 50.0, 14, 50.0, {'search_radius': 200, 'max_search_radius': 200,
                                                  'turn_penalty_factor': 0})]
out = []
for g, nt, npnt, sr, sig, seed, acc, over in cases:
    path = gen.graph_path(g, %r)
    M.configure(M.default_config(path, **over))
    tr = gen.make_traces(path, nt, npnt, sr, sig, seed, 0.0, 0.0, acc)
    r = M.Matcher().match_batch(tr, copy_out=True, route_work=True)
    assert r.status == 0, r.status
    small = int(r.route_tier_work[12][0]) + int(r.route_tier_work[13][0])  # (small and tiny tiers)
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(**{k: float(v) for k, v in over.items()}), threads=8)
    errors, stats = compare(got, want)
    assert not errors, (g, sr, errors)
    r2 = M.Matcher().match_batch(tr, copy_out=True, route_work=False)
    errors, stats = compare(_lib.result_to_numpy(r2), got)
    assert not errors and all(stats.values()), (errors, stats)
    out.append((small, int(r.route_tier_code[12]) + int(r.route_tier_code[13]),
                {k: np.asarray(v) for k, v in got.items()}))
pickle.dump(out, open(%r, 'wb'))
print('small ok')
'''


def _run(graph_dir, tmp_path, keys, tiny=None):
    env = dict(os.environ)
    for k in ('OTR_SMALL_KEYS', 'OTR_SMALL_PATH_KEYS', 'OTR_TINY_KEYS', 'OTR_TIERS', 'OTR_EST_K', 'OTR_LIB'):
        env.pop(k, None)
    if keys is not None:  # (route and winner-path small tiers alike; 0 also turns the tiny tier off)
        env['OTR_SMALL_KEYS'] = keys
        env['OTR_SMALL_PATH_KEYS'] = keys
    if tiny is not None:
        env['OTR_TINY_KEYS'] = tiny
    dst = str(tmp_path / ('out_%s_%s.pkl' % (keys, tiny)))
    p = subprocess.run([sys.executable, '-c', CHILD % (ROOT, graph_dir, dst)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0 and 'small ok' in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
    import pickle
    return pickle.load(open(dst, 'rb'))


def test_small_tier_equals_two_search_tier(graph_dir, tmp_path):
    off = _run(graph_dir, tmp_path, '0')
    dflt = _run(graph_dir, tmp_path, None)
    every = _run(graph_dir, tmp_path, '1e9', '1e9')  # steps of <= 8 targets tiny, of 9..16 small
    small = _run(graph_dir, tmp_path, '1e9', '0')  # no tiny tier: every eligible step small
    assert all(s == 0 and c == 0 for s, c, _ in off)  # tiers off: not launched
    assert dflt[0][0] > 0 and dflt[0][1] in (804, 408, 1212), dflt[0][:2]  # 1 Hz steps: the small tiers search
    for v in (every, small):
        assert all(s > 0 for s, _, _ in v[:3])  # (the 200 m case keeps 32 candidates: > 16 targets)
    sys.path.insert(0, ROOT)
    from oracle.compare import compare
    for a, b, c, d in zip(off, dflt, every, small):  # field by field, floats bit for bit
        for other in (b, c, d):
            errors, stats = compare(other[2], a[2])
            assert not errors and all(stats.values()), (errors, stats)
