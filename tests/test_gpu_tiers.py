"""Retry tiers give the first tier's results: a test build of the library
(libotr_tiercheck.so, -DOTR_FORCE_RETRY) sends EVERY first-tier search down the
retry kernels, and must still match the oracle field by field.  Parametrised over
the retry-tier list (OTR_TIERS): the default 256 → 448x2 → 1024 → 2048 → 4096 chain, a chain
that starts with two-searches-per-wave 384-slot tables, and direct 1024/4096; with
OTR_DIRECT_BMM=0 every search skips the first tier on its own.
Runs in a child process (one library per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path.insert(0, %r)
from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import matcher as M
from reporter_amd.tools import gen
# turn_penalty_factor 0 (generate_test_trace.py:47): node searches, i.e. the LDS tiers
for g, nt, npnt, sr, sig, seed, acc, over in [('city', 40, 100, 15, 10.0, 2, None, {'turn_penalty_factor': 0}),
                                             ('metro', 30, 60, 60, 50.0, 4, 50.0,
                                              {'search_radius': 200, 'max_search_radius': 200,
                                               'turn_penalty_factor': 0})]:
    path = gen.graph_path(g, %r)
    M.configure(M.default_config(path, **over))
    tr = gen.make_traces(path, nt, npnt, sr, sig, seed, 0.0, 0.0, acc)
    m = M.Matcher()  # owns the host result arrays
    r = m.match_batch(tr, copy_out=True, route_work=True)
    assert r.status == 0, r.status
    c = [int(r.counters[k]) for k in range(24)]
    assert c[9] > 0, c  # the retry tiers settled nodes (and wrote every transition row)
    from reporter_amd import _lib
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(**{k: float(v) for k, v in over.items()}), threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
print('tiers ok')
'''


@pytest.mark.parametrize('tiers,direct', [(None, None), ('384x2,512', None), ('512x2,2048', None), ('1024', '0')])
def test_retry_tiers_equal_first_tier(graph_dir, tiers, direct):
    lib = os.path.join(ROOT, 'reporter_amd', 'libotr_tiercheck.so')
    assert os.path.exists(lib), 'build first: python -m reporter_amd.build'
    env = dict(os.environ, OTR_LIB=lib)
    env.pop('OTR_TIERS', None)
    env.pop('OTR_DIRECT_BMM', None)
    if tiers:
        env['OTR_TIERS'] = tiers
    if direct is not None:
        env['OTR_DIRECT_BMM'] = direct
    p = subprocess.run([sys.executable, '-c', CHILD % (ROOT, graph_dir)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0 and 'tiers ok' in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


GENERAL_CHILD = r'''
import sys
sys.path.insert(0, %r)
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
    path = gen.graph_path(g, %r)
    M.configure(M.default_config(path, **over))
    tr = gen.make_traces(path, nt, npnt, sr, sig, seed, fb, fp, acc)
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=True, route_work=True)
    assert r.status == 0, r.status
    c = [int(r.counters[k]) for k in range(24)]
    gen_searches = int(r.route_tier_work[6][0])
    assert c[3] == 0 and gen_searches > 0, (c, gen_searches)  # nothing in the LDS tiers, all in k_general
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(**over), threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
print('general ok')
'''


def test_general_search_equals_oracle(graph_dir):
    """libotr_generalcheck.so (-DOTR_FORCE_GENERAL) runs EVERY route search and winner
    path in the global-memory kernel (k_general, edge states, 64-bit labels), also the
    node searches the LDS tiers normally take: it must equal the oracle field by field."""
    lib = os.path.join(ROOT, 'reporter_amd', 'libotr_generalcheck.so')
    assert os.path.exists(lib), 'build first: python -m reporter_amd.build'
    env = dict(os.environ, OTR_LIB=lib)
    p = subprocess.run([sys.executable, '-c', GENERAL_CHILD % (ROOT, graph_dir)], env=env, capture_output=True,
                       text=True, timeout=280)
    assert p.returncode == 0 and 'general ok' in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
