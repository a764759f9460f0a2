"""Retry tiers give the first tier's results: a test build of the library
(libotr_tiercheck.so, -DOTR_FORCE_RETRY) sends EVERY first-tier search down the
retry kernels, and must still match the oracle field by field.  Parametrised over
the retry-tier list (OTR_TIERS): the default 256 → 448x2 → 1024 → 2048 → 4096 chain, a chain
that starts with two-searches-per-wave 384-slot tables, and direct 1024/4096; with the size
estimate scaled up (OTR_EST_K=1000) every search starts in the last retry tier, with it off
(OTR_EST_K=0) every search overflows into the first retry tier; with OTR_FORCE_EDGE=128 every
retry-tier search that has dump slots stops after 2 rounds (3 in a table's second lane group)
and the next tier resumes it from its dump in HBM (search_run NDump), tier after tier, so the
last tier finishes them.
The edge-state tiers (turn costs: the deployed per-mode defaults, a mode mix) the same way:
OTR_FORCE_EDGE fails every search of the chosen tiers, so the next one does all the work —
the 512- and 1024-state lean tiers, k_general, and for winner paths the 2048-state table
and k_general.
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
    stop, max_dumps = %r, %r
    if stop and max_dumps is None:  # forced stops: dumped in one tier, resumed in the next
        assert c[12] > 0 and c[11] > 0 and c[12] >= c[11], c
    if max_dumps is not None:  # dump slots short (or none): the rest restart, same results
        assert c[12] <= max_dumps and c[11] <= c[12], (c, max_dumps)
        if stop and max_dumps > 0:
            assert c[12] > 0, c
    from reporter_amd import _lib
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(**{k: float(v) for k, v in over.items()}), threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    # the timed launches (route_work off: the kernels compiled without the work counting,
    # other task pairings, dump-slot and queue claims) give the same output, field by field
    r2 = M.Matcher().match_batch(tr, copy_out=True, route_work=False)
    assert r2.status == 0, r2.status
    errors, stats = compare(_lib.result_to_numpy(r2), got)
    assert not errors and all(stats.values()), (errors, stats)  # (floats bit-exact too)
print('tiers ok')
'''


def _nd_words(cap):  # otr_kernels.h nd_words: u64 words of one node dump slot
    return 2 + cap + (cap + 1) // 2


# (tiers, size-estimate scale, forced stops, extra environment).  The 768-slot list with the
# estimate at 0.7 sends most C4-like searches through the two-search 448-slot tables, whose
# groups stop in different rounds: the list of round 5's nondeterministic run (a finished
# group's kmin overwritten by its partner's later rounds, dumped with the wrong kmin;
# DESIGN.md §3.4).  OTR_NDUMP_GB small: dump slots run short, the rest restart.
# OTR_OPT_RESERVE_GB huge: no optional buffer at all (no dumps, no task_dump).
TIER_CASES = [(None, None, False, {}), ('384x2,512', None, False, {}), ('512x2,2048', None, False, {}),
              ('1024', '0', False, {}), (None, '1000', False, {}), (None, None, True, {}),
              ('384x2,512', '0', True, {}), ('256,448x2,768,2048', '0.7', False, {}),
              ('256,448x2,768,2048', '0.7', True, {}), (None, None, True, {'OTR_NDUMP_GB': '0.0002'}),
              (None, None, True, {'OTR_OPT_RESERVE_GB': '1000000'})]


@pytest.mark.parametrize('tiers,est,stop,extra', TIER_CASES)
def test_retry_tiers_equal_first_tier(graph_dir, tiers, est, stop, extra):
    lib = os.path.join(ROOT, 'reporter_amd', 'libotr_tiercheck.so')
    assert os.path.exists(lib), 'build first: python -m reporter_amd.build'
    env = dict(os.environ, OTR_LIB=lib)
    for k in ('OTR_TIERS', 'OTR_EST_K', 'OTR_FORCE_EDGE', 'OTR_NDUMP_GB', 'OTR_OPT_RESERVE_GB'):
        env.pop(k, None)
    if tiers:
        env['OTR_TIERS'] = tiers
    if est is not None:
        env['OTR_EST_K'] = est
    if stop:
        env['OTR_FORCE_EDGE'] = '128'
    env.update(extra)
    max_dumps = None
    if 'OTR_NDUMP_GB' in extra:  # every node tier but the last dumps (the test build), at most this many slots
        caps = [256, 448, 1024, 2048]
        max_dumps = sum(int(float(extra['OTR_NDUMP_GB']) * 2 ** 30) // (8 * _nd_words(c)) for c in caps)
    if 'OTR_OPT_RESERVE_GB' in extra:
        max_dumps = 0
    p = subprocess.run([sys.executable, '-c', CHILD % (ROOT, graph_dir, stop, max_dumps)], env=env,
                       capture_output=True, text=True, timeout=240)
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


EDGE_CHILD = r'''
import sys
sys.path.insert(0, %r)
from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import matcher as M
from reporter_amd import _lib
from reporter_amd.tools import gen
force = %d
# the deployed configuration (every mode's default turn penalty), auto only and a mode mix
for g, nt, npnt, sr, sig, seed, fb, fp in [('city', 40, 100, 15, 10.0, 2, 0.0, 0.0),
                                           ('metro', 40, 100, 15, 10.0, 5, 0.25, 0.15)]:
    path = gen.graph_path(g, %r)
    M.configure(M.default_config(path))
    tr = gen.make_traces(path, nt, npnt, sr, sig, seed, fb, fp)
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=True, route_work=True)
    assert r.status == 0, r.status
    w = [int(r.route_tier_work[t][0]) for t in range(12)]
    # slots: 10 the OTR_E1CAP (360)-state lean tier, 9 the 512-state one, 11 the 1024-state one, 6 k_general
    if force & 1:
        assert w[10] == 0 and w[9] + w[11] + w[6] > 0, w
    if (force & 3) == 1:
        assert w[9] > 0, w
    if (force & 7) == 3:
        assert w[9] == 0 and w[11] > 0, w
    if (force & 7) == 7:
        assert w[9] == 0 and w[11] == 0 and w[6] > 0, w
    if force == 0:
        assert w[10] > 0, w
    resumed, dumped = int(r.counters[22]), int(r.counters[23])
    if force & 32:  # every first-table search stopped after 2 rounds and resumed at 512 states
        # (a search counts in its tier only when it completes there: bit 1 fails every 512-state one)
        assert dumped > 0 and (force & 2 or (w[9] > 0 and resumed > 0 and dumped >= resumed)), (w, resumed, dumped)
    if force & 64:  # and every 512-state search after 4 rounds, resumed at 1024
        assert w[11] > 0 and resumed > 0, (w, resumed, dumped)
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), tr, po.params(), threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    r2 = M.Matcher().match_batch(tr, copy_out=True, route_work=False)  # the timed kernels: same output
    assert r2.status == 0, r2.status
    errors, stats = compare(_lib.result_to_numpy(r2), got)
    assert not errors and all(stats.values()), (errors, stats)  # (floats bit-exact too)
print('edge tiers ok')
'''


@pytest.mark.parametrize('force', [0, 1, 3, 7, 24, 32, 96, 34])
def test_edge_tiers_equal_oracle(graph_dir, force):
    """libotr_tiercheck.so with OTR_FORCE_EDGE: bits 0-2 fail every 360 / 512 / 1024-state
    edge-state route search, bits 3-4 every 384 / 2048-state winner path; the next tier takes
    them (route_tier_work shows which did) and the output still equals the oracle.  Bits 5-6
    stop every 360 / 512-state search after 2 / 4 rounds: the next table resumes it from its
    dump in HBM (34: resumed at 512, then failed there and restarted at 1024)."""
    lib = os.path.join(ROOT, 'reporter_amd', 'libotr_tiercheck.so')
    assert os.path.exists(lib), 'build first: python -m reporter_amd.build'
    env = dict(os.environ, OTR_LIB=lib, OTR_FORCE_EDGE=str(force))
    for k in ('OTR_TIERS', 'OTR_EST_K'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, '-c', EDGE_CHILD % (ROOT, force, graph_dir)], env=env, capture_output=True,
                       text=True, timeout=280)
    assert p.returncode == 0 and 'edge tiers ok' in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
