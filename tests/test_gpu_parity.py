"""HIP path vs CPU oracle, field by field, through the C-ABI (include/otr.h)."""
import json

import numpy as np
import pytest

from oracle import pyoracle as po
from oracle.compare import compare
from reporter_amd import _lib
from reporter_amd import matcher as M
from reporter_amd.tools import gen

pytestmark = pytest.mark.gpu

CASES = {
    # name: (graph, n_traces, points, sample_rate, sigma, seed, frac_bike, frac_ped, accuracy, meili overrides)
    'tiny_mixed': ('tiny', 24, 40, 5, 8.0, 7, 0.3, 0.3, None, {}),
    'city_1hz': ('city', 40, 300, 1, 5.0, 1, 0.0, 0.0, None, {}),
    'city_15s': ('city', 60, 100, 15, 10.0, 2, 0.0, 0.0, None, {}),
    'city_sparse_60s': ('city', 30, 60, 60, 50.0, 4, 0.0, 0.0, 50.0,
                        {'search_radius': 200, 'max_search_radius': 200}),
    'metro_15s': ('metro', 100, 100, 15, 10.0, 3, 0.0, 0.0, None, {}),
    # C4 on the metro graph: 60 s sampling, 50 m accuracy, 200 m search radius
    'metro_sparse_60s': ('metro', 40, 60, 60, 50.0, 4, 0.0, 0.0, 50.0,
                         {'search_radius': 200, 'max_search_radius': 200}),
    # C5's mode mix (60 % auto / 25 % bicycle / 15 % pedestrian) on the metro graph
    'metro_mixed_modes': ('metro', 120, 100, 15, 10.0, 5, 0.25, 0.15, None, {}),
}


@pytest.fixture(scope='module')
def matcher():
    return M.Matcher()


# 'deployed': the reference deployment's config (Dockerfile meili overrides, per-mode turn
# penalties auto 200 / bicycle 140 / pedestrian 100, max_route_time_factor 2) — what a
# Batch.java request (mode + levels only, Batch.java:56-65) is matched with;
# 'gtt': the match_options generate_test_trace.py:44-52 sends (turn_penalty_factor 0)
CONFIGS = {'deployed': {}, 'gtt': {'turn_penalty_factor': 0}}


@pytest.mark.parametrize('cfg', list(CONFIGS))
@pytest.mark.parametrize('name', list(CASES))
def test_batch_parity(name, cfg, graph_dir, matcher):
    g, nt, npnt, sr, sig, seed, fb, fp, acc, over = CASES[name]
    over = dict(over, **CONFIGS[cfg])
    path = gen.graph_path(g, graph_dir)
    M.configure(M.default_config(path, **over))
    traces = gen.make_traces(path, nt, npnt, sr, sig, seed, fb, fp, acc)
    got = matcher.match_batch_numpy(traces)
    prm = po.params(**{k: float(v) for k, v in over.items()})
    want = po.match_batch(po.Graph(path), traces, prm, threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    assert stats['n_seg'] > 0
    assert got['status'] == 0


def test_wide_label_tier_parity(graph_dir, matcher):
    """Steps whose packed (length << sh | time) words need more than 32 bits — 120 s between
    states: time bound 2400 ds = 12 time bits, 2 km bound = 21 length bits — run in the
    64-bit-label LDS tier (k_route<2048, 1, true, false, true>): bit-exact oracle parity,
    and that tier did the searches."""
    path = gen.graph_path('metro', graph_dir)
    over = dict(CONFIGS['gtt'])
    M.configure(M.default_config(path, **over))
    traces = gen.make_traces(path, 40, 30, 120, 10.0, 6)
    r = matcher.match_batch(traces, copy_out=True, route_work=True)
    assert r.status == 0
    assert int(r.route_tier_code[8]) == 900000 + 2048
    assert int(r.route_tier_work[8][0]) > 0  # searches in the 64-bit tier
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), traces, po.params(**{k: float(v) for k, v in over.items()}), threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    assert stats['n_seg'] > 0


def test_more_than_32_candidates(graph_dir, matcher):
    """max_candidates 64 with a 200 m radius: states keep more than 32 candidates, so the
    one-state/one-trace-per-wave variants of k_prep, k_tasks and k_viterbi run (every
    other case takes the two-per-wave kernels) and steps with K > 32 targets go to the
    G = 1 route tiers; bit-exact with the oracle."""
    over = {'search_radius': 200, 'max_search_radius': 200, 'max_candidates': 64, 'turn_penalty_factor': 0}
    path = gen.graph_path('metro', graph_dir)
    M.configure(M.default_config(path, **over))
    traces = gen.make_traces(path, 30, 60, 30, 30.0, 9, 0.0, 0.0, 50.0)
    got = matcher.match_batch_numpy(traces)
    assert int(np.max(got['cand_count'])) > 32
    prm = po.params(**{k: float(v) for k, v in over.items()})
    want = po.match_batch(po.Graph(path), traces, prm, threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    assert stats['n_seg'] > 0
    assert got['status'] == 0


def test_forced_steps_more_than_32_candidates(graph_dir, matcher):
    """A gap beyond the breakage distance (the trace jumps 3.3 km half-way: a forced
    step, no route for any candidate pair) at states keeping more than 32 candidates: the
    two-search first tier writes the step's no-route rows for every target, also those
    beyond its 32-lane groups; bit-exact with the oracle."""
    over = {'search_radius': 200, 'max_search_radius': 200, 'max_candidates': 64, 'turn_penalty_factor': 0}
    path = gen.graph_path('metro', graph_dir)
    M.configure(M.default_config(path, **over))
    traces = gen.make_traces(path, 30, 60, 30, 30.0, 9, 0.0, 0.0, 50.0)
    for t in range(traces.n_traces):  # the second half 0.03 deg (3.3 km) north
        a, b = int(traces.offsets[t]), int(traces.offsets[t + 1])
        traces.lat[(a + b) // 2:b] += 0.03
    got = matcher.match_batch_numpy(traces)
    assert int(np.max(got['cand_count'])) > 32
    prm = po.params(**{k: float(v) for k, v in over.items()})
    want = po.match_batch(po.Graph(path), traces, prm, threads=8)
    errors, stats = compare(got, want)
    assert not errors, errors
    assert stats['n_seg'] > 0
    assert got['status'] == 0
