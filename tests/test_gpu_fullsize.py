"""BASELINE.json configs at their full sizes on the GPU: C2 (10,000 x 100
probes @15 s) and C4 (20,000 x 60 probes @60 s, accuracy 50 m, search radius 200 m), with
generate_test_trace.py's match_options (turn_penalty_factor 0) and the deployed
max_route_time_factor 2; C2 once more under the deployed per-mode turn penalties.

The oracle cannot match a whole config in test time, so: every trace is matched on the
GPU in one batch; an evenly spread sample of traces is matched by the oracle and compared
field by field with the GPU output of the same traces (a trace's results do not depend on
its batch, oracle/compare.subset); and size-independent properties hold for EVERY trace
(no trace fails, each sub-path's route is a connected edge walk, segment times lie inside
the trace's time span, reports have t0 < t1 inside it)."""
import numpy as np
import pytest

from oracle import pyoracle as po
from oracle.compare import compare, subset
from reporter_amd import _lib
from reporter_amd import matcher as M
from reporter_amd.graphfile import GraphFile
from reporter_amd.tools import gen

pytestmark = pytest.mark.gpu
GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
CONFIGS = {
    # name: (n_traces, points, rate, sigma, seed, accuracy, options, oracle sample)
    'C2': (10000, 100, 15, 10.0, 2, None, dict(GTT, search_radius=50, gps_accuracy=16.45), 150),
    'C4': (20000, 60, 60, 50.0, 4, 50.0, dict(GTT, search_radius=200, max_search_radius=200, gps_accuracy=82.24),
           120),
    'C2_deployed': (10000, 100, 15, 10.0, 2, None, {}, 60),
}


def _properties(res, tr, gf):
    assert res['status'] == 0 and res['n_overflow'] == 0
    src, dst = gf.edge_src, gf.edge_dst
    ro = res['trace_route_off']
    edges = res['route_edge']
    # connected walks between separators
    nxt_ok = np.ones(len(edges), bool)
    if len(edges) > 1:
        a, b = edges[:-1], edges[1:]
        valid = (a != 0xFFFFFFFF) & (b != 0xFFFFFFFF)
        same_trace = np.zeros(len(edges) - 1, bool)
        tid = np.repeat(np.arange(len(ro) - 1), np.diff(ro))
        same_trace = tid[:-1] == tid[1:]
        chk = valid & same_trace
        nxt_ok[:-1][chk] = dst[a[chk]] == src[b[chk]]
    assert nxt_ok.all(), 'disconnected route at %s' % np.flatnonzero(~nxt_ok)[:5]
    # times inside the trace span
    t_first = tr.time[tr.offsets[:-1]].astype(np.float64)
    t_last = tr.time[tr.offsets[1:] - 1].astype(np.float64)
    so = res['trace_seg_off']
    sid = np.repeat(np.arange(len(so) - 1), np.diff(so))
    for k in ('seg_start', 'seg_end'):
        v = res[k]
        known = v != -1.0
        assert ((v[known] >= t_first[sid[known]] - 1e-9) & (v[known] <= t_last[sid[known]] + 1e-9)).all(), k
    rp = res['trace_rep_off']
    rid = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    assert (res['rep_t0'] < res['rep_t1']).all()
    assert (res['rep_t0'] >= t_first[rid] - 1e-9).all() and (res['rep_t1'] <= t_last[rid] + 1e-9).all()
    assert (res['seg_queue'] >= 0).all()


@pytest.mark.parametrize('name', list(CONFIGS))
def test_full_size_config(name, graph_dir):
    nt, npnt, rate, sig, seed, acc, opts, n_sample = CONFIGS[name]
    path = gen.graph_path('metro', graph_dir)
    M.configure(M.default_config(path, **opts))
    tr = gen.make_traces(path, nt, npnt, rate, sig, seed, 0.0, 0.0, acc, t_begin=gen.T_BEGIN, t_spread=1800)
    got = _lib.result_to_numpy(M.Matcher().match_batch(tr, copy_out=True))
    _properties(got, tr, GraphFile(path))
    idx = np.linspace(0, nt - 1, n_sample).astype(np.int64)
    want = po.match_batch(po.Graph(path), tr.subset(idx), po.params(**opts), threads=16)
    errors, stats = compare(subset(got, idx, tr.offsets), want)
    assert not errors, errors
    assert stats['n_seg'] > 0 and stats['n_rep'] > 0


def test_c3_shard_in_one_batch(graph_dir):
    """The C3 N = 8 share in ONE device batch (125,000 traces, 12.5M probes, ~178M route tasks):
    more first-tier units than one dispatch can address (its grid size counts work-items in
    32 bits), so the first tier runs as several launches.  Every trace must match (status 0)
    and an evenly spread sample equals the oracle."""
    import hashlib
    path = gen.graph_path('metro', graph_dir)
    opts = dict(GTT, search_radius=50, gps_accuracy=16.45)
    M.configure(M.default_config(path, **opts))
    ids = np.array([u for u in range(1000000) if int(hashlib.sha1(('veh%07d' % u).encode()).hexdigest()[:3], 16) % 8 == 0])
    tr = gen.make_traces_ids(path, ids[:125000], 100, 15, 10.0, 3, 0.0, 0.0, None, t_begin=gen.T_BEGIN, t_spread=1800,
                             threads=16)
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=False, route_work=True)
    assert r.status == 0 and r.n_overflow_traces == 0
    assert int(r.counters[5]) > (1 << 25) * 2  # route tasks: more than one first-tier launch holds
    assert int(r.route_tier_work[0][0]) > (1 << 26)  # and the first tier searched them (not a quarter)
    idx = np.linspace(0, tr.n_traces - 1, 60).astype(np.int64)
    sample = tr.subset(idx)
    got = _lib.result_to_numpy(M.Matcher().match_batch(sample, copy_out=True))
    want = po.match_batch(po.Graph(path), sample, po.params(**opts), threads=16)
    errors, _ = compare(got, want)
    assert not errors, errors
