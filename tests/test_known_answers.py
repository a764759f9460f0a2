"""Known-answer tests of the matching semantics on hand-built graphs (oracle), and the
HIP path against the oracle on the same inputs."""
import os

import numpy as np
import pytest

from oracle import pyoracle as po
from oracle.compare import compare
from tests import kat_graphs as K


@pytest.fixture(scope='module')
def kat(graph_dir):
    path = os.path.join(graph_dir, 'kat.otrg')
    ids, segidx, segs = K.build(path)
    return path, ids, segs


def run(path, name):
    pts = K.scenarios()[name]
    b = K.batch([K.trace(pts)])
    return b, po.match_batch(po.Graph(path), b, po.params())


def route(r):
    return [int(e) for e in r['route_edge']]


def test_straight_east(kat):
    path, ids, segs = kat
    b, r = run(path, 'straight_east')
    assert route(r) == [ids['A%d>' % k] for k in range(5)]
    assert r['subpath'].max() == 0
    sid = [int(x) for x in r['seg_id']]
    assert sid == [segs[0]['id'], segs[1]['id'], segs[2]['id']]
    # first segment entered mid-edge: partial start; last: partial end; middle complete
    assert r['seg_start'][0] == -1 and r['seg_end'][-1] == -1
    assert r['seg_length'][1] == 200 and r['seg_length'][0] == -1 and r['seg_length'][2] == -1
    # vehicle at 10 m/s from x=30 at t0: node A1 (x=100) at t0+7 s, A3 (x=300) at t0+27 s
    t0 = b.time[0]
    assert abs(r['seg_start'][1] - (t0 + 7.0)) < 0.05
    assert abs(r['seg_end'][1] - (t0 + 27.0)) < 0.05
    # report(): the complete segment A1-A3 reported with next_id = A3 segment
    assert [int(x) for x in r['rep_id']] == [segs[1]['id']]
    assert int(r['rep_next'][0]) == segs[2]['id']


def test_straight_west(kat):
    path, ids, segs = kat
    b, r = run(path, 'straight_west')
    assert route(r) == [ids['A%d<' % k] for k in (4, 3, 2, 1, 0)]
    assert [int(x) for x in r['seg_id']] == [segs[3]['id']]


def test_turn_north(kat):
    path, ids, segs = kat
    b, r = run(path, 'turn_north')
    assert route(r) == [ids['A0>'], ids['A1>'], ids['B0^'], ids['B1^']]
    sid = [int(x) for x in r['seg_id']]
    assert sid == [segs[0]['id'], segs[1]['id'], segs[4]['id']]
    # the route leaves segment A1-A3 in its middle: end_time -1, length -1
    assert r['seg_end'][1] == -1 and r['seg_length'][1] == -1


def test_dual_carriageway_one_way(kat):
    path, ids, segs = kat
    b, r = run(path, 'dual_carriageway')
    assert route(r) == [ids['N0>'], ids['N1>'], ids['N2>']]
    assert set(int(x) for x in r['seg_id']) == {segs[5]['id']}


def test_breakage(kat):
    path, ids, segs = kat
    b, r = run(path, 'breakage')
    assert r['subpath'].max() == 1
    rt = route(r)
    assert 0xFFFFFFFF in rt
    cut = rt.index(0xFFFFFFFF)
    assert rt[:cut] == [ids['A0>'], ids['A1>']] and rt[cut + 1:] == [ids['I0>'], ids['I1>']]
    # report(): discontinuity = partial end followed by partial start
    assert r['stats'][0][2] >= 1


@pytest.mark.gpu
def test_known_answers_gpu_parity(kat):
    from reporter_amd import matcher as M
    path, ids, segs = kat
    M.configure(M.default_config(path))
    m = M.Matcher()
    sc = K.scenarios()
    b = K.batch([K.trace(p) for p in sc.values()])
    got = m.match_batch_numpy(b)
    want = po.match_batch(po.Graph(path), b, po.params())
    errors, stats = compare(got, want)
    assert not errors, errors


def test_short_length_graph_oracle_sanity(graph_dir):
    """The oracle matches traces on a graph whose lengths undercut its geometry."""
    path = K.build_short_lengths(os.path.join(graph_dir, 'short_len.otrg'))
    from reporter_amd.tools import gen
    tr = gen.make_traces(path, 12, 40, 3, 4.0, 17)
    r = po.match_batch(po.Graph(path), tr, po.params())
    assert r['trace_seg_off'][-1] > 0


@pytest.mark.gpu
def test_short_length_graph_gpu_parity(graph_dir):
    """A* order on the GPU keeps exact labels when stored lengths are below the straight
    line (DevGraph::h_scale) and nodes nearly coincide: bit-exact with the oracle."""
    from oracle.compare import compare
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    path = K.build_short_lengths(os.path.join(graph_dir, 'short_len.otrg'))
    M.configure(M.default_config(path))
    tr = gen.make_traces(path, 40, 60, 3, 6.0, 18)
    got = M.Matcher().match_batch_numpy(tr)
    want = po.match_batch(po.Graph(path), tr, po.params())
    errors, stats = compare(got, want)
    assert not errors, errors
    assert stats['n_seg'] > 0
