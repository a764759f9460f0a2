"""Hand-derived known answers for the route-time bound (max_route_time_factor), turn
costs (turn_penalty_factor), U-turns and queue_length — the semantics of DESIGN.md
§3.4-3.8 — on the CPU oracle, plus GPU parity on the same inputs (-m gpu).

References: max_route_time_factor = 2 (Dockerfile:17,48); per-mode turn_penalty_factor
(valhalla_build_config meili section); queue_length README.md:283,295."""
import math
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


@pytest.fixture(scope='module')
def slow(graph_dir):
    path = os.path.join(graph_dir, 'kat_slow.otrg')
    return path, K.build_slow(path)


def _match(path, pts, dt, **kw):
    b = K.batch([K.trace(pts, dt=dt)])
    return b, po.match_batch(po.Graph(path), b, po.params(**kw))


# ---- graph-derived data ---------------------------------------------------------------
def test_turn_table_values():
    tab = po.turn_table(po.params())  # auto: turn_penalty_factor 200
    for td in (0, 45, 90, 135, 180):
        want = 1000.0 * 200.0 * math.exp(-td / 45.0)
        assert abs(tab[td] - want) <= 1.0, (td, tab[td], want)
    assert tab[0] == 200000 and tab[90] == 27067 and tab[180] == 3663
    assert po.turn_table(po.params(turn_penalty_factor=0)) == [0] * 181


def test_headings_and_edge_times(kat, slow):
    path, ids, _ = kat
    g = po.Graph(path)
    assert g.edge_info(ids['A0>'])[:2] == (90, 90)
    assert g.edge_info(ids['A0<'])[:2] == (270, 270)
    assert g.edge_info(ids['B0^'])[:2] == (0, 0)
    assert g.edge_info(ids['B0v'])[:2] == (180, 180)
    spath, sid = slow
    gs = po.Graph(spath)
    # 100 m at 50 km/h = 7.2 s; at 5 km/h = 72 s (0.1 s units)
    assert gs.edge_info(sid['T0>'])[2] == 72
    assert gs.edge_info(sid['T2>'])[2] == 720
    # bicycle: capped at 18 km/h -> 20 s; pedestrian 5.1 km/h -> 70.6 s
    assert gs.edge_info(sid['T0>'], mode=1)[2] == 200
    assert gs.edge_info(sid['T0>'], mode=2)[2] == 706


# ---- time bound ------------------------------------------------------------------------
def test_route_time_bound_by_hand(slow):
    path, sid = slow
    g = po.Graph(path)
    prm = po.params(turn_penalty_factor=0)
    # T1> at 0.5 -> T3> at 0.5: 50 + 100 + 50 m; 3.6 s + 72 s + 3.6 s = 79.2 s
    r = g.route(sid['T1>'], 0.5, sid['T3>'], 0.5, 1000.0, dt_sec=40, prm=prm)
    assert r is not None and abs(r[0] - 200.0) < 0.1 and r[1] == 792  # lengths from micro-degree nodes
    assert g.route(sid['T1>'], 0.5, sid['T3>'], 0.5, 1000.0, dt_sec=39, prm=prm) is None  # 780 < 792
    assert g.route(sid['T1>'], 0.5, sid['T3>'], 0.5, 1000.0, dt_sec=0, prm=prm) is not None  # no bound
    r = g.route(sid['T1>'], 0.5, sid['T3>'], 0.5, 1000.0, dt_sec=10,
                prm=po.params(turn_penalty_factor=0, max_route_time_factor=0))
    assert r is not None and r[1] == 0  # factor 0: no time bound (times not tracked)
    # same edge forward: part of the edge's time
    r = g.route(sid['T2>'], 0.25, sid['T2>'], 0.75, 1000.0, dt_sec=100, prm=prm)
    assert r is not None and r[1] == 360
    assert g.route(sid['T2>'], 0.25, sid['T2>'], 0.75, 1000.0, dt_sec=17, prm=prm) is None  # 340 < 360


def test_slow_block_breaks_trace(slow):
    """Probes 4 s apart cross a 5 km/h block at 12.5 m/s.  Crossing the block takes 72 s,
    more than any step's bound (2 x 4 s), so no route may use it: the probes on the block
    snap to its end nodes (within the 50 m radius) and the trace breaks exactly once
    between them; the slow edge never appears in the route.  With
    max_route_time_factor = 0 the trace is one sub-path through the block."""
    path, sid = slow
    pts = K.slow_scenarios()['through_slow_block']
    b, r = _match(path, pts, 4, turn_penalty_factor=0)
    assert r['subpath'].tolist() == [0, 0, 0, 0, 0, 1, 1, 1, 1, 1]
    assert [int(e) for e in r['route_edge']] == [sid['T0>'], sid['T1>'], 0xFFFFFFFF, sid['T3>'], sid['T4>']]
    b, r0 = _match(path, pts, 4, turn_penalty_factor=0, max_route_time_factor=0)
    assert r0['subpath'].max() == 0
    assert [int(e) for e in r0['route_edge']] == [sid['T%d>' % k] for k in range(5)]


# ---- turn costs ------------------------------------------------------------------------
def test_turn_penalty_prefers_straight(kat):
    """Without turn costs the last probe matches the side street (nearer, left turn);
    with the auto default (200) going straight on costs 3.7 m instead of 27.1 m and wins."""
    path, ids, segs = kat
    pts = K.turn_scenarios()['straight_or_left']
    b, r0 = _match(path, pts, 10, turn_penalty_factor=0)
    last = int(r0['trace_state_off'][1]) - 1
    assert int(r0['cand_edge'][last][r0['winner'][last]]) == ids['B0^']
    b, r = _match(path, pts, 10)
    assert int(r['cand_edge'][last][r['winner'][last]]) == ids['A2>']
    assert [int(e) for e in r['route_edge']][-2:] == [ids['A1>'], ids['A2>']]


def test_turn_costs_in_route(kat):
    """turn(A1>, A2>) is straight (180 degrees): 3663 mm at 200; a left turn A1> -> B0^ at
    node A2 is 90 degrees: 27067 mm; a U-turn (0 degrees) 200000 mm."""
    path, ids, _ = kat
    g = po.Graph(path)
    prm = po.params()
    r = g.route(ids['A1>'], 0.5, ids['A2>'], 0.5, 1000.0, dt_sec=100, prm=prm)
    assert r[2] == 3663
    r = g.route(ids['A1>'], 0.5, ids['B0^'], 0.5, 1000.0, dt_sec=100, prm=prm)
    assert r[2] == 27067
    r = g.route(ids['A1>'], 0.5, ids['A1<'], 0.5, 1000.0, dt_sec=100, prm=prm)
    assert abs(r[0] - 100.0) < 0.1 and r[2] == 200000  # U-turn at A2
    # straight over two nodes: A0> -> A2> passes A1 and A2 (2 x straight)
    r = g.route(ids['A0>'], 0.5, ids['A2>'], 0.5, 1000.0, dt_sec=100, prm=prm)
    assert r[2] == 2 * 3663
    assert g.route(ids['A1>'], 0.5, ids['B0^'], 0.5, 1000.0, dt_sec=100, prm=po.params(turn_penalty_factor=0))[2] == 0


@pytest.mark.parametrize('tpf', [0, 200])
def test_u_turn_route(kat, tpf):
    """East to x = 290, then back west from x = 280 (2 s later: 30 m of route in 2.2 s at
    50 km/h, inside the 4 s bound): the route U-turns at node A3 (x = 300)."""
    path, ids, segs = kat
    pts = K.turn_scenarios()['u_turn']
    b, r = _match(path, pts, 2, turn_penalty_factor=tpf)
    rt = [int(e) for e in r['route_edge']]
    assert 0xFFFFFFFF not in rt
    assert rt == [ids['A0>'], ids['A1>'], ids['A2>'], ids['A2<'], ids['A1<'], ids['A0<']]


# ---- queue_length ----------------------------------------------------------------------
def test_queue_length_on_deceleration(kat):
    path, ids, segs = kat
    b, r = _match(path, K.queue_scenario(), 2)
    sid = [int(x) for x in r['seg_id']]
    k = sid.index(segs[1]['id'])  # A1-A3, complete
    assert r['seg_length'][k] == 200
    assert r['seg_queue'][k] == 99
    # the first segment (entered mid-edge, exit at x = 100 at 10 m/s) has no queue
    assert r['seg_queue'][0] == 0
    # report() carries it into datastore reports
    rk = [int(x) for x in r['rep_id']].index(segs[1]['id'])
    assert r['rep_queue'][rk] == 99
    # a higher threshold (20 km/h) makes the piece x = 190 -> 201 (11 m in 2 s, 19.8 km/h)
    # slow too, but not the one before it (20 m in 2 s, 36 km/h): 300 - 190 = 110 m
    b, r2 = _match(path, K.queue_scenario(), 2, queue_kph=20.0)
    assert r2['seg_queue'][k] == 110


@pytest.fixture(scope='module')
def square(graph_dir):
    path = os.path.join(graph_dir, 'kat_square.otrg')
    return path, K.build_square(path)


def test_equal_length_routes_decided_by_turns(square):
    """Both ways around the diamond have the same length and time to the millimetre: without
    turn costs the route takes T's smaller-id in-edge; with them it comes via Q, whose
    turn into T-N (45 degrees off straight: turn degree 135) costs less than P's (135 off:
    degree 45); the turns at S and at P / Q mirror each other."""
    path, ids = square
    g = po.Graph(path)
    tab = po.turn_table(po.params())
    d, t, c = g.route(ids['WS>'], 0.5, ids['TN>'], 0.5, 2000.0, dt_sec=40, prm=po.params())
    assert c == tab[135] + tab[90] + tab[135]  # S: 45 off, Q: 90, T: 45 off
    d_p = g.route(ids['WS>'], 0.5, ids['PT>'], 0.999, 2000.0, dt_sec=40, prm=po.params())[0]
    d_q = g.route(ids['WS>'], 0.5, ids['QT>'], 0.999, 2000.0, dt_sec=40, prm=po.params())[0]
    assert d_p == d_q  # the tie
    b, r = _match(path, K.square_trace(), 20)
    route = [int(e) for e in r['route_edge'] if e != 0xFFFFFFFF]
    assert ids['QT>'] in route and ids['PT>'] not in route


# ---- the route key is length + turn cost; the bounds prune during the search ------------
@pytest.fixture(scope='module')
def block(graph_dir):
    path = os.path.join(graph_dir, 'kat_block.otrg')
    return path, K.build_block(path)


@pytest.fixture(scope='module')
def bypass(graph_dir):
    path = os.path.join(graph_dir, 'kat_bypass.otrg')
    return path, K.build_bypass(path)


@pytest.fixture(scope='module')
def stale(graph_dir):
    path = os.path.join(graph_dir, 'kat_stale.otrg')
    return path, K.build_stale(path)


@pytest.fixture(scope='module')
def zero(graph_dir):
    path = os.path.join(graph_dir, 'kat_zero.otrg')
    return path, K.build_zero(path)


def test_zero_length_edge_routes(zero):
    """A zero-length edge is routed as 1 mm, so every label strictly grows
    along a path and the edge-state IN gap (>= 1 mm + the smallest turn) stays a lower bound
    of any later offer: west to east crosses it straight on (route 200 m + 1 mm) and the
    matched trace follows W-J, J-J2, J2-E under the deployed turn costs."""
    path, ids = zero
    g = po.Graph(path)
    d, t, c = g.route(ids['WJ>'], 0.5, ids['J2E>'], 0.5, 1000.0, dt_sec=20, prm=po.params())
    assert abs(d - 100.001) < 0.05
    b, r = _match(path, K.zero_traces()[0], 4)
    rt = [int(e) for e in r['route_edge']]
    k = rt.index(ids['WJ>'])
    assert rt[k:k + 3] == [ids['WJ>'], ids['Z>'], ids['J2E>']]


def test_turn_cost_detour_wins(block):
    """A detour shorter than the turn penalty it avoids: eastbound at x = -10 to westbound
    at x = -40.  The U-turn at P1 is 50 m with turn cost 200 m (+ 3.663 m straight on at R):
    key 253.663 m; round the block it is 90 m with four 90-degree turns (4 x 27.067 m): key
    198.268 m.  At the auto factor (200) the longer block is the route; with no turn costs
    the 50 m U-turn is."""
    path, ids = block
    g = po.Graph(path)
    tab = po.turn_table(po.params())
    assert tab[90] == 27067 and tab[0] == 200000 and tab[180] == 3663
    d, t, c = g.route(ids['RP1>'], 0.5, ids['P0R<'], 0.25, 1000.0, dt_sec=10, prm=po.params())
    assert abs(d - 90.0) < 0.2 and c == 4 * tab[90]  # lengths from micro-degree nodes
    d0, t0, c0 = g.route(ids['RP1>'], 0.5, ids['P0R<'], 0.25, 1000.0, dt_sec=10, prm=po.params(turn_penalty_factor=0))
    assert abs(d0 - 50.0) < 0.2 and c0 == 0
    # the matched trace takes the block under turn costs, the U-turn without them
    b, r = _match(path, K.block_trace(), 10)
    rt = [int(e) for e in r['route_edge']]
    assert 0xFFFFFFFF not in rt
    assert rt[rt.index(ids['RP1>']) + 1:rt.index(ids['RP1>']) + 4] == [ids['P1Q1'], ids['Q1Q0'], ids['Q0R']]
    b, r0 = _match(path, K.block_trace(), 10, turn_penalty_factor=0)
    rt0 = [int(e) for e in r0['route_edge']]
    assert ids['P1Q1'] not in rt0 and ids['RP1<'] in rt0


def test_time_bound_prunes_during_search(bypass):
    """T1 at 0.5 -> T3 at 0.5: through the 5 km/h block 200 m in 79.2 s, round the bypass
    300 m in 21.6 s.  With a 40 s bound (probes 20 s apart) the block's labels are pruned
    while searching and the longer, faster bypass is the route; with an 80 s bound (or
    none) the block is."""
    path, ids = bypass
    g = po.Graph(path)
    prm = po.params(turn_penalty_factor=0)
    d, t, c = g.route(ids['T1>'], 0.5, ids['T3>'], 0.5, 1000.0, dt_sec=20, prm=prm)
    assert abs(d - 300.0) < 0.1 and t == 36 + 36 + 72 + 36 + 36
    d, t, c = g.route(ids['T1>'], 0.5, ids['T3>'], 0.5, 1000.0, dt_sec=40, prm=prm)
    assert abs(d - 200.0) < 0.1 and t == 792
    d, t, c = g.route(ids['T1>'], 0.5, ids['T3>'], 0.5, 1000.0, dt_sec=0, prm=prm)
    assert abs(d - 200.0) < 0.1 and t == 0
    # matched: one sub-path through the bypass
    b, r = _match(path, K.bypass_trace(), 20, turn_penalty_factor=0)
    assert r['subpath'].max() == 0
    rt = [int(e) for e in r['route_edge']]
    k = rt.index(ids['TU2'])
    assert rt[k - 1:k + 4] == [ids['T1>'], ids['TU2'], ids['U2U3'], ids['U3T'], ids['T3>']]
    assert ids['T2>'] not in rt


def test_label_setting_order_withdraws_fast_label(stale):
    """Node labels follow the search key (length), so U's label is the 90 m chain's (36 s),
    not the fast 100 m edge's (7.2 s): under a 40 s bound V (43.2 s through the chain) is out
    of reach and the transition has no route; with a 60 s bound the chain route is valid,
    and with no bound too."""
    path, ids = stale
    g = po.Graph(path)
    prm = po.params(turn_penalty_factor=0)
    assert g.route(ids['WS'], 0.97, ids['VZ'], 0.4, 2000.0, dt_sec=20, prm=prm) is None
    d, t, c = g.route(ids['WS'], 0.97, ids['VZ'], 0.4, 2000.0, dt_sec=30, prm=prm)
    assert abs(d - 233.0) < 0.1 and t == 2 + 9 * 40 + 72 + 29
    d, t, c = g.route(ids['WS'], 0.97, ids['VZ'], 0.4, 2000.0, dt_sec=0, prm=prm)
    assert abs(d - 233.0) < 0.1


# ---- GPU parity on the same inputs -----------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize('opts', [{}, {'turn_penalty_factor': 0}, {'max_route_time_factor': 0}])
def test_semantics_gpu_parity(kat, slow, square, opts):
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    path, ids, segs = kat
    M.configure(M.default_config(path, **opts))
    m = M.Matcher()
    sc = dict(K.turn_scenarios())
    sc['queue'] = K.queue_scenario()
    trs = [K.trace(p, dt=2 if n != 'straight_or_left' else 10) for n, p in sc.items()]
    trs += [K.trace(p) for p in K.scenarios().values()]
    b = K.batch(trs)
    got = m.match_batch_numpy(b)
    want = po.match_batch(po.Graph(path), b, po.params(**opts))
    errors, stats = compare(got, want)
    assert not errors, errors
    # routes whose turns decide between equal lengths: turn modes search edge states
    # (the global-memory search), the result equals the oracle either way
    qpath, qids = square
    M.configure(M.default_config(qpath, **opts))
    b = K.batch([K.trace(K.square_trace(), dt=20)])
    r = M.Matcher().match_batch(b, copy_out=True, route_work=True)
    errors, _ = compare(_lib.result_to_numpy(r), po.match_batch(po.Graph(qpath), b, po.params(**opts)))
    assert not errors, errors
    if opts.get('turn_penalty_factor', 1) != 0:
        # turn modes: the edge-state search (the first edge tier, or the 512-state one)
        assert int(r.route_tier_work[10][0]) + int(r.route_tier_work[9][0]) > 0
    spath, sid = slow
    M.configure(M.default_config(spath, **opts))
    b = K.batch([K.trace(p, dt=4) for p in K.slow_scenarios().values()])
    got = M.Matcher().match_batch_numpy(b)
    want = po.match_batch(po.Graph(spath), b, po.params(**opts))
    errors, stats = compare(got, want)
    assert not errors, errors


@pytest.mark.gpu
@pytest.mark.parametrize('opts', [{}, {'turn_penalty_factor': 0}, {'max_route_time_factor': 0}])
def test_pruning_semantics_gpu_parity(block, bypass, stale, zero, opts):
    """The graphs where the route key (length + turn cost) and the pruning during the search
    decide the answer, and a zero-length edge under turn costs: bit-exact with the oracle
    under the deployed options, without turn costs and without a time bound."""
    from reporter_amd import matcher as M
    for (path, _), trs, dt in ((block, [K.block_trace()], 10), (bypass, [K.bypass_trace()], 20),
                               (stale, K.stale_traces(), 20), (zero, K.zero_traces(), 4)):
        M.configure(M.default_config(path, **opts))
        b = K.batch([K.trace(p, dt=dt) for p in trs])
        got = M.Matcher().match_batch_numpy(b)
        want = po.match_batch(po.Graph(path), b, po.params(**opts))
        errors, stats = compare(got, want)
        assert not errors, (path, errors)


@pytest.mark.gpu
def test_withdrawn_label_never_set(stale):
    """The parallel search must never relax U with the fast edge's (non-final) label: the
    exact rounds settle U only once the chain's shorter label is final (IN criterion), so V
    is never labelled from the withdrawn offer and the first tier itself gives the oracle's
    answer (the transition from W-S has no route; the trace continues through the
    candidate on S-U) — no retry tier, no global-memory search."""
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    path, ids = stale
    M.configure(M.default_config(path, turn_penalty_factor=0))
    b = K.batch([K.trace(K.stale_traces()[0], dt=20)])
    r = M.Matcher().match_batch(b, copy_out=True, route_work=True)
    got = _lib.result_to_numpy(r)
    want = po.match_batch(po.Graph(path), b, po.params(turn_penalty_factor=0))
    errors, _ = compare(got, want)
    assert not errors, errors
    # the first tier searched (the two-search tier, slot 0, or the small / tiny tiers, 12 / 13)
    assert sum(int(r.route_tier_work[t][0]) for t in (0, 12, 13)) > 0
    for t in range(1, 10):
        assert int(r.route_tier_work[t][0]) == 0, t  # and nothing was retried
