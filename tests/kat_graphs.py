"""Hand-built road graphs with known matching answers: straight
road, turn at a junction, one-way dual carriageway 20 m apart, disconnected roads
(breakage).  Used by the oracle known-answer tests and the GPU parity tests."""
import math
import os

import numpy as np

from reporter_amd.graphfile import write_graph
from reporter_amd.tools.gen import Traces

LAT0, LON0 = 14.55, 121.03
M = 20037581.187 / 180.0
MLON = M * math.cos(math.radians(LAT0))


def ll(x_m, y_m):
    """local metres east/north of (LAT0, LON0) → (lat, lon)"""
    return (LAT0 + y_m / M, LON0 + x_m / MLON)


def osmlr(level, tile, idx):
    return (idx << 25) | (tile << 3) | level


def two_way(edges, a, b, way, **kw):
    edges.append(dict(src=a, dst=b, way=way, **kw))
    edges.append(dict(src=b, dst=a, way=way, **kw))
    return len(edges) - 2, len(edges) - 1


def build(path):
    """Returns (new_id map, dict of named things). Layout (metres):
       main street y=0: nodes A0..A5 at x=0,100,...,500 (two-way, level 1)
       side street x=200 going north: B1 (200,100), B2 (200,200)  (two-way, level 2)
       dual carriageway at y=400 (eastbound, one-way) and y=380 (westbound), x=0..300
       island road far away at y=2000: I0..I2 (disconnected)"""
    nodes, names = [], {}

    def node(name, x, y):
        names[name] = len(nodes)
        nodes.append(ll(x, y))
    for k in range(6):
        node('A%d' % k, 100 * k, 0)
    node('B1', 200, 100)
    node('B2', 200, 200)
    for k in range(4):
        node('N%d' % k, 100 * k, 400)
        node('S%d' % k, 100 * k, 380)
    for k in range(3):
        node('I%d' % k, 100 * k, 2000)
    edges = []
    ids = {}
    for k in range(5):
        f, r = two_way(edges, names['A%d' % k], names['A%d' % (k + 1)], 10 + k // 3, level=1, speed=50)
        ids['A%d>' % k], ids['A%d<' % k] = f, r
    ids['B0^'], ids['B0v'] = two_way(edges, names['A2'], names['B1'], 20, speed=30)
    ids['B1^'], ids['B1v'] = two_way(edges, names['B1'], names['B2'], 20, speed=30)
    for k in range(3):
        edges.append(dict(src=names['N%d' % k], dst=names['N%d' % (k + 1)], way=30, speed=50, level=1))
        ids['N%d>' % k] = len(edges) - 1
        edges.append(dict(src=names['S%d' % (k + 1)], dst=names['S%d' % k], way=31, speed=50, level=1))
        ids['S%d<' % k] = len(edges) - 1
    for k in range(2):
        ids['I%d>' % k], ids['I%d<' % k] = two_way(edges, names['I%d' % k], names['I%d' % (k + 1)], 40)
    segs = [
        dict(id=osmlr(1, 100, 1), edges=[ids['A0>']]),
        dict(id=osmlr(1, 100, 2), edges=[ids['A1>'], ids['A2>']]),
        dict(id=osmlr(1, 100, 3), edges=[ids['A3>'], ids['A4>']]),
        dict(id=osmlr(1, 100, 4), edges=[ids['A4<'], ids['A3<'], ids['A2<'], ids['A1<'], ids['A0<']]),
        dict(id=osmlr(2, 200, 1), edges=[ids['B0^'], ids['B1^']]),
        dict(id=osmlr(1, 100, 5), edges=[ids['N0>'], ids['N1>'], ids['N2>']]),
        dict(id=osmlr(1, 100, 6), edges=[ids['S2<'], ids['S1<'], ids['S0<']]),
        dict(id=osmlr(2, 300, 1), edges=[ids['I0>'], ids['I1>']]),
    ]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}, {s['id']: i for i, s in enumerate(segs)}, segs


def trace(points, t0=1483228800, dt=2):
    """points: [(x_m, y_m)] every dt seconds."""
    lat = np.array([ll(x, y)[0] for x, y in points])
    lon = np.array([ll(x, y)[1] for x, y in points])
    lat = np.round(lat, 6)
    lon = np.round(lon, 6)
    tm = t0 + dt * np.arange(len(points), dtype=np.int64)
    return lat, lon, tm


def batch(traces, modes=None):
    lats, lons, tms, offs = [], [], [], [0]
    for la, lo, tm in traces:
        lats.append(la)
        lons.append(lo)
        tms.append(tm)
        offs.append(offs[-1] + len(la))
    modes = np.zeros(len(traces), np.uint8) if modes is None else np.asarray(modes, np.uint8)
    return Traces(np.concatenate(lats), np.concatenate(lons), np.concatenate(tms), np.asarray(offs, np.int64),
                  modes)


def scenarios():
    """name → list of (x,y) points, driven at 10 m/s, sampled every 2 s (20 m)."""
    s = {}
    # straight east along the main street, from x=30 to x=470, 3 m north of the centreline
    s['straight_east'] = [(30 + 20 * k, 3) for k in range(23)]
    # east to the junction at x=200, then north up the side street
    s['turn_north'] = [(40 + 20 * k, -2) for k in range(8)] + [(202, 20 + 20 * k) for k in range(9)]
    # eastbound on the north carriageway with noise pulling toward the westbound one
    s['dual_carriageway'] = [(20 + 20 * k, 393 - 2 * (k % 3)) for k in range(14)]
    # westbound on main street
    s['straight_west'] = [(480 - 20 * k, -3) for k in range(23)]
    # jump to a disconnected road → breakage into two sub-paths
    s['breakage'] = [(30 + 20 * k, 2) for k in range(6)] + [(20 + 20 * k, 2002) for k in range(6)]
    return s


def build_short_lengths(path, seed=5, n=14, spacing=40.0):
    """A street grid whose stored edge lengths undercut the geometry (as whole-metre
    rounding does: 0.6-1.0 x the straight-line length, some 0 m) and with clusters of
    nearly coincident nodes (a few cm apart): the graphs a tile flattener can produce.
    Routing must still equal plain Dijkstra (oracle)."""
    rng = np.random.default_rng(seed)
    nodes, edges, segs = [], [], []
    idx = {}
    for r in range(n):
        for c in range(n):
            idx[(r, c)] = len(nodes)
            nodes.append(ll(c * spacing + rng.uniform(-3, 3), r * spacing + rng.uniform(-3, 3)))

    def dist(a, b):
        (la1, lo1), (la2, lo2) = nodes[a], nodes[b]
        x = (lo1 - lo2) * M * math.cos(math.radians(0.5 * (la1 + la2)))
        y = (la1 - la2) * M
        return math.hypot(x, y)

    way = 1
    for r in range(n):
        for c in range(n):
            for dr, dc in ((0, 1), (1, 0)):
                if r + dr >= n or c + dc >= n:
                    continue
                a, b = idx[(r, c)], idx[(r + dr, c + dc)]
                # split the street at a node a few cm past its start (near-coincident pair)
                la, lo = nodes[a]
                lb, lob = nodes[b]
                f = rng.uniform(0.0003, 0.002)
                m = len(nodes)
                nodes.append((la + f * (lb - la), lo + f * (lob - lo)))
                for u, v in ((a, m), (m, b)):
                    d = dist(u, v)
                    k = rng.random()
                    length = 0.0 if k < 0.05 else (math.floor(d) if k < 0.6 else d * rng.uniform(0.6, 1.0))
                    for s_, t_ in ((u, v), (v, u)):
                        edges.append(dict(src=s_, dst=t_, way=way, level=2, speed=30, length=float(length)))
                segs.append(dict(id=osmlr(2, 500, len(segs) + 1), edges=[len(edges) - 4, len(edges) - 2]))
                way += 1
    write_graph(path, nodes, edges, segs)
    return path


def build_slow(path):
    """Time-bound graph: a two-way road T0..T5 at x = 0..500 m (y = 0),
    50 km/h except the block T2-T3 (x = 200..300 m), which is 5 km/h both ways."""
    nodes = [ll(100 * k, 0) for k in range(6)]
    edges, ids = [], {}
    for k in range(5):
        sp = 5 if k == 2 else 50
        ids['T%d>' % k], ids['T%d<' % k] = two_way(edges, k, k + 1, 50 + k, level=1, speed=sp)
    segs = [dict(id=osmlr(1, 400, 1), edges=[ids['T%d>' % k] for k in range(5)])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def build_square(path):
    """Equal-length alternatives (DESIGN.md §3.5 ties): W (0, -100) -> S (0, 0), then a
    diamond S-P-T / S-Q-T with P = (100, 100), Q = (-100, 100), T = (0, 200), mirror images
    in whole micro-degrees (equal lengths and times to the millimetre), then T -> N
    (100, 200) east; all two-way, 50 km/h, level 1.  The turns at S and at P / Q mirror
    each other; at T the route from Q bends 45 degrees into T-N and the one from P 135."""
    lat0, lon0 = int(round(LAT0 * 1e6)), int(round(LON0 * 1e6))
    dx, dy = int(round(100 / MLON * 1e6)), int(round(100 / M * 1e6))

    def e6(i, j):  # i, j: multiples of 100 m east / north, exact micro-degrees
        return ((lat0 + j * dy) * 1e-6, (lon0 + i * dx) * 1e-6)
    nodes = [e6(0, -1), e6(0, 0), e6(1, 1), e6(-1, 1), e6(0, 2), e6(1, 2)]
    W, S, P, Q, T, N = range(6)
    edges, ids = [], {}
    for name, a, b, way in (('WS', W, S, 71), ('SP', S, P, 72), ('PT', P, T, 73), ('SQ', S, Q, 74),
                            ('QT', Q, T, 75), ('TN', T, N, 76)):
        ids[name + '>'], ids[name + '<'] = two_way(edges, a, b, way, level=1, speed=50)
    segs = [dict(id=osmlr(1, 401, 1), edges=[ids['WS>']]), dict(id=osmlr(1, 401, 2), edges=[ids['TN>']])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def square_trace():
    """North on W-S, then east on T-N: two probes each (20 s apart)."""
    return [(2, -60), (2, -20), (40, 202), (80, 202)]


def slow_scenarios():
    """Eastbound at 12.5 m/s, a probe every 4 s (50 m), 3 m north of the centreline."""
    return {'through_slow_block': [(20 + 50 * k, 3) for k in range(10)]}


def turn_scenarios():
    """On the 'kat' graph: east along the main street, the last probe 48 m east of the side
    street (x = 200, going north) and 50 m north of the main street: nearer the side street
    (emission) but straight ahead costs one straight pass instead of a left turn."""
    return {'straight_or_left': [(50, 0), (150, 0), (248, 50)],
            # east to x = 290, turning at the node x = 300, back west to x = 60
            'u_turn': [(30 + 20 * k, -3) for k in range(14)] + [(280 - 20 * k, -3) for k in range(12)]}


def queue_scenario():
    """East on the main street at 10 m/s (a probe every 2 s) to x = 190, then 1 m/s from
    x = 201 to 319: states every 10 m in the slow part, so the slow pieces start at the
    state at x = 201 and segment A1-A3 (x = 100..300) ends 99 m later."""
    pts = [(30 + 20 * k, 3) for k in range(9)]        # x = 30..190, t = 0..16 s
    pts += [(201 + 2 * m, 3) for m in range(60)]      # x = 201..319, t = 18..136 s
    return pts


def build_block(path):
    """Turn costs against length (the route key is length + turn cost): a
    two-way main street y = 0 with nodes P0 (-100, 0), R (-20, 0), P1 (0, 0), P2 (100, 0)
    and a one-way block north of it, P1 -> Q1 (0, 20) -> Q0 (-20, 20) -> R, all 50 km/h,
    level 1.  Eastbound at x = -10 to westbound at x = -40: the U-turn at P1 is 50 m long
    with a 200 m turn (auto), the block is 90 m long with four 90-degree turns (4 x 27.067
    m): under turn costs the longer block wins."""
    nodes = [ll(-100, 0), ll(-20, 0), ll(0, 0), ll(100, 0), ll(0, 20), ll(-20, 20)]
    P0, R, P1, P2, Q1, Q0 = range(6)
    edges, ids = [], {}
    ids['P0R>'], ids['P0R<'] = two_way(edges, P0, R, 81, level=1, speed=50)
    ids['RP1>'], ids['RP1<'] = two_way(edges, R, P1, 81, level=1, speed=50)
    ids['P1P2>'], ids['P1P2<'] = two_way(edges, P1, P2, 81, level=1, speed=50)
    for name, a, b in (('P1Q1', P1, Q1), ('Q1Q0', Q1, Q0), ('Q0R', Q0, R)):
        edges.append(dict(src=a, dst=b, way=82, level=1, speed=50))
        ids[name] = len(edges) - 1
    segs = [dict(id=osmlr(1, 402, 1), edges=[ids['P0R>'], ids['RP1>'], ids['P1P2>']]),
            dict(id=osmlr(1, 402, 2), edges=[ids['P1P2<'], ids['RP1<'], ids['P0R<']])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def block_trace():
    """East past x = -10, then west at x = -40 (10 s apart: 90 m at 50 km/h is 6.5 s)."""
    return [(-60, 2), (-10, 2), (-40, -2), (-80, -2)]


def build_bypass(path):
    """The time bound during the search: the road T0..T5 of build_slow
    (the block T2-T3 at 5 km/h) plus a 50 km/h bypass T2 -> U2 (200, 50) -> U3 (300, 50)
    -> T3 (one-way).  T1 at 0.5 -> T3 at 0.5 with a 40 s bound: the 200 m route through the
    block takes 79.2 s and is pruned, the 300 m bypass (21.6 s) is the route."""
    nodes = [ll(100 * k, 0) for k in range(6)] + [ll(200, 50), ll(300, 50)]
    edges, ids = [], {}
    for k in range(5):
        sp = 5 if k == 2 else 50
        ids['T%d>' % k], ids['T%d<' % k] = two_way(edges, k, k + 1, 50 + k, level=1, speed=sp)
    for name, a, b in (('TU2', 2, 6), ('U2U3', 6, 7), ('U3T', 7, 3)):
        edges.append(dict(src=a, dst=b, way=59, level=1, speed=50))
        ids[name] = len(edges) - 1
    segs = [dict(id=osmlr(1, 403, 1), edges=[ids['T%d>' % k] for k in range(5)])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def bypass_trace():
    """Eastbound at 15 m/s on the fast road, a probe every 20 s (x = 50, 150, 350, 450):
    the step from x = 150 to x = 350 is only routable through the bypass."""
    return [(50, 3), (150, 3), (350, 3), (450, 3)]


def build_stale(path):
    """A label the parallel search sets early and must withdraw: from S
    (0, 0) to U (90, 0) a single 50 km/h edge whose stored length is 100 m (7.2 s), and a
    chain of nine 10 m edges along the same line at 9 km/h (90 m, 36 s).  U -> V (190, 0)
    is 100 m at 50 km/h (7.2 s), V -> Z (290, 0) continues.  Under a 40 s bound U's label
    is the chain's (shorter) one, so V is out of time reach (43.2 s): a search that
    relaxed U with the fast edge's label first must not keep V's label from it.  The
    source road W (-100, 0) -> S, and a second road Y (0, -100) -> S so that candidates near
    S share the search root with different exit times."""
    nodes = [ll(0, 0), ll(90, 0), ll(190, 0), ll(290, 0), ll(-100, 0), ll(0, -100)]
    S, U, V, Z, W, Y = range(6)
    chain = []
    for k in range(1, 9):
        chain.append(len(nodes))
        nodes.append(ll(10 * k, 0.0))
    edges, ids = [], {}

    def one(name, a, b, **kw):
        edges.append(dict(src=a, dst=b, way=90 + len(ids), level=1, **kw))
        ids[name] = len(edges) - 1
    one('WS', W, S, speed=50)
    one('YS', Y, S, speed=50)
    one('SU', S, U, speed=50, length=100.0)
    seq = [S] + chain + [U]
    for k in range(9):
        one('C%d' % k, seq[k], seq[k + 1], speed=9, length=10.0)
    one('UV', U, V, speed=50)
    one('VZ', V, Z, speed=50)
    segs = [dict(id=osmlr(1, 404, 1), edges=[ids['UV'], ids['VZ']])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def stale_traces():
    """Probes 20 s apart: near S on W-S (and near the Y-S road), then on V-Z."""
    return [[(-60, 2), (-3, 3), (230, 2), (270, 2)],
            [(-60, 2), (-5, -2), (210, 2), (250, 2)]]


def build_zero(path):
    """A zero-length edge under turn costs (the edge-state IN criterion's gap):
    a junction split in two nodes at the same point, J (0, 0) and J2 (0, 0), joined by a
    two-way edge of stored length 0 (routing length 1 mm; heading 0 from
    its degenerate shape).  W (-100, 0) - J - J2 - E (100, 0) is the main street, J - N
    (0, 100) and J2 - S (0, -100) the side streets, all two-way 50 km/h level 1.  Routes
    cross J -> J2 with the turns into and out of the zero-length edge, and a U-turn at J2
    or J offers to the zero-length state again through the smallest turn."""
    nodes = [ll(-100, 0), ll(0, 0), ll(0, 0), ll(100, 0), ll(0, 100), ll(0, -100)]
    W, J, J2, E, N, S = range(6)
    edges, ids = [], {}
    ids['WJ>'], ids['WJ<'] = two_way(edges, W, J, 71, level=1, speed=50)
    ids['Z>'], ids['Z<'] = two_way(edges, J, J2, 72, level=1, speed=50, length=0.0)
    ids['J2E>'], ids['J2E<'] = two_way(edges, J2, E, 73, level=1, speed=50)
    ids['JN>'], ids['JN<'] = two_way(edges, J, N, 74, level=1, speed=50)
    ids['J2S>'], ids['J2S<'] = two_way(edges, J2, S, 75, level=1, speed=50)
    segs = [dict(id=osmlr(1, 405, 1), edges=[ids['WJ>'], ids['Z>'], ids['J2E>']]),
            dict(id=osmlr(1, 405, 2), edges=[ids['J2E<'], ids['Z<'], ids['WJ<']])]
    new = write_graph(path, nodes, edges, segs)
    return {k: int(new[v]) for k, v in ids.items()}


def zero_traces():
    """Across the split junction: west to east, west to south, north to east, and east to
    north (through the zero-length edge the other way)."""
    return [[(-80, 2), (-30, 2), (30, 2), (80, 2)],
            [(-80, 2), (-30, 2), (2, -30), (2, -80)],
            [(2, 80), (2, 30), (30, -2), (80, -2)],
            [(80, -2), (30, -2), (-2, 30), (-2, 80)]]
