"""GPU tests of the drop-in entry points and the device tail stages, through the C-ABI."""
import json

import numpy as np
import pytest

from oracle import pyoracle as po
from oracle.hist import histogram
from reporter_amd import matcher as M
from reporter_amd.graphfile import GraphFile
from reporter_amd.tools import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def city(graph_dir):
    path = gen.graph_path('city', graph_dir)
    M.configure(M.default_config(path))
    return path


def _trace_json(tr, t, report_levels=(0, 1), transition_levels=(0, 1), mode='auto', extra=None):
    a, b = tr.offsets[t], tr.offsets[t + 1]
    pts = [{'lat': float(tr.lat[i]), 'lon': float(tr.lon[i]), 'time': int(tr.time[i])} for i in range(a, b)]
    mo = {'mode': mode, 'report_levels': list(report_levels), 'transition_levels': list(transition_levels)}
    mo.update(extra or {})
    return json.dumps({'uuid': 'veh%07d' % t, 'trace': pts, 'match_options': mo}, separators=(',', ':'))


def test_valhalla_shim_match(city):
    from reporter_amd import valhalla
    sm = valhalla.SegmentMatcher()
    tr = gen.make_traces(city, 3, 60, 2, 5.0, 11)
    want = po.match_batch(po.Graph(city), tr, po.params())
    for t in range(3):
        out = json.loads(sm.Match(_trace_json(tr, t)))
        a, b = want['trace_seg_off'][t], want['trace_seg_off'][t + 1]
        assert len(out['segments']) == b - a
        for k, s in enumerate(out['segments']):
            sid = int(want['seg_id'][a + k])
            assert s.get('segment_id') == (None if sid == po.NO_ID else sid)
            assert s['start_time'] == want['seg_start'][a + k]
            assert s['end_time'] == want['seg_end'][a + k]
            assert s['length'] == want['seg_length'][a + k]
            assert s['begin_shape_index'] == want['seg_begin_shape'][a + k]


def test_report_endpoint_matches_report_of_match(city):
    """otr_report (one call) == report(json.loads(Match(json))) (reporter_service.py:240-243)."""
    from reporter_amd import reporter_service as rs
    from reporter_amd import valhalla
    sm = valhalla.SegmentMatcher()
    tr = gen.make_traces(city, 4, 80, 3, 6.0, 12)
    for t in range(4):
        body = _trace_json(tr, t)
        code, out = rs.handle_request(body)
        assert code == 200, out
        got = json.loads(out)
        match = json.loads(sm.Match(body))
        want = rs.report(match, json.loads(body), 15, {0, 1}, {0, 1})
        assert got['datastore'] == want['datastore']
        assert got['stats'] == want['stats']
        assert got.get('shape_used') == want.get('shape_used')
        assert got['segment_matcher']['mode'] == 'auto'


def test_match_options_override(city):
    """per-request match_options (generate_test_trace.py:44-52) change the search radius"""
    m = M.Matcher()
    tr = gen.make_traces(city, 1, 30, 15, 40.0, 13)
    a = json.loads(m.match_json(_trace_json(tr, 0, extra={'search_radius': 10, 'max_search_radius': 10})))
    b = json.loads(m.match_json(_trace_json(tr, 0, extra={'search_radius': 100, 'max_search_radius': 100})))
    assert len(b['segments']) >= 1
    assert a != b


def test_device_histogram_matches_restatement(city):
    m = M.Matcher()
    tr = gen.make_traces(city, 200, 100, 15, 10.0, 14, t_begin=gen.T_BEGIN, t_spread=1800)
    G = GraphFile(city)
    r = m.match_batch(tr, hist_hours=3, hist_base_time=gen.T_BEGIN, copy_out=True)
    import ctypes
    from reporter_amd import _lib
    res = _lib.result_to_numpy(r)
    import torch
    n = int(r.hist_len)
    dev = torch.empty(n, dtype=torch.int32, device='cuda')
    torch.cuda.synchronize()
    # copy the library-owned device histogram via a HIP memcpy through torch
    src = torch.as_tensor(_DevArr(r.d_hist, n), device='cuda')
    dev.copy_(src)
    torch.cuda.synchronize()
    got = dev.cpu().numpy().reshape(3, len(G.seg_id), _lib.HIST_BINS)
    idx = {int(s): i for i, s in enumerate(G.seg_id)}
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    want, rows = histogram(res, first, last, idx, len(G.seg_id), gen.T_BEGIN, 3)
    assert rows == res['n_rows'] and rows > 0
    assert np.array_equal(got, want)


class _DevArr:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {'shape': (n,), 'typestr': '<i4', 'data': (int(ptr), False),
                                         'version': 2}


def test_simple_reporter_end_to_end(city):
    """windows → one batched match → hour buckets → cull, vs the same rules applied to
    the oracle's reports."""
    from reporter_amd import simple_reporter as sr
    m = M.Matcher()
    tr = gen.make_traces(city, 50, 120, 10, 8.0, 15, t_begin=gen.T_BEGIN, t_spread=3600)
    tiles = sr.match_traces(m, tr)
    want = po.match_batch(po.Graph(city), tr, po.params())
    wt = {}
    for t in range(tr.n_traces):
        reps = []
        for k in range(want['trace_rep_off'][t], want['trace_rep_off'][t + 1]):
            d = {'id': int(want['rep_id'][k]), 't0': float(want['rep_t0'][k]), 't1': float(want['rep_t1'][k]),
                 'length': int(want['rep_length'][k]), 'queue_length': int(want['rep_queue'][k])}
            if int(want['rep_next'][k]) != po.NO_ID:
                d['next_id'] = int(want['rep_next'][k])
            reps.append(d)
        a, b = tr.offsets[t], tr.offsets[t + 1]
        for key, rows in sr.bucket(int(tr.time[a]), int(tr.time[b - 1]), reps, 3600, 'auto', 'smpl_rprt').items():
            wt.setdefault(key, []).extend(rows)
    assert tiles == wt and len(tiles) > 0
    culled = sr.report_tiles(tiles, 2)
    assert sum(len(v) for v in culled.values()) <= sum(len(v) for v in tiles.values())


def _mixed_bodies(city):
    """Bodies a batching caller would hold: several option groups, modes and invalid
    requests interleaved."""
    tr = gen.make_traces(city, 36, 60, 5, 8.0, 21, 0.2, 0.1)
    bodies = []
    for t in range(tr.n_traces):
        mode = ['auto', 'bicycle', 'pedestrian'][int(tr.mode[t])]
        if t % 9 == 4:
            bodies.append(_trace_json(tr, t, report_levels=(0,), transition_levels=(0, 1, 2), mode=mode))
        elif t % 9 == 7:
            bodies.append(_trace_json(tr, t, mode=mode, extra={'sigma_z': 6.5, 'search_radius': 40}))
        else:
            bodies.append(_trace_json(tr, t, mode=mode))
        if t % 10 == 3:
            bodies.append('{"uuid":"x","trace":[{"lat":1,"lon":2,"time":3}]}')
        if t % 10 == 6:
            bodies.append(_trace_json(tr, t).replace('"time"', '"tim"', 1))
    return bodies


def test_report_batch_equals_single(city):
    """otr_report_batch: the same bytes as otr_report, body by body, across option groups."""
    m = M.Matcher()
    bodies = _mixed_bodies(city)
    single = [m.report_json(b) for b in bodies]
    batch = m.report_json_batch(bodies)
    assert batch == single
    codes = [c for c, _ in batch]
    assert codes.count(200) >= 30 and 400 in codes and 500 in codes


def test_coalesced_threads_equal_single(city):
    """otr_coalesce: concurrent otr_report calls from many threads share device batches
    and each caller receives exactly its uncoalesced response."""
    import threading
    bodies = _mixed_bodies(city)
    m = M.Matcher()
    want = [m.report_json(b) for b in bodies]
    got = [None] * len(bodies)
    M.coalesce(16, 20000)
    try:
        def worker(k):
            mk = M.Matcher()
            for i in range(k, len(bodies), 6):
                got[i] = mk.report_json(bodies[i])
        th = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
    finally:
        M.coalesce(0)
    assert got == want
