"""Tile stage on the GPU (K9 rows, K10 sort + cull) vs the CPU restatement of
simple_reporter.py:176-239, through the C-ABI."""
import numpy as np
import pytest

from oracle import pyoracle as po
from oracle import tiles as ot
from reporter_amd import _lib
from reporter_amd import matcher as M
from reporter_amd import simple_reporter as sr
from reporter_amd.tools import gen

pytestmark = pytest.mark.gpu


class _DevArr:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {'shape': (nbytes,), 'typestr': '|u1', 'data': (int(ptr), False),
                                         'version': 2}


@pytest.fixture(scope='module')
def city(graph_dir):
    path = gen.graph_path('city', graph_dir)
    M.configure(M.default_config(path))
    return path


@pytest.fixture(scope='module')
def workload(city):
    tr = gen.make_traces(city, 120, 120, 10, 8.0, 31, t_begin=gen.T_BEGIN, t_spread=3 * 3600)
    want = po.match_batch(po.Graph(city), tr, po.params(), threads=8)
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    return tr, ot.rows_from_reports(want, first, last)


def _device_rows(m, tr):
    import torch
    r = m.match_batch(tr, copy_out=False, tile_rows=True)
    n = int(r.n_rows)
    w = _lib.TILE_ROW.itemsize
    buf = torch.as_tensor(_DevArr(r.d_rows, n * w), device='cuda').clone().cpu().numpy()
    return r, buf.view(_lib.TILE_ROW)


def test_device_rows_equal_restatement(workload):
    tr, want = workload
    m = M.Matcher()
    _, got = _device_rows(m, tr)
    assert len(got) == len(want) > 100
    assert np.array_equal(got, want)


@pytest.mark.parametrize('privacy', [1, 2, 3, 5])
def test_device_cull_equals_restatement(workload, privacy):
    tr, want_rows = workload
    m = M.Matcher()
    r, _ = _device_rows(m, tr)
    kept = sr.cull_rows(m, None, privacy, device_ptr=r.d_rows, n=r.n_rows)
    assert sr.rows_to_tiles(kept) == ot.tiles(want_rows, privacy)


def _crafted():
    """Runs whose string order differs from numeric order (12 vs 123, 9 vs 10), trailing
    singletons, equal lines, one-row files, INVALID next ids."""
    rng = np.random.default_rng(7)
    rows = []
    ids = [12, 123, 1234, 9, 10, 100, 99, 7, 70, 700]
    for f in range(40):
        file = ((412008 + f % 3) << 25) | ((f % 3) << 22) | (f * 37)
        n = int(rng.integers(1, 12))
        for _ in range(n):
            sid = int(rng.choice(ids)) * 8 + f % 3
            nx = ot.INVALID_SEGMENT_ID if rng.random() < 0.2 else int(rng.choice(ids)) * 8
            st = 1483228800 + int(rng.integers(0, 5000))
            du = int(rng.choice([1, 9, 10, 11, 100]))
            rows.append((file, sid, nx, st, st + du, du, int(rng.choice([5, 50, 500])), 0, 0))
    return np.array(rows, dtype=ot.TILE_ROW)


@pytest.mark.parametrize('privacy', [1, 2, 3])
def test_crafted_order_and_quirk(privacy):
    rows = _crafted()
    m = M.Matcher()
    kept = sr.cull_rows(m, rows, privacy)
    assert sr.rows_to_tiles(kept) == ot.tiles(rows, privacy)


def test_cull_edge_sizes():
    m = M.Matcher()
    assert len(sr.cull_rows(m, np.zeros(0, ot.TILE_ROW), 2)) == 0
    one = _crafted()[:1]
    assert len(sr.cull_rows(m, one, 2)) == 0 and len(sr.cull_rows(m, one, 1)) == 1


def test_report_tiles_device_equals_host_path(city):
    tr = gen.make_traces(city, 60, 150, 5, 8.0, 32, t_begin=gen.T_BEGIN, t_spread=2 * 3600)
    m = M.Matcher()
    want = sr.report_tiles(sr.match_traces(m, tr), 2)
    got = sr.report_tiles_device(m, tr, 2)
    assert got == want and len(got) > 0
    assert sr.report(m, tr, 2) == want  # (the module's product entry point: the device path)


@pytest.fixture(scope='module')
def stream_workload(city):
    tr = gen.make_traces(city, 120, 120, 10, 8.0, 33, t_begin=gen.T_BEGIN, t_spread=3 * 3600)
    want = po.match_batch(po.Graph(city), tr, po.params(), threads=8)
    return tr, ot.stream_rows_from_reports(want)


def test_stream_rows_equal_restatement(stream_workload):
    import torch
    tr, want = stream_workload
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=False, tile_rows=True, tile_rules=_lib.OTR_TILE_RULES_STREAM)
    w = _lib.TILE_ROW.itemsize
    got = torch.as_tensor(_DevArr(r.d_rows, int(r.n_rows) * w), device='cuda').clone().cpu().numpy()
    got = got.view(_lib.TILE_ROW)
    assert len(got) == len(want) > 100
    assert np.array_equal(got, want)


@pytest.mark.parametrize('privacy', [1, 2, 3])
def test_stream_cull_equals_restatement(stream_workload, privacy):
    tr, want_rows = stream_workload
    m = M.Matcher()
    got = sr.stream_tiles_device(m, tr, privacy, source='reporter')
    assert got == ot.stream_tiles(want_rows, privacy, source='reporter')
