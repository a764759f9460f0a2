"""Keyed speed histogram on the GPU (otr_hist_reduce) vs the CPU
restatement oracle/hist.py: device tile rows (K9) sort-reduced by (file, id, next_id,
speed bin), pair cull at privacy p; entries merged across inputs (the owner's side of
the exchange); the single-GPU end of the exchange (all entries owned by rank 0)."""
import numpy as np
import pytest

from oracle import hist as oh
from oracle import pyoracle as po
from oracle import tiles as ot
from reporter_amd import _lib
from reporter_amd import matcher as M
from reporter_amd import simple_reporter as sr
from reporter_amd.tools import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def city(graph_dir):
    path = gen.graph_path('city', graph_dir)
    M.configure(M.default_config(path))
    return path


@pytest.fixture(scope='module')
def workload(city):
    tr = gen.make_traces(city, 160, 120, 10, 8.0, 47, t_begin=gen.T_BEGIN, t_spread=3 * 3600)
    want = po.match_batch(po.Graph(city), tr, po.params(), threads=8)
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    return tr, ot.rows_from_reports(want, first, last)


@pytest.mark.parametrize('privacy', [1, 2, 3])
def test_device_rows_reduce_equals_oracle(workload, privacy):
    tr, rows = workload
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=False, tile_rows=True)
    assert int(r.n_rows) == len(rows) > 100
    got = sr.hist_reduce(m, r.d_rows, r.n_rows, privacy=privacy, rows_in=True)
    want = oh.reduce(oh.entries_from_rows(rows), privacy)
    assert len(want) > 0
    assert np.array_equal(got, want)
    if privacy == 1:
        assert int(got['count'].sum()) == len(rows)


def test_entries_merge_equals_oracle(workload):
    """The owner's merge: two partial reductions concatenated (host input) reduce to the
    reduction of the whole; then with privacy the pair cull applies to merged totals."""
    tr, rows = workload
    m = M.Matcher()
    half = len(rows) // 2
    a = sr.hist_reduce(m, rows[:half], half, rows_in=True, memory='host')
    b = sr.hist_reduce(m, rows[half:], len(rows) - half, rows_in=True, memory='host')
    both = np.concatenate([a, b])
    for p in (1, 2, 4):
        got = sr.hist_reduce(m, both, len(both), privacy=p, memory='host')
        assert np.array_equal(got, oh.reduce(oh.entries_from_rows(rows), p))


def test_device_output_and_edge_cases(workload):
    import torch
    tr, rows = workload
    m = M.Matcher()
    e = oh.entries_from_rows(rows)
    src = torch.from_numpy(e.view(np.uint8).copy()).cuda()
    out = torch.zeros(len(e) * _lib.HIST_ENTRY.itemsize, dtype=torch.uint8, device='cuda')
    n = sr.hist_reduce(m, src.data_ptr(), len(e), privacy=2, out=out.data_ptr())
    got = out[:n * _lib.HIST_ENTRY.itemsize].cpu().numpy().view(_lib.HIST_ENTRY)
    assert np.array_equal(got, oh.reduce(e, 2))
    # empty input; one entry; a count that saturates the u32 field
    assert len(sr.hist_reduce(m, e[:0], 0, memory='host')) == 0
    assert np.array_equal(sr.hist_reduce(m, e[:1], 1, memory='host'), oh.reduce(e[:1]))
    big = np.repeat(e[:1], 3)
    big['count'] = 0x7FFFFFFF
    assert np.array_equal(sr.hist_reduce(m, big, 3, memory='host'), oh.reduce(big))
    assert int(oh.reduce(big)['count'][0]) == 0xFFFFFFFF


def test_owner_cull_trailing_singleton_equals_reference_loop(workload):
    """The owner cull on crafted files (tests/test_hist_cull_cpu.py CRAFTED: trailing single-line
    runs, string order != numeric order) on the device: the oracle's entries, and the pairs and
    line counts the reference loop keeps (oracle/tiles.sort_and_cull)."""
    from tests.test_hist_cull_cpu import CRAFTED, _pairs_from_entries, _pairs_from_lines, _rows
    m = M.Matcher()
    rows = _rows(CRAFTED)
    for p in (2, 3):
        got = sr.hist_reduce(m, rows, len(rows), privacy=p, rows_in=True, memory='host')
        assert np.array_equal(got, oh.reduce(oh.entries_from_rows(rows), p))
        assert _pairs_from_entries(got) == _pairs_from_lines(rows, p)
