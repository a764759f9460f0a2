"""Tile stage on CPU: the oracle restatement pinned to the reference's cull goldens and to
the product's bucketing mirror, the C-ABI line writer, and the 2-rank gloo exchange
that routes rows to their file's owner (simple_reporter.py:176-239)."""
import json
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import tiles as ot

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))
CULL = json.load(open(os.path.join(HERE, 'golden', 'cull_cases.json')))['cases']


@pytest.mark.parametrize('i', range(len(CULL)))
def test_oracle_cull_matches_reference_goldens(i):
    c = CULL[i]
    assert ot.sort_and_cull(sorted(c['lines']), c['privacy']) == c['expected']


def _oracle_workload(graph_dir, n=30, seed=5):
    from oracle import pyoracle as po
    from reporter_amd.tools import gen
    path = gen.graph_path('tiny', graph_dir)
    tr = gen.make_traces(path, n, 40, 5, 8.0, seed, t_begin=gen.T_BEGIN, t_spread=7200)
    res = po.match_batch(po.Graph(path), tr, po.params())
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    return tr, res, first, last


def _reports(res, t):
    reps = []
    for k in range(res['trace_rep_off'][t], res['trace_rep_off'][t + 1]):
        d = {'id': int(res['rep_id'][k]), 't0': float(res['rep_t0'][k]), 't1': float(res['rep_t1'][k]),
             'length': int(res['rep_length'][k]), 'queue_length': int(res['rep_queue'][k])}
        if int(res['rep_next'][k]) != ot.NO_ID:
            d['next_id'] = int(res['rep_next'][k])
        reps.append(d)
    return reps


def test_oracle_rows_match_bucketing_mirror(graph_dir):
    from reporter_amd import simple_reporter as sr
    tr, res, first, last = _oracle_workload(graph_dir)
    rows = ot.rows_from_reports(res, first, last)
    want = {}
    for t in range(tr.n_traces):
        for k, v in sr.bucket(int(first[t]), int(last[t]), _reports(res, t), 3600, 'auto', 'smpl_rprt').items():
            want.setdefault(k, []).extend(v)
    got = {}
    for r, line in zip(rows, ot.lines_of(rows)):
        got.setdefault(ot.file_name(r['file']), []).append(line)
    assert got == want and len(rows) > 0


def test_format_lines_match_oracle(graph_dir):
    from reporter_amd import simple_reporter as sr
    tr, res, first, last = _oracle_workload(graph_dir)
    rows = ot.rows_from_reports(res, first, last)
    rows = rows[np.argsort(rows['file'], kind='stable')]  # rows_to_tiles expects rows grouped by file
    tiles = sr.rows_to_tiles(rows, 3600, 'auto', 'smpl_rprt')
    want = {}
    for r, line in zip(rows, ot.lines_of(rows)):
        want.setdefault(ot.file_name(r['file']), []).append(line)
    assert tiles == want


def _store(tmp_path):
    # a FileStore rendezvous: a probed-then-released TCP port can be taken by a parallel test
    return 'file://' + str(tmp_path / 'rdzv')


def _rank(rank, world, store, graph_dir, q):
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group('gloo', init_method=store, rank=rank, world_size=world)
    from reporter_amd import simple_reporter as sr
    tr, res, first, last = _oracle_workload(graph_dir)
    # each rank holds the rows of its uuid shard (simple_reporter.py:116)
    mine = [t for t in range(tr.n_traces) if sr.shard_of(tr.uuids[t], world) == rank]
    rows = ot.rows_from_reports(res, first, last)
    per_trace = np.concatenate([[0], np.cumsum([len(ot.rows_from_reports(
        {k: (v[t:t + 2] if k == 'trace_rep_off' else v) for k, v in res.items()}, first[t:t + 1], last[t:t + 1]))
        for t in range(tr.n_traces)])])
    sel = np.concatenate([np.arange(per_trace[t], per_trace[t + 1]) for t in mine]) if mine else np.zeros(0, int)
    local = rows[sel.astype(np.int64)]
    got = sr.exchange_rows(torch.from_numpy(local.view(np.uint8).copy()), world)
    owned = got.numpy().view(ot.TILE_ROW)
    # every received row belongs here, and owners hold complete files
    assert np.all(sr.file_owner(owned['file'].astype(np.int64), world) == rank)
    q.put((rank, ot.tiles(owned, 2), len(owned)))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4, 8])
def test_row_exchange(tmp_path, graph_dir, world):
    tr, res, first, last = _oracle_workload(graph_dir)
    all_rows = ot.rows_from_reports(res, first, last)
    want = ot.tiles(all_rows, 2)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    store = _store(tmp_path)
    ps = [ctx.Process(target=_rank, args=(r, world, store, graph_dir, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    merged = {}
    for _, t, _ in outs:
        assert not (set(t) & set(merged))  # a file lives on exactly one owner
        merged.update(t)
    assert merged == want and len(want) > 0
    assert sum(n for _, _, n in outs) == len(all_rows)  # every row reached exactly one owner
    if world == 2:
        assert all(n > 0 for _, _, n in outs)


def test_java_clean_matches_python_cull_on_numeric_order():
    """AnonymisingProcessor.clean and simple_reporter's loop are the same rule: on rows
    whose ids have equal digit counts (string order == numeric order) they agree."""
    rng = np.random.default_rng(3)
    for trial in range(200):
        n = int(rng.integers(1, 14))
        rows = np.zeros(n, ot.TILE_ROW)
        rows['id'] = 8 * rng.integers(100, 104, n) + 2
        rows['next_id'] = 8 * rng.integers(100, 102, n)
        rows['duration'] = rng.integers(10, 20, n)
        rows['start'] = 1483228800 + rng.integers(0, 9, n)
        rows['end'] = rows['start'] + rows['duration']
        rows['length'] = 50
        order = np.lexsort((np.arange(n), rows['next_id'], rows['id']))
        for p in (1, 2, 3):
            kept = ot.java_clean(rows[order], p)
            pairs = [(int(r['id']), int(r['next_id'])) for r in kept]
            lines = ot.sort_and_cull(ot.lines_of(rows), p)
            want = [(int(l.split(',')[0]), int(l.split(',')[1])) for l in lines]
            assert pairs == want


def test_stream_format_matches_oracle(graph_dir):
    from reporter_amd import _lib
    from reporter_amd import simple_reporter as sr
    tr, res, first, last = _oracle_workload(graph_dir)
    rows = ot.stream_rows_from_reports(res)
    rows = rows[np.argsort(rows['file'], kind='stable')]
    got = sr.rows_to_tiles(rows, 3600, 'auto', 'reporter', rules=_lib.OTR_TILE_RULES_STREAM)
    want = {}
    for r in rows:
        want.setdefault(ot.file_name(r['file']), []).append(ot.java_line(r, 'reporter', 'auto'))
    assert got == want and len(rows) > 0
    # INVALID next ids print as an empty field (Segment.java:62-64)
    assert any(l.split(',')[1] == '' for v in got.values() for l in v)
