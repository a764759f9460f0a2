"""N>1 path on CPU: world_size-2, -4 and -8 gloo ranks shard traces by uuid hash
(simple_reporter.py:116), each matches its shard (CPU oracle stands in for the GPU
here), builds the [hour][segment][speed] histogram, and the cross-rank combine
(all-reduce-sum then owner slice, the gloo analogue of the RCCL reduce-scatter in
bench.py) equals the single-process histogram of the whole set."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _store(tmp_path):
    # a FileStore rendezvous: a probed-then-released TCP port can be taken by a parallel test
    return 'file://' + str(tmp_path / 'rdzv')


def _workload(graph_dir):
    from reporter_amd.tools import gen
    path = gen.graph_path('tiny', graph_dir)
    tr = gen.make_traces(path, 40, 30, 5, 8.0, 5, t_begin=gen.T_BEGIN, t_spread=1800)
    return path, tr


def _hist_for(path, tr):
    from oracle import pyoracle as po
    from oracle.hist import histogram
    from reporter_amd.graphfile import GraphFile
    G = GraphFile(path)
    idx = {int(s): i for i, s in enumerate(G.seg_id)}
    r = po.match_batch(po.Graph(path), tr, po.params())
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    return histogram(r, first, last, idx, len(G.seg_id), __import__('reporter_amd.tools.gen').tools.gen.T_BEGIN, 2)


def _rank(rank, world, store, graph_dir, out):
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group('gloo', init_method=store, rank=rank, world_size=world)
    from reporter_amd import simple_reporter as sr
    path, tr = _workload(graph_dir)
    mine = np.array([i for i, u in enumerate(tr.uuids) if sr.shard_of(u, world) == rank])
    h, rows = _hist_for(path, tr.subset(mine))
    t = torch.from_numpy(h.reshape(-1).copy())
    pad = (-t.numel()) % world
    t = torch.cat([t, torch.zeros(pad, dtype=t.dtype)])
    dist.all_reduce(t)                       # gloo: reduce-scatter = all-reduce + owner slice
    n = t.numel() // world
    own = t[rank * n:(rank + 1) * n].clone()
    gathered = [torch.zeros_like(own) for _ in range(world)]
    dist.all_gather(gathered, own)
    cnt = torch.tensor([len(mine)])
    dist.all_reduce(cnt)
    if rank == 0:
        np.save(out, torch.cat(gathered)[:h.size].numpy())
        np.save(out + '.cnt.npy', cnt.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4, 8])
def test_shard_and_combine(tmp_path, graph_dir, world):
    out = str(tmp_path / 'hist.npy')
    mp.spawn(_rank, args=(world, _store(tmp_path), graph_dir, out), nprocs=world, join=True)
    path, tr = _workload(graph_dir)
    whole, rows = _hist_for(path, tr)
    combined = np.load(out)
    assert int(np.load(out + '.cnt.npy')[0]) == tr.n_traces  # shards partition the traces
    assert rows > 0 and whole.sum() > 0
    assert np.array_equal(combined, whole.reshape(-1))


def _entries_for(path, tr):
    """Oracle match → tile rows (simple_reporter.py:176-196) → keyed entries, reduced
    locally (the CPU stands in for the GPU's otr_hist_reduce here)."""
    from oracle import pyoracle as po
    from oracle import hist, tiles
    r = po.match_batch(po.Graph(path), tr, po.params())
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    rows = tiles.rows_from_reports(r, first, last)
    return hist.reduce(hist.entries_from_rows(rows), 1), rows


def _keyed_rank(rank, world, store, graph_dir, out, privacy):
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group('gloo', init_method=store, rank=rank, world_size=world)
    from oracle import hist
    from reporter_amd import simple_reporter as sr
    path, tr = _workload(graph_dir)
    mine = np.array([i for i, u in enumerate(tr.uuids) if sr.shard_of(u, world) == rank])
    local, _ = _entries_for(path, tr.subset(mine))
    got = sr.exchange_hist(torch.from_numpy(local.view(np.uint8).copy()), world)
    recv = got.numpy().view(hist.HIST_ENTRY)
    owned = hist.reduce(recv, privacy)  # the owner's merge + cull
    ok = bool(np.all(hist.owner_of(recv['file'], world) == rank))
    # gather every owner's result on rank 0 (sizes first: gloo all_gather needs equal shapes)
    n = torch.tensor([len(owned)])
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = max(int(x) for x in ns)
    buf = torch.zeros(m * hist.HIST_ENTRY.itemsize, dtype=torch.uint8)
    buf[:len(owned) * hist.HIST_ENTRY.itemsize] = torch.from_numpy(owned.view(np.uint8).copy())
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    oks = torch.tensor([int(ok)])
    dist.all_reduce(oks)
    if rank == 0:
        parts = [b.numpy()[:int(k) * hist.HIST_ENTRY.itemsize].view(hist.HIST_ENTRY) for b, k in zip(bufs, ns)]
        np.save(out, np.concatenate(parts))
        np.save(out + '.ok.npy', oks.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize('world,privacy', [(2, 1), (2, 2), (4, 2), (8, 1), (8, 2)])
def test_keyed_histogram_exchange(tmp_path, graph_dir, world, privacy):
    """§8e keyed exchange: per-rank (file, pair, speed bin) entries → all-to-all by the
    (hour, tile) owner → owner reduce + pair cull; the owners' union equals the
    single-process reduction of the whole set, and every entry reached its owner (at
    N = 8 some owners receive no entry at all)."""
    from oracle import hist
    out = str(tmp_path / 'keyed.npy')
    mp.spawn(_keyed_rank, args=(world, _store(tmp_path), graph_dir, out, privacy), nprocs=world, join=True)
    path, tr = _workload(graph_dir)
    _, rows = _entries_for(path, tr)
    whole = hist.reduce(hist.entries_from_rows(rows), privacy)
    got = np.load(out)
    assert int(np.load(out + '.ok.npy')[0]) == world
    assert len(whole) > 0 and int(whole['count'].sum()) > 0
    order = np.lexsort((got['speed_bin'], got['next_id'], got['id'], got['file']))
    assert np.array_equal(got[order], whole)
