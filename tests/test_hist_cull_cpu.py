"""The keyed histogram's owner-side privacy cull is the reference loop's (simple_reporter.py:
218-239, SURVEY §8e "apply the cull in sorted order, including the trailing-singleton
quirk").  oracle/hist.reduce culls (file, id, next_id, speed bin) entries; oracle/tiles.
sort_and_cull is the reference loop restated line for line on the same rows' text (pinned by
tests/golden/cull_cases.json).  Both must keep the same pairs with the same line counts:
on random files here, and — through the real keyed exchange (simple_reporter.exchange_hist,
gloo, world 2) — on crafted files whose trailing run is a singleton."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import hist, tiles

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(spec):
    """spec: list of (bucket, segment id, next id, speed bin, n lines) -> tile rows."""
    out = []
    for b, sid, nx, sb, n in spec:
        f = (b << 25) | ((sid & 7) << 22) | ((sid >> 3) & 0x3FFFFF)
        for k in range(n):
            out.append((f, sid, nx, b * 3600 + k, b * 3600 + k + 30, 30, 300, 0, sb))
    return np.array(out, dtype=tiles.TILE_ROW) if out else np.zeros(0, tiles.TILE_ROW)


def _pairs_from_lines(rows, privacy):
    """kept (file, id, next_id) -> line count, by the reference loop on each file's lines"""
    by_file = {}
    for r, line in zip(rows, tiles.lines_of(rows)):
        by_file.setdefault(int(r['file']), []).append(line)
    out = {}
    for f, lines in by_file.items():
        for line in tiles.sort_and_cull(lines, privacy):
            x = line.split(',')
            k = (f, int(x[0]), int(x[1]))
            out[k] = out.get(k, 0) + 1
    return out


def _pairs_from_entries(e):
    out = {}
    for f, i, n, c in zip(e['file'].tolist(), e['id'].tolist(), e['next_id'].tolist(), e['count'].tolist()):
        out[(f, i, n)] = out.get((f, i, n), 0) + c
    return out


# segments of one tile (5, level 0: one file per hour) whose ids' decimal strings sort
# differently from their values: indices 1, 2, 3, 30 give 33554472 < 67108904 < 100663336 <
# 1006633000 but '1006633000,' < '100663336,' < '33554472,' < '67108904,', so the string-last
# run of a file is not its numeric-last one
IDS = [(k << 25) | (5 << 3) for k in (1, 2, 3, 30)]


@pytest.mark.parametrize('seed', range(40))
def test_keyed_cull_equals_reference_loop(seed):
    rng = np.random.default_rng(seed)
    spec = []
    for b in range(int(rng.integers(1, 4))):
        for _ in range(int(rng.integers(1, 7))):
            sid = int(rng.choice(IDS)) + int(rng.integers(0, 2))  # levels 0 / 1: different files
            nx = int(rng.choice(IDS + [tiles.INVALID_SEGMENT_ID]))
            spec.append((b, sid, nx, int(rng.integers(0, 8)), int(rng.choice([1, 1, 1, 2, 3]))))
    rows = _rows(spec)
    rows = rows[rng.permutation(len(rows))]
    for privacy in (1, 2, 3):
        want = _pairs_from_lines(rows, privacy)
        got = _pairs_from_entries(hist.reduce(hist.entries_from_rows(rows), privacy))
        assert got == want, (privacy, spec)


def test_trailing_singleton_cases():
    a, b = IDS[1], IDS[2]  # '100663336,' < '67108904,' in string order: b's run is first, a's last
    inv = tiles.INVALID_SEGMENT_ID
    # [B, A] (a file with two single-line runs): the trailing one is judged with the one
    # before it — 2 lines >= 2, both kept; [B, B, A]: both kept; [A] alone: culled
    for spec, kept in [([(0, b, inv, 1, 1), (0, a, inv, 2, 1)], 2), ([(0, b, inv, 1, 2), (0, a, inv, 3, 1)], 2),
                       ([(0, a, inv, 1, 1)], 0), ([(0, a, b, 1, 1), (0, a, inv, 1, 1), (0, b, a, 1, 1)], 2)]:
        rows = _rows(spec)
        got = _pairs_from_entries(hist.reduce(hist.entries_from_rows(rows), 2))
        assert got == _pairs_from_lines(rows, 2)
        assert len(got) == kept, (spec, got)


def _store(tmp_path):
    return 'file://' + str(tmp_path / 'rdzv')


# crafted files: [A, B] (both kept at privacy 2 by the quirk), [A, A, B], [A] (culled), and
# a file whose string order differs from its numeric order, spread over two hours and
# two levels so both owners receive files
CRAFTED = [(0, IDS[0], IDS[1], 1, 1), (0, IDS[1], IDS[0], 2, 1),
           (1, IDS[0], IDS[1], 1, 2), (1, IDS[1], IDS[0], 3, 1),
           (2, IDS[2], IDS[3], 4, 1),
           (3, IDS[3] + 1, IDS[2], 1, 1), (3, IDS[2] + 1, IDS[3], 1, 1), (3, IDS[0] + 1, IDS[2], 2, 3),
           (4, IDS[2] + 1, IDS[0], 1, 2), (4, IDS[1] + 1, IDS[0], 1, 1), (4, IDS[3] + 1, IDS[0], 5, 1)]


def _crafted_rank(rank, world, store, out, privacy):
    import sys
    sys.path.insert(0, ROOT)
    dist.init_process_group('gloo', init_method=store, rank=rank, world_size=world)
    from reporter_amd import simple_reporter as sr
    rows = _rows(CRAFTED)
    mine = rows[rank::world]  # each rank holds some lines of every file
    local = hist.reduce(hist.entries_from_rows(mine), 1)
    recv = sr.exchange_hist(torch.from_numpy(local.view(np.uint8).copy()), world).numpy().view(hist.HIST_ENTRY)
    owned = hist.reduce(recv, privacy)  # the owner's merge + the reference cull
    n = torch.tensor([len(owned)])
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = max(int(x) for x in ns) or 1
    buf = torch.zeros(m * hist.HIST_ENTRY.itemsize, dtype=torch.uint8)
    buf[:len(owned) * hist.HIST_ENTRY.itemsize] = torch.from_numpy(owned.view(np.uint8).copy())
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    if rank == 0:
        parts = [b.numpy()[:int(k) * hist.HIST_ENTRY.itemsize].view(hist.HIST_ENTRY) for b, k in zip(bufs, ns)]
        np.save(out, np.concatenate(parts))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,privacy', [(2, 2), (2, 3), (4, 2), (8, 2), (8, 3)])
def test_owner_cull_equals_reference_loop(tmp_path, world, privacy):
    """gloo world 2, 4, 8: the owners' union after the keyed exchange keeps exactly the
    pairs (and line counts) the reference loop keeps on the whole set's files (at N = 8
    some ranks hold no line and some owners receive no entry)."""
    out = str(tmp_path / 'owned.npy')
    mp.spawn(_crafted_rank, args=(world, _store(tmp_path), out, privacy), nprocs=world, join=True)
    got = _pairs_from_entries(np.load(out))
    want = _pairs_from_lines(_rows(CRAFTED), privacy)
    assert want and got == want
    # (a cull of whole pairs by their totals alone keeps a different set here)
    tot = _pairs_from_entries(hist.reduce(hist.entries_from_rows(_rows(CRAFTED)), 1))
    assert {k: v for k, v in tot.items() if v >= privacy} != want
