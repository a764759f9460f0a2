"""The RCCL branch of the multi-GPU exchange executed on the
one GPU a box has: a `nccl` (RCCL) process group of world size 1 on cuda:0, the keyed
histogram entries and the tile rows sent through `exchange_hist` / `exchange_rows` as
DEVICE tensors (the N > 1 code path, simple_reporter.py's uuid-shard layout of :116 and
:288-294 with one shard), then the owner's reduce + privacy cull.  The result must equal
the N = 1 direct reduce of the rows and the CPU restatement oracle/hist.reduce."""
import os
import socket

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


class _DevBytes:
    """A library-owned device byte range as a torch tensor view (no copy)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {'shape': (int(nbytes),), 'typestr': '|u1', 'data': (int(ptr), False),
                                         'version': 2}


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope='module')
def rccl():
    import torch
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    assert dist.get_backend() == 'nccl'
    yield dist
    dist.destroy_process_group()


@pytest.fixture(scope='module')
def workload(graph_dir):
    path = gen.graph_path('city', graph_dir)
    M.configure(M.default_config(path))
    tr = gen.make_traces(path, 160, 120, 10, 8.0, 53, t_begin=gen.T_BEGIN, t_spread=3 * 3600)
    want = po.match_batch(po.Graph(path), tr, po.params(), threads=8)
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    return tr, ot.rows_from_reports(want, first, last)


def test_rccl_world1_keyed_exchange(rccl, workload):
    import torch
    tr, rows = workload
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=False, tile_rows=True)
    n_rows = int(r.n_rows)
    assert n_rows == len(rows) > 100
    EW = _lib.HIST_ENTRY.itemsize
    # this GPU's (file, pair, speed bin) counts, in HBM (privacy 1: the per-GPU side)
    ebuf = torch.empty(n_rows * EW, dtype=torch.uint8, device='cuda')
    n_local = sr.hist_reduce(m, r.d_rows, n_rows, privacy=1, rows_in=True, out=ebuf.data_ptr())
    local_e = ebuf[:n_local * EW]
    # the RCCL all-to-all on device tensors (counts, then entries)
    recv = sr.exchange_hist(local_e, 1)
    torch.cuda.synchronize()
    assert recv.is_cuda and recv.numel() == local_e.numel()
    assert torch.equal(recv, local_e)  # world 1: rank 0 owns every (hour, tile) file
    for privacy in (1, 2):
        owned = sr.hist_reduce(m, recv.data_ptr(), n_local, privacy=privacy)
        direct = sr.hist_reduce(m, r.d_rows, n_rows, privacy=privacy, rows_in=True)
        want = oh.reduce(oh.entries_from_rows(rows), privacy)
        assert len(want) > 0
        assert np.array_equal(owned, direct)
        assert np.array_equal(owned, want)


def test_rccl_world1_row_exchange(rccl, workload):
    """Tile rows to their file's owner over RCCL, then the owner's sort + cull (K10) equals
    the oracle's tiles (simple_reporter.py:211-239)."""
    import torch
    tr, rows = workload
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=False, tile_rows=True)
    RW = _lib.TILE_ROW.itemsize
    dev_rows = torch.as_tensor(_DevBytes(r.d_rows, int(r.n_rows) * RW), device='cuda').clone()
    got = sr.exchange_rows(dev_rows, 1)
    torch.cuda.synchronize()
    assert got.is_cuda and torch.equal(got, dev_rows)
    owner = sr.file_owner(torch.from_numpy(rows['file'].astype(np.int64)), 1)
    assert int(owner.max()) == 0
    kept = sr.cull_rows(m, None, 2, device_ptr=got.data_ptr(), n=int(r.n_rows))
    assert sr.rows_to_tiles(kept) == ot.tiles(rows, 2)


def test_bench_dist_flag_world1(tmp_path):
    """bench.py --dist runs the N > 1 code path (process group, shard, keyed RCCL exchange)
    at world size 1, in a child process (its own process group)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--dist', '--workload', 'c2',
                          '--traces-per-gpu', '2000', '--steps', '2', '--warmup', '1', '--cpu-traces', '200',
                          '--e2e-steps', '0'], cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith('{')][-1])
    assert line['n_gpus'] == 1 and line['parity']['ok']
    assert 'RCCL' in line['config']['parallelism']
    h = line['config']['histogram']
    assert h['received'] == h['local_entries'] > 0 and h['exchange_bytes_sent'] > 0
