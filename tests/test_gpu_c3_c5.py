"""BASELINE.json configs C3 and C5 on the GPU.

C3: 1,000,000 vehicles "veh%07d" x 100 probes @15 s, sharded by int(sha1(uuid)[:3], 16) % 8
(simple_reporter.py:116); this GPU runs rank 0's share (capped at C3_TRACES traces of it, the
bench's --traces-per-gpu rehearsal), matched in one batch with device tile rows, then the
keyed speed histogram (hour-tile, segment pair, speed bin) sort-reduced and pair-culled on
the device (otr_hist_reduce, the per-GPU side of the §8e exchange).  Checked: an evenly
spread oracle sample field by field, the size-independent properties of every trace
(test_gpu_fullsize._properties), and the device histogram against oracle/hist.py's
reduction of the tile rows that oracle/tiles.py derives from the GPU's reports.

C5: the country graph (7,072 x 7,072 grid, 50M nodes, 134M directed edges, 61M OSMLR
segments; generated once into build/graphs, ~2.5 min and 11.4 GB on a 16-core host) with the
60/25/15 auto/bicycle/pedestrian mode mix over 24 h; a slice of rank 0's N = 8 share, an
oracle sample and the full-batch properties."""
import functools
import hashlib
import os
import sys
import time

import numpy as np
import pytest

from oracle import hist as oh
from oracle import pyoracle as po
from oracle import tiles as ot
from oracle.compare import compare, subset
from reporter_amd import _lib
from reporter_amd import matcher as M
from reporter_amd import simple_reporter as sr
from reporter_amd.graphfile import GraphFile
from reporter_amd.tools import gen

from .test_gpu_fullsize import _properties

pytestmark = pytest.mark.gpu
GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000, 'search_radius': 50,
       'gps_accuracy': 16.45}
C3_TRACES = 20000
C5_TRACES = 12000


@functools.lru_cache(maxsize=None)
def _share(world, rank, n_uuid=1000000):
    """the uuid numbers rank `rank` owns: int(sha1('veh%07d')[:3], 16) % world == rank"""
    return np.array([u for u in range(n_uuid)
                     if int(hashlib.sha1(('veh%07d' % u).encode()).hexdigest()[:3], 16) % world == rank], np.int64)


def _progress(msg):
    # straight to the real stderr (past pytest's capture): a long graph build shows life
    sys.__stderr__.write('[test_gpu_c3_c5] %s\n' % msg)
    sys.__stderr__.flush()


def test_c3_uuid_shard_keyed_histogram(graph_dir):
    path = gen.graph_path('metro', graph_dir)
    M.configure(M.default_config(path, **GTT))
    ids = _share(8, 0)
    assert 120000 < len(ids) < 130000  # ~1/8 of the fleet
    ids = ids[:C3_TRACES]
    tr = gen.make_traces_ids(path, ids, 100, 15, 10.0, 3, t_begin=gen.T_BEGIN, t_spread=1800)
    assert tr.uuids[0] == 'veh%07d' % ids[0]
    m = M.Matcher()
    r = m.match_batch(tr, copy_out=True, tile_rows=True)
    got = _lib.result_to_numpy(r)
    _properties(got, tr, GraphFile(path))
    # the keyed histogram on the device vs the CPU restatement of rows + reduction
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    rows = ot.rows_from_reports(got, first, last)
    assert int(r.n_rows) == len(rows) > 10000
    for privacy in (1, 2):
        dev = sr.hist_reduce(m, r.d_rows, r.n_rows, privacy=privacy, rows_in=True)
        want = oh.reduce(oh.entries_from_rows(rows), privacy)
        assert len(want) > 0 and np.array_equal(dev, want), privacy
    # the matcher itself: an evenly spread oracle sample
    idx = np.linspace(0, len(ids) - 1, 120).astype(np.int64)
    ref = po.match_batch(po.Graph(path), tr.subset(idx), po.params(**GTT), threads=16)
    errors, stats = compare(subset(got, idx, tr.offsets), ref)
    assert not errors, errors
    assert stats['n_seg'] > 0 and stats['n_rep'] > 0


@pytest.mark.timeout(900)  # the country graph is generated in-test on a fresh box
def test_c5_country_graph_mode_mix(graph_dir):
    t0 = time.time()
    _progress('country graph: generating into %s if absent (~2.5 min)' % graph_dir)
    path = gen.graph_path('country', graph_dir)
    _progress('country graph ready after %.0f s' % (time.time() - t0))
    M.configure(M.default_config(path, **GTT))
    ids = _share(8, 0)[:C5_TRACES]
    tr = gen.make_traces_ids(path, ids, 100, 15, 10.0, 5, 0.25, 0.15, t_begin=gen.T_BEGIN, t_spread=86400)
    modes = np.bincount(tr.mode, minlength=3) / tr.n_traces
    assert abs(modes[0] - 0.60) < 0.03 and abs(modes[1] - 0.25) < 0.03 and abs(modes[2] - 0.15) < 0.03, modes
    got = _lib.result_to_numpy(M.Matcher().match_batch(tr, copy_out=True))
    _progress('country batch matched (%d traces)' % tr.n_traces)
    _properties(got, tr, GraphFile(path))
    # oracle sample: every mode present
    idx = np.linspace(0, tr.n_traces - 1, 90).astype(np.int64)
    assert len(set(tr.mode[idx].tolist())) == 3
    ref = po.match_batch(po.Graph(path), tr.subset(idx), po.params(**GTT), threads=16)
    errors, stats = compare(subset(got, idx, tr.offsets), ref)
    assert not errors, errors
    assert stats['n_seg'] > 0 and stats['n_rep'] > 0
    _progress('country sample bit-exact (%d segments)' % stats['n_seg'])
