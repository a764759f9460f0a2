"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (ASan
/UBSan on the CPU oracle): `make -C oracle asan` builds the oracle with a standalone
driver; batches with every routing mode (node searches with the time bound, edge-based
searches with turn costs, long C4 bounds, breakage) run clean, and the sanitizer build's
result digest equals the regular build's."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import pyoracle as po
from reporter_amd.tools import gen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OR = os.path.join(ROOT, 'oracle')


@pytest.fixture(scope='module')
def binaries():
    r = subprocess.run(['make', '-C', OR, 'asan'], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(OR, '_asan', 'oracle_asan'), os.path.join(OR, '_asan', 'oracle_plain')


def _dump(path, tr, prm, threads=4):
    with open(path, 'wb') as f:
        f.write(struct.pack('<ii', tr.n_traces, threads))
        f.write(bytes(prm))
        f.write(np.ascontiguousarray(tr.offsets, np.int64).tobytes())
        f.write(np.ascontiguousarray(tr.lat, np.float64).tobytes())
        f.write(np.ascontiguousarray(tr.lon, np.float64).tobytes())
        f.write(np.ascontiguousarray(tr.time, np.int64).tobytes())
        f.write(np.ascontiguousarray(tr.mode, np.uint8).tobytes())


@pytest.mark.parametrize('case', ['deployed_mixed', 'gtt_city', 'c4_long_bounds'])
def test_oracle_clean_under_asan_ubsan(case, binaries, graph_dir, tmp_path):
    asan, plain = binaries
    if case == 'c4_long_bounds':
        g = gen.graph_path('metro', graph_dir)
        tr = gen.make_traces(g, 6, 40, 60, 50.0, 4)
        prm = po.params(search_radius=200, max_search_radius=200, turn_penalty_factor=0)
    elif case == 'gtt_city':
        g = gen.graph_path('city', graph_dir)
        tr = gen.make_traces(g, 12, 80, 15, 10.0, 2)
        prm = po.params(turn_penalty_factor=0)
    else:
        g = gen.graph_path('city', graph_dir)
        tr = gen.make_traces(g, 12, 60, 5, 8.0, 7, 0.3, 0.3)
        prm = po.params()
    b = str(tmp_path / 'batch.bin')
    _dump(b, tr, prm)
    # verify_asan_link_order=0: the environment may preload libraries ahead of ASan's runtime
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1:verify_asan_link_order=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    a = subprocess.run([asan, g, b], capture_output=True, text=True, env=env, timeout=600)
    assert a.returncode == 0, a.stderr[-4000:]
    assert 'runtime error' not in a.stderr and 'ERROR: AddressSanitizer' not in a.stderr, a.stderr[-4000:]
    p = subprocess.run([plain, g, b], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0
    assert a.stdout == p.stdout and 'digest' in a.stdout
