"""The C-ABI library loads and exports every symbol include/otr.h declares (no GPU call)."""
import ctypes
import os
import re

from reporter_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_match_header():
    hdr = open(os.path.join(ROOT, 'include', 'otr.h')).read()
    declared = set(re.findall(r'\b(otr_[a-z_]+)\s*\(', hdr))
    assert declared == set(_lib.EXPORTS)
    L = _lib.lib()
    for s in declared:
        assert hasattr(L, s), s


def test_struct_layout():
    # otr_trace_batch / otr_batch_result sizes must match the C declarations
    assert ctypes.sizeof(_lib.TraceBatch) == 4 + 4 + 6 * 8 + 4 * 4 + 8 + 4 + 4 + 8 + 4 + 4
    assert ctypes.sizeof(_lib.BatchResult) > 0


def test_batch_limit_launch_plan():
    """The batch limit keeps every per-state / per-trace dispatch below 2^32 work-items
    (otr_launch.h; a wave per state: 64 work-items, k_candidates in groups of 8 states)."""
    L = _lib.lib()
    cap = L.otr_max_batch_probes()
    assert cap == (1 << 26) - 64
    lim = (1 << 32) - 1
    for n in (cap, (1 << 26) - 1, 1 << 26, (1 << 26) + 1):
        for g in (1, 2):
            items = L.otr_launch_max_items(n, n, g)
            # 64 work-items per state, the state count rounded up to 8 (k_candidates)
            assert items == 64 * 8 * ((n + 7) // 8)
            assert (items <= lim) == (n <= (1 << 26) - 8), (n, g, items)
    # every accepted batch fits: states <= probes and traces <= probes
    for s, t in ((cap, 1), (1, cap), (cap, cap), (cap // 2, cap)):
        assert L.otr_launch_max_items(s, t, 1) <= lim
    # the first refused size is the first whose widest launch could exceed it by design
    assert L.otr_launch_max_items(0, 0, 1) == 0


def test_not_configured_errors():
    from reporter_amd import matcher as M
    # a bad config fails loudly (no fallback)
    try:
        M.configure({'otr': {'graph': '/nonexistent.otrg'}})
    except RuntimeError as e:
        assert 'graph' in str(e) or 'open' in str(e)
    else:
        raise AssertionError('configure should fail')


def test_report_request_validation_without_gpu():
    """otr_report's 400 paths (reporter_service.py:214-235) run before any device call."""
    from reporter_amd import matcher as M
    m = M.Matcher()
    code, body = m.report_json('{"trace":[]}')
    assert (code, body) == (400, '{"error":"uuid is required"}')
    code, body = m.report_json('{"uuid":"a","trace":[{"lat":1,"lon":2,"time":3}]}')
    assert code == 400 and 'non zero length array' in body
    code, body = m.report_json('{"uuid":"a","trace":[{"lat":1,"lon":2,"time":3},{"lat":1,"lon":2,"time":4}]}')
    assert (code, body) == (400, '{"error":"match_options must include report_levels array"}')
    code, body = m.report_json('{"uuid":"a","match_options":{"report_levels":[0]},'
                               '"trace":[{"lat":1,"lon":2,"time":3},{"lat":1,"lon":2,"time":4}]}')
    assert (code, body) == (400, '{"error":"match_options must include transition_levels array"}')


def test_struct_layouts_against_c_header(tmp_path):
    """ctypes mirrors of the header structs have the C compiler's sizes and offsets."""
    import shutil
    import subprocess
    if not shutil.which('gcc'):
        import pytest
        pytest.skip('no C compiler')
    structs = {'otr_trace_batch': _lib.TraceBatch, 'otr_ingest_format': _lib.IngestFormat,
               'otr_ingest_result': _lib.IngestResult, 'otr_batch_result': _lib.BatchResult,
               'otr_service_split': _lib.ServiceSplit}
    prog = ['#include <stdio.h>', '#include <stddef.h>', '#include "otr.h"', 'int main(void) {']
    for cname, cls in structs.items():
        prog.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in cls._fields_:
            prog.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f[0], cname, f[0]))
    prog.append('return 0; }')
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(prog))
    exe = tmp_path / 'layout'
    subprocess.check_call(['gcc', '-I' + os.path.join(ROOT, 'include'), str(src), '-o', str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)], text=True).splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f in cls._fields_:
            assert int(got['%s.%s' % (cname, f[0])]) == getattr(cls, f[0]).offset, (cname, f[0])


def test_result_subset_equals_subset_match(graph_dir):
    """oracle.compare.subset: the results of a trace subset sliced out of a batch equal
    matching that subset alone (the property the full-size GPU tests rely on)."""
    import numpy as np
    from oracle import pyoracle as po
    from oracle.compare import compare, subset
    from reporter_amd.tools import gen
    path = gen.graph_path('city', graph_dir)
    tr = gen.make_traces(path, 30, 60, 15, 10.0, 3)
    prm = po.params(turn_penalty_factor=0)
    full = po.match_batch(po.Graph(path), tr, prm, threads=8)
    idx = np.arange(0, 30, 3)
    errors, stats = compare(subset(full, idx, tr.offsets), po.match_batch(po.Graph(path), tr.subset(idx), prm,
                                                                            threads=8))
    assert not errors, errors
    assert stats['n_seg'] > 0
