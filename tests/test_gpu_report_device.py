"""The device tail of K7 — report_segments compiled for gfx950, the code k_segments runs
per trace — against the golden vectors produced by running the reference's own report()
(reporter_service.py:79-179; tests/golden/make_goldens.py), all cases in one launch
through otr_report_lists_device (include/otr.h)."""
import ctypes
import json
import os

import numpy as np
import pytest

from tests.test_golden_report import CASES, _check

pytestmark = pytest.mark.gpu
NO_ID = 0xFFFFFFFFFFFFFFFF


def _mask(levels):
    m = 0
    for l in levels:
        if 0 <= int(l) < 32:
            m |= 1 << int(l)
    return m


def test_device_report_equals_reference_goldens(graph_dir):
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    M.configure(M.default_config(gen.graph_path('tiny', graph_dir)))  # selects the device
    L = _lib.lib()
    segs = [c['segments']['segments'] for c in CASES]
    n = len(CASES)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum([len(s) for s in segs])
    S = max(int(off[-1]), 1)
    flat = [s for ss in segs for s in ss]
    sid = np.array([int(s['segment_id']) if s.get('segment_id') is not None else NO_ID for s in flat] or [0],
                   np.uint64)
    st = np.array([float(s['start_time']) for s in flat] or [0], np.float64)
    en = np.array([float(s['end_time']) for s in flat] or [0], np.float64)
    internal = np.array([bool(s.get('internal', False)) for s in flat] or [0], np.uint8)
    q = np.array([int(s.get('queue_length') or 0) for s in flat] or [0], np.int32)
    hl = np.array([s.get('length') is not None for s in flat] or [0], np.uint8)
    ln = np.array([int(s.get('length') or 0) for s in flat] or [0], np.int32)
    bs = np.array([int(s.get('begin_shape_index') or 0) for s in flat] or [0], np.int32)
    end_time = np.array([int(c['trace'][-1]['time']) for c in CASES], np.int64)
    thr = np.array([float(c['threshold_sec']) for c in CASES], np.float64)
    rl = np.array([_mask(c['report_levels']) for c in CASES], np.uint32)
    tl = np.array([_mask(c['transition_levels']) for c in CASES], np.uint32)
    rid, rnx = np.zeros(S, np.uint64), np.zeros(S, np.uint64)
    t0, t1 = np.zeros(S), np.zeros(S)
    rlen, rq = np.zeros(S, np.int32), np.zeros(S, np.int32)
    nrep, shape = np.zeros(n, np.int32), np.zeros(n, np.int32)
    counts, lengths, lset = np.zeros(6 * n, np.int32), np.zeros(2 * n), np.zeros(2 * n, np.int32)
    ptr = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    L.otr_report_lists_device.restype = ctypes.c_int
    rc = L.otr_report_lists_device(ctypes.c_int32(n), *[ptr(a) for a in (
        off, sid, st, en, internal, q, hl, ln, bs, end_time, thr, rl, tl, rid, rnx, t0, t1, rlen, rq, nrep, shape,
        counts, lengths, lset)])
    assert rc == 0, _lib.last_error()
    for c in range(n):
        o = int(off[c])
        reports = []
        for i in range(o, o + int(nrep[c])):
            r = {'id': int(rid[i]), 't0': float(t0[i]), 't1': float(t1[i]), 'length': int(rlen[i]),
                 'queue_length': int(rq[i])}
            if int(rnx[i]) != NO_ID:
                r['next_id'] = int(rnx[i])
            reports.append(r)
        k = counts[6 * c:6 * c + 6]
        stats = {'successful_matches': {'count': int(k[0]), 'length': float(lengths[2 * c]) if lset[2 * c] else 0},
                 'unreported_matches': {'count': int(k[1]),
                                        'length': float(lengths[2 * c + 1]) if lset[2 * c + 1] else 0},
                 'match_errors': {'discontinuities': int(k[2]), 'invalid_speeds': int(k[3]),
                                  'invalid_times': int(k[4])},
                 'unassociated_segments': int(k[5])}
        want = CASES[c]['expected']
        _check({'mode': 'auto', 'reports': reports}, want['datastore'], 'case %d datastore' % c)
        _check(stats, want['stats'], 'case %d stats' % c)
        assert (int(shape[c]) if shape[c] >= 0 else None) == want.get('shape_used'), c
