"""K11 ingest on the GPU through the C-ABI (otr_ingest) against the CPU restatement in
oracle/ingest.py: the traces must be identical — same windows in the same order, the
same doubles bit for bit — and the whole text → match → tiles path must equal the
oracle's."""
import numpy as np
import pytest

from oracle import ingest as oi
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


def _host(ptr, n, dtype):
    import torch
    dt = np.dtype(dtype)
    if n == 0:
        return np.zeros(0, dt)
    return torch.as_tensor(_DevArr(ptr, n * dt.itemsize), device='cuda').clone().cpu().numpy().view(dt)


def _got(text, r, b):
    nt, npr = int(r.n_traces), int(r.n_probes)
    off = _host(b.arrays['trace_offsets'], nt + 1, np.int64)
    uo = _host(b.uuid_off, nt, np.int64)
    ul = _host(b.uuid_len, nt, np.int32)
    uuids = [text[int(o):int(o) + int(n)].decode('latin-1') for o, n in zip(uo, ul)]
    return (uuids, off, _host(b.arrays['lat'], npr, np.float64), _host(b.arrays['lon'], npr, np.float64),
            _host(b.arrays['time'], npr, np.int64), _host(b.arrays['accuracy'], npr, np.float32))


def _same(got, want):
    assert got[0] == want[0]
    for g, w in zip(got[1:], want[1:]):
        assert g.dtype == w.dtype and g.shape == w.shape
        assert g.tobytes() == w.tobytes()


@pytest.fixture(scope='module')
def city(graph_dir):
    path = gen.graph_path('city', graph_dir)
    M.configure(M.default_config(path))
    return path


@pytest.fixture(scope='module')
def traces(city):
    return gen.make_traces(city, 150, 60, 10, 8.0, 41, t_begin=gen.T_BEGIN, t_spread=3 * 3600)


def test_shard_text_equals_restatement(traces):
    text = gen.probe_text(traces, 'shard', seed=1, shuffle=0.3, split_gap=600)
    m = M.Matcher()
    r, b = m.ingest(text, rules=_lib.OTR_INGEST_SHARD, inactivity=120)
    want = oi.to_soa(oi.shard_traces(text, 120))
    assert r.n_lines == traces.n_probes and r.n_uuids == traces.n_traces
    assert r.n_traces == len(want[0]) > traces.n_traces  # the pauses split traces
    _same(_got(text, r, b), want)


def test_raw_text_equals_restatement(traces):
    text = gen.probe_text(traces, 'raw', seed=2, shuffle=0.2, crlf=True)
    lat = np.sort(traces.lat)
    bbox = [float(lat[len(lat) // 5]), -180.0, 90.0, 180.0]  # drops about a fifth
    m = M.Matcher()
    r, b = m.ingest(text, rules=_lib.OTR_INGEST_RAW, bbox=bbox, inactivity=120)
    want = oi.to_soa(oi.raw_traces(text, 120, bbox=bbox))
    assert 0 < r.n_kept < r.n_lines
    _same(_got(text, r, b), want)


def test_java_sv_equals_restatement(traces):
    text = gen.probe_text(traces, 'raw', seed=3, shuffle=0.1)
    m = M.Matcher()
    r, b = m.ingest(text, rules=_lib.OTR_INGEST_JAVA_SV, inactivity=120)
    _same(_got(text, r, b), oi.to_soa(oi.java_sv_traces(text, 120)))


def test_formatter_known_answer_on_device():
    # FormatterTest.java:30-45, twice 15 s apart so that one window of 2 comes out
    line2 = b'2017-01-01 06:05:55|w00t||||6.5||||0.0|0.0'
    text = b'2017-01-01 06:05:40|w00t||||6.5||||0.0|0.0\n' + line2
    m = M.Matcher()
    for rules in (_lib.OTR_INGEST_JAVA_SV, _lib.OTR_INGEST_RAW):
        r, b = m.ingest(text, rules=rules)
        uuids, off, lat, lon, tm, acc = _got(text, r, b)
        assert uuids == ['w00t'] and list(off) == [0, 2]
        assert list(tm) == [1483250740, 1483250755] and list(acc) == [7, 7] and not lat.any() and not lon.any()


def test_edge_texts():
    m = M.Matcher()
    r, _ = m.ingest(b'', rules=_lib.OTR_INGEST_SHARD)
    assert r.n_lines == 0 and r.n_traces == 0
    r, _ = m.ingest(b'a,1,1.0,2.0,5\n', rules=_lib.OTR_INGEST_SHARD)  # one point: no window
    assert r.n_lines == 1 and r.n_traces == 0
    text = b'a,1,1.0,2.0,5\r\n  b,2,1.0,2.0,5\na,2,1.5,2.5,5\nb,1,1.5,2.5,5'
    r, b = m.ingest(text, rules=_lib.OTR_INGEST_SHARD)
    _same(_got(text, r, b), oi.to_soa(oi.shard_traces(text, 120)))


@pytest.mark.parametrize('rules,text', [
    (_lib.OTR_INGEST_SHARD, b'a,1,1.0,2.0,5\na,2,1.0,2.0\na,3,x,2.0,5\n'),
    (_lib.OTR_INGEST_SHARD, b'a,1,1.0,2.0,5\na,2,1.0,2.0,5\n\n'),
    (_lib.OTR_INGEST_SHARD, b'a,1,1.0,2.0,5\na,2.5,1.0,2.0,5\n'),
    (_lib.OTR_INGEST_SHARD, b'a,1,1.0,2.0,5\na,2,1.0,nan,5\n'),
    (_lib.OTR_INGEST_RAW, b'2017-01-01 06:05:40|w00t||||6.5||||0.0|0.0\n2017-13-01 06:05:40|w||||6.5||||0.0|0.0\n'),
    (_lib.OTR_INGEST_RAW, b'2017-01-01 06:05:40|w00t||||6.5||||0.0\n'),
])
def test_rejected_line_matches_restatement(rules, text):
    want = None
    try:
        if rules == _lib.OTR_INGEST_SHARD:
            oi.shard_traces(text)
        else:
            oi.raw_traces(text)
    except oi.IngestError as e:
        want = e
    assert want is not None
    m = M.Matcher()
    with pytest.raises(ValueError) as e:
        m.ingest(text, rules=rules)
    assert str(e.value) == 'line %d: %s' % (want.line, want.reason)


def test_text_to_tiles_equals_oracle(city, traces):
    """simple_reporter end to end from a shard file: ingest (K11) → match (K1-K8) → tile
    rows (K9) → sort + cull (K10), all in HBM, against the CPU restatements."""
    text = gen.probe_text(traces, 'shard', seed=4, shuffle=0.3, split_gap=600)
    m = M.Matcher()
    got = sr.text_tiles_device(m, text, 2)
    uuids, off, lat, lon, tm, acc = oi.to_soa(oi.shard_traces(text, 120))
    tr = gen.Traces(lat, lon, tm, off, np.zeros(len(uuids), np.uint8), accuracy=acc)
    want = po.match_batch(po.Graph(city), tr, po.params(), threads=8)
    rows = ot.rows_from_reports(want, tm[off[:-1]], tm[off[1:] - 1])
    assert got == ot.tiles(rows, 2) and len(got) > 0
