"""Ingest (§8 f rank 4) on the CPU: the restatement in oracle/ingest.py against the
reference's own known answers, and the device number parsers (host build,
reporter_amd/tools/libparsecheck.so) against Python's float() / int() / str()."""
import calendar
import ctypes
import math
import os
import random
import struct

import numpy as np
import pytest

from oracle import ingest as oi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# FormatterTest.java:30-45: the raw '|' line and the Point it must give
FMT_LINE = b'2017-01-01 06:05:40|w00t||||6.5||||0.0|0.0'
FMT_POINT = ('w00t', (0.0, 0.0, 1483250740, 7))


def test_formatter_known_answer_java():
    assert oi.java_sv_records(FMT_LINE + b'\n') == [FMT_POINT]


def test_formatter_known_answer_download():
    # the same line through simple_reporter.download()'s default valuer (:352) and
    # time pattern (:353): min(ceil(6.5), 1000) = 7, str(0.0) = '0.0'
    assert oi.raw_to_shard_text(FMT_LINE) == b'w00t,1483250740,0.0,0.0,7\n'


def test_shard_windows_hand_derived():
    # uuid a: times 0, 100, 500 (gap 400 > 120), 510, 505 (sorted), b: one point,
    # c: a single window of 2; the lone point at 500..510 window keeps 3 points
    text = (b'a,0,1.0,2.0,5\n b,7,1.5,2.5,5\r\na,100,1.1,2.1,5\na,510,1.3,2.3,6\n'
            b'c,1,0.5,0.5,1\na,505,1.2,2.2,5\nc,2,0.6,0.6,1\na,500,1.25,2.25,5')
    got = oi.shard_traces(text, inactivity=120)
    assert got == [('a', [(1.0, 2.0, 0, 5), (1.1, 2.1, 100, 5)]),
                   ('a', [(1.25, 2.25, 500, 5), (1.2, 2.2, 505, 5), (1.3, 2.3, 510, 6)]),
                   ('c', [(0.5, 0.5, 1, 1), (0.6, 0.6, 2, 1)])]


def test_shard_errors_name_the_line():
    with pytest.raises(oi.IngestError) as e:
        oi.shard_traces(b'a,0,1.0,2.0,5\na,1,1.0,2.0\n')
    assert e.value.line == 1 and e.value.reason == 'fields'
    with pytest.raises(oi.IngestError) as e:
        oi.shard_traces(b'a,0,1.0,2.0,5\n\n')  # ''.split(',') has one field
    assert e.value.line == 1
    with pytest.raises(oi.IngestError) as e:
        oi.shard_traces(b'a,0,1.0,2.0,5\na,1.5,1.0,2.0,5\n')
    assert e.value.reason == 'int'


def test_raw_bbox_skips_before_time_and_accuracy():
    # out of the bbox: never parsed further, even with a broken time (:103-105)
    bad = '|'.join(['garbage', 'u', '', '', '', 'x', '', '', '', '50.0', '50.0'])
    good = '|'.join(['2017-01-01 00:00:00', 'u', '', '', '', '3', '', '', '', '1.0', '1.0'])
    text = (bad + '\n' + good + '\n').encode()
    assert oi.raw_to_shard_text(text, bbox=[-10, -10, 10, 10]) == b'u,1483228800,1.0,1.0,3\n'
    with pytest.raises(oi.IngestError):
        oi.raw_to_shard_text(text)


def test_py2_str_is_twelve_digits():
    assert oi.py2_str_float(1.1234567890123) == '1.12345678901'
    assert oi.py2_str_float(14.0) == '14.0'
    assert oi.py2_str_float(-0.5) == '-0.5'


# ---- the device parsers, host build ------------------------------------------------

@pytest.fixture(scope='module')
def pc():
    from reporter_amd import build
    lib = ctypes.CDLL(build.build_parsecheck())
    lib.pc_float.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)]
    lib.pc_py2_str.argtypes = lib.pc_float.argtypes
    lib.pc_int.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.pc_ymdhms.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    lib.pc_hash.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    lib.pc_hash.restype = ctypes.c_uint64
    return lib


def _bits(x):
    return struct.pack('<d', x)


def _digits(s):
    t = s.strip().lstrip('+-').lower().split('e')[0].replace('.', '').lstrip('0')
    return len(t)


def _float_cases(rng, n):
    for _ in range(n):
        k = rng.randrange(7)
        if k == 0:
            yield repr(rng.uniform(-180, 180))
        elif k == 1:
            yield '%.*f' % (rng.randrange(0, 16), rng.uniform(-180, 180))
        elif k == 2:
            yield repr(struct.unpack('<d', struct.pack('<Q', rng.getrandbits(64)))[0])
        elif k == 3:
            d = ''.join(rng.choice('0123456789') for _ in range(rng.randrange(1, 19)))
            yield d[:rng.randrange(len(d) + 1)] + '.' + d + ('e%d' % rng.randrange(-330, 310) if rng.random() < .5
                                                              else '')
        elif k == 4:
            yield '%de%d' % (rng.getrandbits(rng.randrange(1, 64)), rng.randrange(-40, 40))
        elif k == 5:
            # exact binary midpoints printed with up to 19 significant digits
            x = rng.uniform(1e-3, 1e3)
            m, e = math.frexp(x)
            mid = 2 * int(m * 2 ** 53) + 1
            yield repr(mid * 2.0 ** (e - 54))
        else:
            yield rng.choice([' 1.5 ', '+.5', '-0', '-0.0', '1e', '1.', '.', 'e5', '1e+', '0x10', '', ' ', '--1',
                              '1.2.3', '4e-320', '2.2250738585072011e-308', '9007199254740993', '\t12\n', '1E5',
                              '1e400', '-1e-400', '00000.000001', '1_0', 'inf', 'nan'])


def test_float_parser_equals_python(pc):
    rng = random.Random(11)
    out = ctypes.c_double()
    n_ok = 0
    for s in _float_cases(rng, 40000):
        b = s.encode()
        rc = pc.pc_float(b, len(b), ctypes.byref(out))
        try:
            want = float(s) if '_' not in s and s.strip().lower() not in ('inf', 'nan') else None
        except ValueError:
            want = None
        if want is None:
            assert rc == 1, s
            continue
        if rc == 2:  # refused: only beyond 19 significant digits
            assert _digits(s) > 19, s
            continue
        assert rc == 0, s
        assert _bits(out.value) == _bits(want), (s, out.value, want)
        n_ok += 1
    assert n_ok > 35000


def test_py2_str_roundtrip_equals_python(pc):
    rng = random.Random(12)
    out = ctypes.c_double()
    for _ in range(30000):
        k = rng.randrange(3)
        if k == 0:
            s = repr(rng.uniform(-180, 180))
        elif k == 1:
            w = rng.randrange(10 ** 11, 10 ** 12)
            s = str(w) + rng.choice(['5', '49999', '50001', '5000000', '4999999'])
            s = s[:2] + '.' + s[2:]
        else:
            s = '%.17g' % (rng.uniform(-1, 1) * 10 ** rng.randrange(-8, 8))
        b = s.encode()
        assert pc.pc_py2_str(b, len(b), ctypes.byref(out)) == 0, s
        assert _bits(out.value) == _bits(float(oi.py2_str_float(float(s)))), s


def test_int_parser_equals_python(pc):
    out = ctypes.c_int64()
    for s in ['0', '-0', '+7', ' 12 ', '\t-3\n', '9223372036854775807', '-9223372036854775808',
              '9223372036854775808', '', '+', '1.0', '1e3', '12a', '0012']:
        b = s.encode()
        rc = pc.pc_int(b, len(b), ctypes.byref(out), 0)
        try:
            want = int(s)
            ok = -2 ** 63 <= want < 2 ** 63
        except ValueError:
            ok = False
        assert (rc == 0) == ok, s
        if ok:
            assert out.value == want
    b = b' 12'
    assert pc.pc_int(b, len(b), ctypes.byref(out), 1) == 1  # Long.parseLong: no whitespace


def test_fast_time_equals_timegm(pc):
    rng = random.Random(13)
    out = ctypes.c_int64()
    for _ in range(5000):
        y, mo, d = rng.randrange(1, 10000), rng.randrange(1, 13), rng.randrange(1, 29)
        h, mi, se = rng.randrange(0, 24), rng.randrange(0, 60), rng.randrange(0, 60)
        s = '%04d-%02d-%02d %02d:%02d:%02d' % (y, mo, d, h, mi, se)
        s += rng.choice(['', '.123', 'Z'])
        b = s.encode()
        assert pc.pc_ymdhms(b, len(b), ctypes.byref(out)) == 0, s
        assert out.value == calendar.timegm((y, mo, d, h, mi, se, 0, 0, 0)), s
    for s in ['2017-13-01 00:00:00', '2017-00-01 00:00:00', '0000-01-01 00:00:00', '2017-01-01 0a:00:00', '']:
        b = s.encode()
        assert pc.pc_ymdhms(b, len(b), ctypes.byref(out)) != 0, s
        assert oi._fast_time(s)[1] is not None


def test_uuid_hash_spreads(pc):
    hs = {pc.pc_hash(('veh%07d' % i).encode(), 10) for i in range(100000)}
    assert len(hs) == 100000
