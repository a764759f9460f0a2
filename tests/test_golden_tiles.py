"""simple_reporter filter/hour-bucketing (:176-196) and privacy cull (:218-239) against
golden vectors from the reference's own code; plus the HIP path's shared C++ rules
(bucket_span / py2 rounding) are exercised on GPU in test_gpu_pipeline.py."""
import json
import os

import pytest

from reporter_amd import simple_reporter as sr

HERE = os.path.dirname(os.path.abspath(__file__))
CULL = json.load(open(os.path.join(HERE, 'golden', 'cull_cases.json')))['cases']
BUCKET = json.load(open(os.path.join(HERE, 'golden', 'bucket_cases.json')))['cases']


@pytest.mark.parametrize('i', range(len(CULL)))
def test_cull(i):
    c = CULL[i]
    assert sr.cull(c['lines'], c['privacy']) == c['expected']


def test_cull_trailing_singleton_quirk():
    # verified against the reference loop: [A,A,B] p=2 keeps all; [A,B] p=2 keeps both; [A] p=2 deletes
    assert sr.cull(['A,B,1\n', 'A,B,2\n', 'C,D,1\n'], 2) == ['A,B,1\n', 'A,B,2\n', 'C,D,1\n']
    assert sr.cull(['A,B,1\n', 'C,D,1\n'], 2) == ['A,B,1\n', 'C,D,1\n']
    assert sr.cull(['A,B,1\n'], 2) == []


@pytest.mark.parametrize('i', range(len(BUCKET)))
def test_bucket(i):
    c = BUCKET[i]
    got = sr.bucket(c['first_time'], c['last_time'], c['reports'], c['quantisation'], c['mode'], c['source'])
    want = {k.split('/', 1)[1]: v for k, v in c['expected'].items()}  # drop the dest_dir prefix
    assert got == want


def test_windows_and_shard():
    assert sr.windows([0, 10, 20, 300, 310, 1000], 120) == [(0, 3), (3, 5)]
    assert sr.shard_key('veh0000001') == __import__('hashlib').sha1(b'veh0000001').hexdigest()[:3]
    assert all(0 <= sr.shard_of('veh%07d' % i, 8) < 8 for i in range(100))
    assert sr.INVALID_SEGMENT_ID == 0x3fffffffffff
