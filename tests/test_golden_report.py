"""report() (reporter_service.py:79-179) against golden vectors produced by running the
reference's own function (tests/golden/make_goldens.py) — both the CPU oracle and the
product's C++ report() (the routine the device segment scan shares) must match."""
import json
import math
import os

import pytest

from oracle import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, 'golden', 'report_cases.json')))['cases']


def _norm(x):
    """Compare parsed JSON with float tolerance 0 but int/float equality (0 == 0.0)."""
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_norm(v) for v in x]
    return x


def _check(got, want, path=''):
    if isinstance(want, dict):
        assert isinstance(got, dict), path
        assert set(got) == set(want), (path, sorted(set(got) ^ set(want)))
        for k in want:
            _check(got[k], want[k], path + '/' + k)
    elif isinstance(want, list):
        assert isinstance(got, list) and len(got) == len(want), (path, got, want)
        for i, (a, b) in enumerate(zip(got, want)):
            _check(a, b, '%s[%d]' % (path, i))
    elif isinstance(want, float) or isinstance(got, float):
        assert got == want or (math.isnan(got) and math.isnan(want)), (path, got, want)
    else:
        assert got == want, (path, got, want)


def test_golden_count():
    assert len(CASES) >= 100


@pytest.mark.parametrize('i', range(len(CASES)))
def test_oracle_report(i):
    c = CASES[i]
    segs = c['segments']['segments']
    got = po.report_segments(segs, c['trace'][-1]['time'], c['threshold_sec'], c['report_levels'],
                             c['transition_levels'])
    want = c['expected']
    _check(got['datastore'], want['datastore'])
    _check(got['stats'], want['stats'])
    assert got.get('shape_used') == want.get('shape_used')


@pytest.mark.parametrize('i', range(len(CASES)))
def test_product_report(i):
    from reporter_amd import reporter_service
    c = CASES[i]
    got = reporter_service.report(c['segments'], {'trace': c['trace']}, c['threshold_sec'], c['report_levels'],
                                  c['transition_levels'])
    _check(got, c['expected'])
