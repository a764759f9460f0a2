"""Tile hierarchy (reference py/get_tiles.py:30-171): the CPU restatement
oracle/get_tiles.py and the library's otr_tilehier_* (host code in libotr.so, no GPU)
against tests/golden/tile_cases.json (the reference's own classes and listing loop
executed under Python 2 semantics by tests/golden/make_tile_goldens.py)."""
import json
import os

import pytest

from oracle import get_tiles as og

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, 'golden', 'tile_cases.json')))['cases']


def test_oracle_rows_cols_files():
    lv = dict(og.levels())
    for c in CASES['row']:
        assert lv[c['level']].row(c['y']) == c['row'], c
    for c in CASES['col']:
        assert lv[c['level']].col(c['x']) == c['col'], c
    for c in CASES['file']:
        assert lv[c['level']].get_file(c['tile_id'], c['level'], c['suffix']) == c['file'], c


def test_oracle_listing():
    for c in CASES['listing']:
        b = [float(x) for x in c['bbox'].split(',')]
        assert og.tile_files(*b, c['suffix']) == c['files'], c['bbox']


@pytest.fixture(scope='module')
def gt():
    from reporter_amd import get_tiles
    return get_tiles


def test_library_rows_cols_files(gt):
    th = gt.TileHierarchy()
    for c in CASES['row']:
        assert th.levels[c['level']].Row(c['y']) == c['row'], c
    for c in CASES['col']:
        assert th.levels[c['level']].Col(c['x']) == c['col'], c
    for c in CASES['file']:
        assert th.levels[c['level']].GetFile(c['tile_id'], suffix=c['suffix']) == c['file'], c


def test_library_listing_and_cli(gt, capsys):
    for c in CASES['listing']:
        b = [float(x) for x in c['bbox'].split(',')]
        assert gt.tile_files(*b, c['suffix']) == c['files'], c['bbox']
    c = CASES['listing'][0]
    assert gt.main(['-b', c['bbox'], '-s', c['suffix']]) == 0
    assert capsys.readouterr().out.splitlines() == c['files']


def test_known_names():
    # hand-checked: Valhalla level 2 tile of lower Manhattan (row 523, col 425)
    t = dict(og.levels())[2]
    assert (t.row(40.7), t.col(-74.0)) == (522, 424)
    assert t.get_file(522 * 1440 + 424, 2, 'gph') == '2/000/752/104.gph'
    assert dict(og.levels())[0].get_file(2906, 0, 'gph') == '0/002/906.gph'
