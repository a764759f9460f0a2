"""CPU restatement of the reference's tile hierarchy — TEST INFRASTRUCTURE ONLY.

py/get_tiles.py:30-102 (TileHierarchy, Tiles.Row / Col / Digits / GetFile) and the
listing loop of its main block (:132-171), restated in Python 3 with the reference's
Python 2 semantics written out: integer division in Digits, and the level order in
which Python 2 iterates the dict {2: .., 1: .., 0: ..} (small-int keys sit in hash
slots 0, 1, 2: levels 0, 1, 2).  Pinned by tests/golden/tile_cases.json, which
tests/golden/make_tile_goldens.py produced by executing the reference's own classes
and loop under those semantics.  Checker for otr_tilehier_* (include/otr.h).
"""
import math

MINX, MINY, MAXX, MAXY = -180, -90, 180, 90
SIZES = {0: 4, 1: 1, 2: .25}


class Tiles:
    def __init__(self, size):
        self.tilesize = size
        self.ncolumns = int(math.ceil((MAXX - MINX) / size))
        self.nrows = int(math.ceil((MAXY - MINY) / size))
        self.max_tile_id = self.ncolumns * self.nrows - 1

    def row(self, y):
        if y < MINY or y > MAXY:
            return -1
        if y == MAXY:
            return self.nrows - 1
        return int((y - MINY) / self.tilesize)

    def col(self, x):
        if x < MINX or x > MAXX:
            return -1
        if x == MAXX:
            return self.ncolumns - 1
        c = (x - MINX) / self.tilesize
        return int(c) if c >= 0.0 else int(c - 1)

    @staticmethod
    def digits(n):
        d = 1 if n < 0 else 0
        while n:
            n = int(n / 10) if n < 0 else n // 10  # Python 2 long division (non-negative ids)
            d += 1
        return d

    def get_file(self, tile_id, level, suffix):
        ml = self.digits(self.max_tile_id)
        if ml % 3:
            ml += 3 - ml % 3
        base = 10 ** ml
        s = '{:,}'.format((base if level == 0 else level * base) + tile_id).replace(',', '/') + '.' + suffix
        return '0' + s[1:] if level == 0 else s


def levels():
    return [(lv, Tiles(SIZES[lv])) for lv in (0, 1, 2)]


def tile_files(min_lon, min_lat, max_lon, max_lat, suffix):
    """The names get_tiles.py prints for `-b min_lon,min_lat,max_lon,max_lat -s suffix`."""
    b = [min_lon, min_lat, max_lon, max_lat]
    if b[0] >= b[2]:
        b[0] = b[0] - 360
    rng = MAXX - MINX
    if b[0] < MINX and b[2] > MINX:
        boxes = [(MINX, b[1], b[2], b[3]), (b[0] + rng, b[1], MAXX, b[3])]
    elif b[0] < MAXX and b[2] > MAXX:
        boxes = [(b[0], b[1], MAXX, b[3]), (MINX, b[1], b[2] - rng, b[3])]
    else:
        boxes = [tuple(b)]
    out = []
    for bx in boxes:
        for lv, t in levels():
            mincol = t.col(bx[0])
            i = t.row(bx[1])
            while i <= t.row(bx[3]):
                tid = i * t.ncolumns + mincol
                j = mincol
                while j <= t.col(bx[2]):
                    out.append(t.get_file(tid, lv, suffix))
                    tid += 1
                    j += 1
                i += 1
    return out
