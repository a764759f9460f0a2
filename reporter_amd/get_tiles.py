#!/usr/bin/env python3
"""The reference's py/get_tiles.py (tile hierarchy and tile listing, :22-171) over the
library's C-ABI (include/otr.h otr_tilehier_*): same classes, methods and command line

    python -m reporter_amd.get_tiles -b -74.251961,40.512764,-73.755405,40.903125 -s gph

prints the tile files a bbox needs, in the order the reference prints them.  Used by
download_tiles.sh:55 (`get_tiles.py -b ${BBOX} -s ${FILE_TYPE} > files.txt`).
"""
import ctypes
import getopt
import sys

from . import _lib

minx_, miny_, maxx_, maxy_ = -180, -90, 180, 90
SIZES = {0: 4, 1: 1, 2: .25}


class BoundingBox(object):
    def __init__(self, min_x, min_y, max_x, max_y):
        self.minx, self.miny, self.maxx, self.maxy = min_x, min_y, max_x, max_y


class Tiles(object):
    """Tiles of one hierarchy level (get_tiles.py:44-102)."""

    def __init__(self, level):
        self.level = level
        self.tilesize = SIZES[level]
        self.ncolumns = int(360 / self.tilesize)
        self.nrows = int(180 / self.tilesize)
        self.max_tile_id = self.ncolumns * self.nrows - 1

    def Row(self, y):
        return _lib.lib().otr_tilehier_row(self.level, float(y))

    def Col(self, x):
        return _lib.lib().otr_tilehier_col(self.level, float(x))

    def GetFile(self, tile_id, level=None, suffix='gph'):
        buf = ctypes.create_string_buffer(64)
        lv = self.level if level is None else level
        rc = _lib.lib().otr_tilehier_file(lv, int(tile_id), suffix.encode(), buf, len(buf))
        if rc != 0:
            raise ValueError('bad tile level or id')
        return buf.value.decode()


class TileHierarchy(object):
    def __init__(self):
        self.levels = {2: Tiles(2), 1: Tiles(1), 0: Tiles(0)}


def tile_files(min_lon, min_lat, max_lon, max_lat, suffix):
    """The file names the reference prints for this bbox (otr_tilehier_files)."""
    L = _lib.lib()
    out, n = ctypes.c_void_p(), ctypes.c_size_t()
    rc = L.otr_tilehier_files(float(min_lon), float(min_lat), float(max_lon), float(max_lat), suffix.encode(),
                              ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError('otr_tilehier_files failed (%d)' % rc)
    return _lib.take_string(out, n).splitlines()


USAGE = ('tiles.py -b lower_left_lng_lat, upper_right_lng_lat -s file_suffix\n'
         'tiles.py -b -74.251961,40.512764,-73.755405,40.903125 -s json')


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    try:
        opts, _ = getopt.getopt(argv, 'h:b:s:', ['help=', 'bbox=', 'suffix='])
    except getopt.GetoptError:
        print(USAGE)
        return 2
    bbox = suffix = None
    for opt, arg in opts:
        if opt in ('-h', '--help'):
            print(USAGE)
            return 0
        if opt in ('-b', '--bbox'):
            bbox = arg
        elif opt in ('-s', '--suffix'):
            suffix = arg
    if bbox is None or suffix is None:
        print(USAGE)
        return 0
    b = [float(i) for i in bbox.split(',')]
    for f in tile_files(b[0], b[1], b[2], b[3], suffix):
        print(f)
    return 0


if __name__ == '__main__':
    sys.exit(main())
