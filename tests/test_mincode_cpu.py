"""The node search tables' IN-gap codes (reporter_amd/csrc/otr_mincode.h, host build
tools/libmincheck.so): the exact rounds settle a pending node once its length is below
kmin + gap(code(minin)), which is exact only while the decoded gap is a
lower bound of every in-edge.  Checked for the 2-byte code (16-mm units) and the one-byte
minifloat of the 384..1024-slot retry tables: a lower bound >= 1 mm, monotone, >= 15/16 of
the length (less 16 mm) below 8 km, exact re-encoding of every code, and the bound kept
when a dump moves a search between tables of the two codes."""
import ctypes

from reporter_amd import build


def _lib():
    L = ctypes.CDLL(build.build_mincheck())
    L.mc_lengths.restype = ctypes.c_uint64
    L.mc_lengths.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    L.mc_codes.restype = ctypes.c_uint64
    return L


def test_gap_codes_every_length_below_2_24():
    assert _lib().mc_lengths(0, 1 << 24, 1) == 0


def test_gap_codes_sampled_to_2_32():
    L = _lib()
    assert L.mc_lengths(1 << 24, 1 << 32, 4093) == 0  # (a prime stride: every residue class)
    assert L.mc_lengths((1 << 32) - 4096, 1 << 32, 1) == 0  # the top, 0xFFFFFFFF (no in-edge) included


def test_every_code_reencodes():
    assert _lib().mc_codes() == 0
