// Host build of the node tables' IN-gap codes (reporter_amd/csrc/otr_mincode.h) so that the
// CPU tests can check the properties the exact rounds rely on.
// TEST INFRASTRUCTURE ONLY: the codes are used by the GPU search (otr_kernels.h).
#include "../csrc/otr_mincode.h"

using namespace otr;

extern "C" {
// lengths m in [lo, hi) by `step`: the decoded gaps of both codes are >= 1 and <= max(m, 1)
// (a lower bound of any in-edge of that length), monotone in m, and the one-byte code keeps
// at least 15/16 of m - 16 mm below its 8 km saturation; returns the violations
uint64_t mc_lengths(uint64_t lo, uint64_t hi, uint64_t step) {
  uint64_t bad = 0;
  uint32_t prev16 = 0, prev8 = 0;
  for (uint64_t x = lo; x < hi; x += step) {
    const uint32_t m = (uint32_t)x;
    const uint32_t g16 = in_gap(mi_of(m)), g8 = mf8_gap(mf8_of(m));
    const uint32_t ub = m > 1u ? m : 1u;
    bad += (g16 < 1u || g16 > ub) ? 1 : 0;
    bad += (g8 < 1u || g8 > ub) ? 1 : 0;
    bad += (g16 < prev16 || g8 < prev8) ? 1 : 0;
    if (m >= 32u && m < (1u << 23)) bad += ((uint64_t)g8 * 16u + 256u < (uint64_t)m * 15u) ? 1 : 0;
    prev16 = g16;
    prev8 = g8;
  }
  return bad;
}
// every code: re-encoding its gap gives the code back (a dump between tables of the same
// code is exact), and re-encoding into the other code keeps a lower bound (a dump from a
// 2-byte-code table into a 1-byte one and back)
uint64_t mc_codes(void) {
  uint64_t bad = 0;
  for (uint32_t c = 0; c < 256u; ++c) {
    const uint32_t g = mf8_gap((uint8_t)c);
    bad += mf8_of(g) != (uint8_t)c && g != 1u ? 1 : 0;
    bad += in_gap(mi_of(g)) > g ? 1 : 0;
  }
  for (uint32_t c = 0; c < 65536u; ++c) {
    const uint32_t g = in_gap((uint16_t)c);
    bad += mi_of(g) != (uint16_t)c && g != 1u ? 1 : 0;
    bad += mf8_gap(mf8_of(g)) > g ? 1 : 0;
  }
  return bad;
}
}
