// otr_mincode.h — the IN-criterion gap codes of the node search tables (otr_kernels.h
// SearchLds::mi): minin(node), the shortest in-edge in mm, stored rounded DOWN so that
// the decoded gap is a lower bound of every later offer's increment (the exact rounds,
// DESIGN.md §3.4).  Host and device: tools/mincheck.cpp checks the properties the search
// relies on (lower bound, >= 1, monotone, exact re-encoding, the bound kept when a dump
// moves a search between tables of different codes) over every code and 2^32 lengths.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace otr {

// minin(node) as stored in the search table: 16-mm units rounded down, saturating at
// 65535 (1.05 km).  A lower bound of the shortest in-edge keeps the IN criterion exact.
__host__ __device__ inline uint16_t mi_of(uint32_t m) { return (uint16_t)((m >> 4) < 65535u ? (m >> 4) : 65535u); }
// the IN criterion's margin of a node: any later offer is >= kmin + this (every edge >= 1 mm)
__host__ __device__ inline uint32_t in_gap(uint16_t mq) { return mq ? (uint32_t)mq << 4 : 1u; }
// The same in one byte (the large retry tables, whose LDS bytes per slot set their
// occupancy): a 4-bit exponent, 4-bit mantissa float of 16-mm units, rounded down (>= 94 %
// of the length, up to 8 km): code c < 16 is c units, else (16 + c % 16) << (c / 16 - 1).
__host__ __device__ inline uint8_t mf8_of(uint32_t m) {
  const uint32_t u = m >> 4;
  if (u < 16u) return (uint8_t)u;
  const int e = 27 - __builtin_clz(u);  // u in [2^(e+4), 2^(e+5)); u >= 16 (one count for host and device)
  if (e > 14) return 255;
  return (uint8_t)(((e + 1) << 4) | ((u >> e) & 15u));
}
__host__ __device__ inline uint32_t mf8_gap(uint8_t c) {
  const uint32_t u = c < 16u ? (uint32_t)c : (16u | (c & 15u)) << ((c >> 4) - 1);
  return u ? u << 4 : 1u;
}

}  // namespace otr
