// otr_launch.h — the launch plan of the per-state and per-trace kernels of one batch
// (host only, no HIP types: tests/test_lib.py checks it on the CPU through
// otr_launch_max_items).
//
// A dispatch counts its work-items in 32 bits.  The per-state kernels give every state a
// wave (k_candidates, k_prep<1>, k_tasks<1>: 64 work-items per state; k_candidates rounds
// the state count up to whole 8-wave XCD groups), the per-trace kernels every trace a wave
// (k_link, k_segments, k_histogram, k_tile_rows, k_compact).  Every one of them is
// launched with the grid below, and a batch is accepted only when the widest launch of a
// batch of that many probes (states <= probes, traces <= probes) stays below 2^32
// work-items: kMaxBatchProbes = 2^26 - 64.  The route, Viterbi and path tiers are
// persistent or piecewise (their grids do not grow with the batch).
#pragma once
#include <cstdint>

namespace otr {

struct Grid {
  uint64_t blocks;
  uint32_t threads;
  uint64_t items() const { return blocks * (uint64_t)threads; }
};

inline uint64_t div_up(int64_t n, int64_t d) { return n <= 0 ? 0 : (uint64_t)((n + d - 1) / d); }

// K1 k_candidates: one 64-lane wave per state, states in groups of 8 (one per XCD)
inline Grid grid_candidates(int64_t S) { return Grid{8 * div_up(S, 8), 64}; }
// K2 k_prep / k_tasks: 4 waves per block, one state per wave (G = 1) or two (G = 2)
inline Grid grid_per_state_waves(int64_t S, int G) { return Grid{div_up(div_up(S, G), 4), 256}; }
// k_link: one wave per trace, 4 per block
inline Grid grid_link(int64_t T) { return Grid{div_up(T, 4), 256}; }
// k_segments: one wave per trace, groups of 8 traces (XCD-mapped)
inline Grid grid_segments(int64_t T) { return Grid{8 * div_up(T, 8), 64}; }
// k_histogram / k_tile_rows: kTraceWaves (4) traces per 256-thread block
inline Grid grid_trace_rows(int64_t T) { return Grid{div_up(T, 4), 256}; }
// k_compact: one 64-lane block per trace
inline Grid grid_compact(int64_t T) { return Grid{T > 0 ? (uint64_t)T : 0, 64}; }
// k_paths first tier: two searches per wave, steps <= states
inline Grid grid_paths(int64_t S) { return Grid{8 * div_up(div_up(S, 2), 8), 64}; }

// the most work-items any per-state / per-trace launch of a batch with S states and T
// traces dispatches (G: states per wave of k_prep / k_tasks)
inline uint64_t max_launch_items(int64_t S, int64_t T, int G) {
  const uint64_t c[] = {grid_candidates(S).items(), grid_per_state_waves(S, G).items(), grid_link(T).items(),
                        grid_segments(T).items(),  grid_trace_rows(T).items(),         grid_compact(T).items(),
                        grid_paths(S).items()};
  uint64_t m = 0;
  for (uint64_t v : c) m = v > m ? v : m;
  return m;
}

constexpr uint64_t kMaxDispatchItems = 0xFFFFFFFFull;  // 32-bit work-item count per dispatch
constexpr int64_t kMaxBatchProbes = (1ll << 26) - 64;   // otr_match_batch (include/otr.h)
static_assert((uint64_t)64 * 8 * (((uint64_t)kMaxBatchProbes + 7) / 8) <= kMaxDispatchItems,
              "the widest per-state launch of a full batch fits one dispatch");

}  // namespace otr
