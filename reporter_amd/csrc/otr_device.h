// otr_device.h — device-side views, parameters and deterministic geometry shared by
// the HIP kernels (otr_kernels.hip) and the host engine (otr_engine.hip).
//
// Floating-point contract: everything on a decision path is IEEE
// binary64 +,-,*,/,sqrt compiled with -ffp-contract=off, and cos() is the fixed
// Taylor polynomial below, so the kernels reproduce the CPU oracle bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/otr_graph_format.h"

#define OTR_KMAX 64          // candidate slots per state (lanes of one wave)
#define OTR_MODES 3          // auto, bicycle, pedestrian
#define OTR_WAVE 64
#define OTR_COUNTERS 24      // counter kinds, see otr_batch_result.counters

namespace otr {

constexpr double kMetersPerDeg = 20037581.187 / 180.0;  // Batch.java:36

struct MatchParams {          // one per travel mode (meili.default + meili.<mode>)
  double sigma_z;             // Dockerfile:14
  double beta;                // Dockerfile:15
  double max_route_distance_factor;  // Dockerfile:16
  double breakage_distance;
  double interpolation_distance;
  double search_radius;
  double max_search_radius;
  double gps_accuracy;
  double max_route_time_factor;  // Dockerfile:17,48 (2): route time <= factor * dt
  double turn_penalty_factor;    // per mode, valhalla_build_config: auto 200, bicycle 140, pedestrian 100
  double speed_kph;           // mode speed cap for route times (0 = edge speed); fixed at configure
  double queue_kph;           // queue_length speed threshold (README.md:283,295)
  double inv2s2;              // 1 / (sigma_z * sigma_z * 2)
  double inv_beta;            // 1 / beta
  int32_t kmax;               // max_candidates <= OTR_KMAX
  int32_t pad;
};

struct ModeParams {
  MatchParams m[OTR_MODES];
  double delta;               // distance-bucket width of the routing search (metres)
};

// Route-label limits shared with the oracle (oracle/oracle.h ORC_*)
constexpr double kMaxBreakage = 30000.0;  // metres: route lengths <= 3e7 mm
constexpr int64_t kTbMax = 131070;        // larger time bounds are not applied (route times < 2^17)
constexpr uint32_t kTcCap = 2097151;      // routes whose turn cost exceeds this are pruned (mm, 21 bits)

// the step's time bound in 0.1 s from the states' time difference, -1 = none (oracle step_ctx)
__host__ __device__ inline int32_t time_bound_ds(const MatchParams& p, int64_t dt) {
  if (!(p.max_route_time_factor > 0.0) || dt <= 0) return -1;
  const double b = floor(p.max_route_time_factor * (double)dt * 10.0);
  return b <= (double)kTbMax ? (int32_t)b : -1;
}

// turn degree from in-edge a (end heading ha) into out-edge b (begin heading hb): the
// angle between the heading back along a and out along b, 0 (U-turn) .. 180 (straight).
// Headings are integer degrees 0..359 (seg_heading), so the wraps are one compare each
// (the oracle's `% 360` form, oracle.c turn_degree, gives the same value on that range).
__host__ __device__ inline int turn_from_back(int back, int hb_begin) {  // back = the in-edge's reversed heading
  int td = hb_begin - back;
  td += td < 0 ? 360 : 0;
  return td <= 180 ? td : 360 - td;
}
__host__ __device__ inline int heading_back(int ha_end) { return ha_end >= 180 ? ha_end - 180 : ha_end + 180; }
__host__ __device__ inline int turn_degree(int ha_end, int hb_begin) {
  return turn_from_back(heading_back(ha_end), hb_begin);
}

struct DevGraph {
  const uint32_t* node_row;
  const uint32_t* rev_row;
  const uint32_t* rev_edge;
  const uint32_t* edge_src;
  const uint32_t* edge_dst;
  const float* edge_len;
  const uint32_t* edge_attr;
  const uint32_t* edge_shape;
  const uint32_t* edge_seg;
  const uint32_t* edge_way;
  const int2* shape_ll;        // (lat_e6, lon_e6)
  const unsigned long long* seg_id;
  const uint32_t* seg_len;
  const uint32_t* cell_row;
  const uint32_t* cell_edge;
  const uint4* cell_rec;       // per cell entry 3 x 16 B: {edge, shape begin, shape end, attr}, shape points 0-1, 2-3
  const uint4* edge_pack;      // {dst, len_mm, attr, minin(dst)}: one 16-B load per relaxed edge (CSR tail)
  const uint4* eprep;          // {len_mm, src, minin(src), dst}: a candidate edge's terms in one load (k_prep)
  const uint4* adj;            // 4 x uint4 per node: {dst | access<<28 | more<<31, len_mm, minin(dst), 0}
  const uint32_t* node_minin;  // per node: its shortest in-edge, mm (0xFFFFFFFF: none), the IN criterion
  const uint32_t* len_mm;      // routing length, whole millimetres
  const int2* node_ll;         // (lat_e6, lon_e6)
  const uint32_t* adj_t;       // [mode][4 per node like adj]: route time of the slot's edge, 0.1 s
  const uint32_t* edge_t;      // [mode][edge]: route time, 0.1 s
  uint32_t adj_t_stride, edge_t_stride;  // elements per mode
  const short2* edge_head;     // per edge {begin heading, end heading}, integer degrees
  const uint2* adj_e;          // 4 per node like adj: {edge id, begin heading | end heading << 16} (edge-state searches)
  const uint4* erec;           // [4 per edge state b]: b's out-edge slots {e | access | more, len_mm, turn degree b -> e
                               // | end heading of b << 8, dst(b)} (otr_edge1.h, the edge-state search)
  const uint32_t* erec_t;      // [mode][4 per edge state]: the slot's route time, 0.1 s (saturated at 2^17 - 1)
  size_t erec_stride;          // records per mode of erec_t
  uint32_t n_nodes, n_edges, n_segments, grid_rows, grid_cols;
  double grid_min_lat, grid_min_lon, grid_cell_deg;
  __device__ const uint32_t* et(int mode) const { return edge_t + (size_t)mode * edge_t_stride; }
};

// cos of an angle in degrees, |deg| <= 90: Taylor series to x^22 (Horner).
__host__ __device__ inline double cos_deg(double deg) {
  double x = deg * (3.14159265358979323846 / 180.0);
  double x2 = x * x;
  double r = -1.0 / 1124000727777607680000.0;
  r = r * x2 + 1.0 / 2432902008176640000.0;
  r = r * x2 - 1.0 / 6402373705728000.0;
  r = r * x2 + 1.0 / 20922789888000.0;
  r = r * x2 - 1.0 / 87178291200.0;
  r = r * x2 + 1.0 / 479001600.0;
  r = r * x2 - 1.0 / 3628800.0;
  r = r * x2 + 1.0 / 40320.0;
  r = r * x2 - 1.0 / 720.0;
  r = r * x2 + 1.0 / 24.0;
  r = r * x2 - 1.0 / 2.0;
  r = r * x2 + 1.0;
  return r;
}

// equirectangular distance in metres (Batch.java:37-41, lat/lon in binary64)
__host__ __device__ inline double gc_dist(double lat1, double lon1, double lat2, double lon2) {
  double x = (lon1 - lon2) * kMetersPerDeg * cos_deg(0.5 * (lat1 + lat2));
  double y = (lat1 - lat2) * kMetersPerDeg;
  return sqrt(x * x + y * y);
}

__host__ __device__ inline double e6(int32_t v) { return (double)v * 1e-6; }

// route bound B = min(breakage, factor * max(g, interpolation_distance))  
__host__ __device__ inline double route_bound(const MatchParams& p, double g) {
  double gf = g > p.interpolation_distance ? g : p.interpolation_distance;
  double b = p.max_route_distance_factor * gf;
  return b > p.breakage_distance ? p.breakage_distance : b;
}

__device__ inline uint32_t hmix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ inline int lane_id() { return (int)__lane_id(); }

// Blocks are dealt round-robin over the 8 XCDs (b and b+8 share one, MI355X_MICROARCH.md
// §Workgroup dispatch): give each XCD a contiguous run of logical work items so that
// neighbouring items (same trace / same step → same graph neighbourhood) share an L2.
// Speed only; any placement gives the same results.  grid = 8 * per.
__device__ inline int64_t xcd_remap(int64_t b, int64_t per) { return (b & 7) * per + (b >> 3); }

// A dynamic work queue over a list of n units split into 8 contiguous ranges, one per XCD
// (the dispatcher deals workgroups to XCDs round robin by blockIdx.x % 8): a one-wave
// workgroup claims its range's next unit with one atomic on its XCD's counter (counters
// 128 B apart, zeroed before the launch).  A wave that drew short searches takes more of
// them, and the grid may hold any number of resident waves: a fixed stride over a grid
// larger than the resident waves runs in generations whose last one can be a small tail.
struct XcdQueue {
  int64_t lo, hi;
  unsigned long long* ctr;
  __device__ XcdQueue(unsigned long long* q, int64_t n) {
    // (a grid of fewer than 8 workgroups would leave ranges unclaimed: one range then)
    const int parts = gridDim.x >= 8 ? 8 : 1;
    const int x = parts == 8 ? (int)(blockIdx.x & 7) : 0;
    const int64_t per = (n + parts - 1) / parts;
    lo = (int64_t)x * per;
    hi = lo + per < n ? lo + per : n;
    ctr = q + 16 * x;
  }
  // claim(): the atomic, its result in lane 0 (not waited for); take(): the claimed unit
  __device__ unsigned long long claim() {
    unsigned long long v = 0;
    if (threadIdx.x == 0) v = atomicAdd(ctr, 1ull);
    return v;
  }
  __device__ int64_t take(unsigned long long v) const {
    const uint32_t l = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return lo + (int64_t)(((unsigned long long)h << 32) | l);
  }
  __device__ int64_t next() { return take(claim()); }  // (wave-uniform; one-wave workgroups)
};

// One 16-B load whose four words are all materialised here: keeps the compiler from
// splitting a record load into dependent pieces sunk into the branches that use them.
__device__ inline uint4 ld16(const uint4* p) {
  uint4 r = *p;
  asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w));
  return r;
}

constexpr int kShards = 64;  // path-buffer regions and bump cursors are sharded 64 ways
// device work counters: [bank][kind][kCShards], a wave adds to shard blockIdx % kCShards.
// 256 shards spread one kind over 16 cache lines: with 64 (4 lines a kind) the route
// kernels' end-of-wave atomics queued on the L2 lines (k_route<160,2> 15.1 -> 13.9 ms
// without them, tools/ab_libs.sh); k_ctr_reduce folds the shards before the copy-out.
constexpr int kCShards = 256;
__device__ inline int cshard() { return (int)(blockIdx.x & (kCShards - 1)); }
constexpr uint32_t kAdjDstMask = 0x0FFFFFFFu;
constexpr uint32_t kAdjMore = 0x80000000u;

__device__ inline int prefix_count(unsigned long long mask) {
  // set bits of `mask` below my lane: v_mbcnt_lo + v_mbcnt_hi (two VALU ops instead of a
  // 64-bit shift, two masks and two bit counts)
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace otr
