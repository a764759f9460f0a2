// otr_kernels.h — the HIP kernels of the matching hot path (gfx950, wave64).
//
//   K0 k_select_states   thread/trace   interpolation_distance state selection
//   K1 k_candidates      wave/state     grid-cell edge projection, LDS top-K
//   K2 (emission)        fused into K5  sq_dist / (2 sigma_z^2)
//   K_link               wave/trace     active-state chain, g, route bound
//   K3 k_route           wave/(step,src) bounded one-to-many search, LDS hash
//   K4 (transition)      epilogue of K3 |route - g| / beta
//   K5 k_viterbi         group/trace    fp64 min-sum Viterbi + backtrack (2 traces per wave)
//   K6 k_paths           group/step     winner path reconstruction
//   K7 k_segments        wave/trace     route stitch, OSMLR segments, report()
//   K8 k_histogram       thread/trace   simple_reporter filter + hour buckets
//
// Every decision-path expression mirrors oracle/oracle.c operation for operation
// (DESIGN.md §3); the tests compare the two bit for bit.
#pragma once
#include <cstddef>
#include <type_traits>

#include "otr_device.h"
#include "otr_mincode.h"  // IN-gap codes of the node tables (mi_of / in_gap, mf8_of / mf8_gap)
#include "otr_report.h"

// the first tier's table (slots per search, two searches per wave) and its load limit in
// eighths (A/B knobs)
#ifndef OTR_CAP1
#define OTR_CAP1 160
#endif
#ifndef OTR_LOAD1
#define OTR_LOAD1 7
#endif
// the lean first edge-state tier's table (otr_edge1.h): 360 states with a 32-state settled
// list and 16 relax scratch words, 10.1 KB of LDS, 16 waves per CU (c2dep with work queues:
// branching relax at 368 states 5.71M, 384 at 15 waves 5.35M; branch-free relax at 360
// states 6.12M probes/s); its load limit in sixteenths (14: 7/8; 15: slower)
#ifndef OTR_E1CAP
#define OTR_E1CAP 360
#endif
#ifndef OTR_E1LOAD
#define OTR_E1LOAD 14
#endif

namespace otr {

struct BatchDev {
  int32_t n_traces;
  const int64_t* trace_off;
  const double* lat;
  const double* lon;
  const int64_t* time;
  const float* acc;
  const uint8_t* mode;
};

// ------------------------------------------------------------------------------
// K0: state selection (thread per trace).  Pass 1 counts, pass 2 writes.
// ------------------------------------------------------------------------------
__global__ void k_select_states(BatchDev b, ModeParams mp, int64_t* state_cnt, const int64_t* state_off,
                                int64_t* state_probe, int32_t* state_trace) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= b.n_traces) return;
  const int64_t lo = b.trace_off[t], hi = b.trace_off[t + 1];
  const MatchParams& P = mp.m[b.mode[t] < OTR_MODES ? b.mode[t] : 0];
  int64_t cnt = 0;
  int64_t base = state_off ? state_off[t] : 0;
  // the last state's coordinates stay in registers and the next probe's are loaded one
  // iteration ahead: the loop's only dependence is the distance test itself
  double la_last = 0.0, lo_last = 0.0;
  double la_n = lo < hi ? b.lat[lo] : 0.0, lo_n = lo < hi ? b.lon[lo] : 0.0;
  for (int64_t i = lo; i < hi; ++i) {
    const double la = la_n, lg = lo_n;
    if (i + 1 < hi) {
      la_n = b.lat[i + 1];
      lo_n = b.lon[i + 1];
    }
    const bool st = (i == lo || i == hi - 1) || gc_dist(la_last, lo_last, la, lg) >= P.interpolation_distance;
    if (st) {
      if (state_off) {
        state_probe[base + cnt] = i;
        state_trace[base + cnt] = t;
      }
      ++cnt;
      la_last = la;
      lo_last = lg;
    }
  }
  if (!state_off) state_cnt[t] = cnt;
}

// ------------------------------------------------------------------------------
// K1: candidate search, one wave (block of 64) per state.
// ------------------------------------------------------------------------------
struct CandBuf {
  uint32_t* edge;   // [n_states][OTR_KMAX]
  double* p;
  double* sqd;
  int32_t* count;
  double* radius;   // per state search radius
};

__device__ inline bool cand_less(double da, uint32_t ea, double db, uint32_t eb) {
  return da < db || (da == db && ea < eb);
}

// Projection of probe (plat, plon) onto edge e's polyline in the probe-local metric;
// true when the edge is a candidate owned by grid cell (r, c) (the cell holding the
// snapped point), with squared distance d2 and fraction along the edge.
// rec = the cell entry's {edge, first shape point, end shape point, attr}, pts01/pts23 its
// first four shape points (DevGraph::cell_rec, 48 B per entry).
// Returns the grid cell (sr, sc) of the snapped point through *sr/*sc.
__device__ inline bool project_edge(const DevGraph& g, uint4 rec, uint4 pts01, uint4 pts23, uint32_t mode_bit,
                                    double plat, double plon, double mpl, double r2, int64_t* sr_out, int64_t* sc_out,
                                    double* d2_out, double* frac_out, unsigned long long* tests) {
  if (!(rec.w & mode_bit)) return false;
  double best = __builtin_huge_val();
  double best_along = 0.0, bqx = 0.0, bqy = 0.0, acc = 0.0;
  const uint32_t k0 = rec.y, k1 = rec.z;
  // the first kPre shape points travel in the cell record itself (DevGraph::cell_rec:
  // no dependent shape load for edges of up to 4 points — every edge of the synthetic
  // graphs); longer polylines continue point by point from shape_ll
  constexpr uint32_t kPre = 4;
  const int2 pre0 = make_int2((int)pts01.x, (int)pts01.y);
  int2 q1 = make_int2((int)pts01.z, (int)pts01.w);
  int2 q2 = make_int2((int)pts23.x, (int)pts23.y);
  int2 q3 = make_int2((int)pts23.z, (int)pts23.w);
  int2 pa = pre0;
  for (uint32_t k = k0; k + 1 < k1; ++k) {
    const uint32_t i = k + 1 - k0;
    int2 pb;
    if (i < kPre) {
      pb = q1;
      q1 = q2;
      q2 = q3;
    } else {
      pb = g.shape_ll[k + 1];
    }
    const double ax = (e6(pa.y) - plon) * mpl;
    const double ay = (e6(pa.x) - plat) * kMetersPerDeg;
    const double bx = (e6(pb.y) - plon) * mpl;
    const double by = (e6(pb.x) - plat) * kMetersPerDeg;
    const double dx = bx - ax, dy = by - ay;
    const double l2 = dx * dx + dy * dy;
    double t = 0.0;
    if (l2 > 0.0) {
      t = -(ax * dx + ay * dy) / l2;
      if (t < 0.0) t = 0.0;
      if (t > 1.0) t = 1.0;
    }
    const double qx = ax + t * dx, qy = ay + t * dy;
    const double d2 = qx * qx + qy * qy;
    const double sl = sqrt(l2);
    if (d2 < best) {
      best = d2;
      best_along = acc + t * sl;
      bqx = qx;
      bqy = qy;
    }
    acc = acc + sl;
    pa = pb;
  }
  *tests += k1 - k0 - 1;
  if (!(best <= r2)) return false;
  const double slat = plat + bqy / kMetersPerDeg, slon = plon + bqx / mpl;
  *sr_out = (int64_t)floor((slat - g.grid_min_lat) / g.grid_cell_deg);
  *sc_out = (int64_t)floor((slon - g.grid_min_lon) / g.grid_cell_deg);
  *d2_out = best;
  *frac_out = acc > 0.0 ? best_along / acc : 0.0;
  return true;
}

// Wave sum (mod 2^32) by DPP row shifts and row broadcasts, result read from lane 63.
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Wave minimum by DPP row shifts and row broadcasts (GFX9), result read from lane 63.
__device__ inline uint32_t wave_min_u32(uint32_t v) {
  const int I = -1;
  auto mn = [](uint32_t a, int b) { return a < (uint32_t)b ? a : (uint32_t)b; };
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// G independent searches per wave, GL = 64 / G lanes each (G = 1, 2, 4 or 8).  Per-group
// ballots, prefix counts, minima and wave-uniform loop bounds.
template <int G>
struct Grp {
  static constexpr int GL = OTR_WAVE / G;
  __device__ static int g() { return G == 1 ? 0 : (int)threadIdx.x / GL; }
  __device__ static int gl() { return G == 1 ? (int)threadIdx.x : (int)threadIdx.x % GL; }
  __device__ static unsigned long long mine(unsigned long long m) {
    return G == 1 ? m : (m >> (GL * g())) & ((1ull << GL) - 1ull);
  }
  // my group's set bits below my lane (G = 1: mbcnt, prefix_count)
  __device__ static int prefix(unsigned long long m) {
    if (G == 1) return prefix_count(m);
    return __popcll(mine(m) & ((1ull << gl()) - 1ull));
  }
  __device__ static int count(unsigned long long m) { return __popcll(mine(m)); }
  // maximum over groups of a group-uniform value (a wave-uniform loop bound)
  __device__ static int umax(int v) {
    if (G == 1) return __builtin_amdgcn_readfirstlane(v);
    if (G == 8) {
      int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
      for (int q = 1; q < 8; ++q) {
        const int x = __builtin_amdgcn_readlane(v, q * GL);
        m = x > m ? x : m;
      }
      return m;
    }
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, GL);
    if (G == 2) return a > b ? a : b;
    const int c = __builtin_amdgcn_readlane(v, 2 * GL), d = __builtin_amdgcn_readlane(v, 3 * GL);
    const int ab = a > b ? a : b, cd = c > d ? c : d;
    return ab > cd ? ab : cd;
  }
  __device__ static bool all(bool v) {
    if (G == 1) return __builtin_amdgcn_readfirstlane((int)v) != 0;
    if (G == 8) {
      bool r = true;
#pragma unroll
      for (int q = 0; q < 8; ++q) r = r && __builtin_amdgcn_readlane((int)v, q * GL) != 0;
      return r;
    }
    const bool ab = __builtin_amdgcn_readlane((int)v, 0) != 0 && __builtin_amdgcn_readlane((int)v, GL) != 0;
    if (G == 2) return ab;
    return ab && __builtin_amdgcn_readlane((int)v, 2 * GL) != 0 && __builtin_amdgcn_readlane((int)v, 3 * GL) != 0;
  }
  __device__ static uint32_t min_u32(uint32_t v) {
    if (G == 1) return wave_min_u32(v);
    if (G == 8) {  // (8-lane groups: a butterfly of lane swaps within the group)
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        const uint32_t x = (uint32_t)__shfl_xor((int)v, o, 8);
        v = x < v ? x : v;
      }
      return v;
    }
    const int I = -1;
    auto mn = [](uint32_t a, int b) { return a < (uint32_t)b ? a : (uint32_t)b; };
    v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    if (G == 4) {  // a group is one DPP row: lane 15 of the row holds its minimum
      const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
      const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
      const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
      const int q = g();
      return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
    }
    v = mn(v, __builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return g() ? b : a;
  }
};

constexpr int kWin = 16;  // flattened cell windows up to 16 x 16 cells
// waves per SIMD of the two-states-per-wave candidate search (its registers)
#ifndef OTR_CAND2_WAVES
#define OTR_CAND2_WAVES 5
#endif

// K1: G states per wave (lane groups of GL = 64 / G; G = 2 when every mode keeps at most
// 32 candidates: the search is a chain of dependent loads — probe, cell window, cell
// records — so two states per wave keep twice the chains in flight).  Every loop runs to
// the longer group's trip count (a group past its own idles), so the wave stays converged.
template <int G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(G == 2 ? OTR_CAND2_WAVES : 8, 8))) void k_candidates(
    DevGraph g, BatchDev b, ModeParams mp, int64_t n_states, const int64_t* state_probe, const int32_t* state_trace,
    CandBuf out, unsigned long long* counters) {
  using Gr = Grp<G>;
  constexpr int GL = Gr::GL;
  constexpr int LB = 2 * GL;                  // candidate list (<= kmax + GL entries), one buffer:
  __shared__ double s_d2[G][LB];              // compaction stages each lane's <= 2 entries in registers
  __shared__ double s_p[G][LB];
  __shared__ uint32_t s_e[G][LB];
  __shared__ uint32_t s_bnd[G][kWin][kWin + 1];  // cell_row boundaries of the window, per row
  __shared__ uint32_t s_pre[G][kWin + 1];        // entries before each row
  const int gi = Gr::g(), lane = Gr::gl();
  const int64_t n_units = (n_states + G - 1) / G;
  const int64_t s = xcd_remap(blockIdx.x, (n_units + 7) / 8) * G + gi;
  if (Gr::umax(s < n_states ? 1 : 0) == 0) return;  // (wave-uniform)
  const bool have = s < n_states;
#ifdef OTR_STAMPS_CAND
  const unsigned long long cs0 = __builtin_amdgcn_s_memtime();
  unsigned long long cs1 = cs0, cs2 = cs0;
#endif
  const int64_t probe = have ? state_probe[s] : 0;
  const int mode = have && b.mode[state_trace[s]] < OTR_MODES ? b.mode[state_trace[s]] : 0;
  // the mode's parameters by selects (G = 2: the mode is a per-group register, and a
  // register-indexed kernel argument would go through scratch)
  auto pick = [&](auto f) { return mode == 0 ? f(mp.m[0]) : (mode == 1 ? f(mp.m[1]) : f(mp.m[OTR_MODES - 1])); };
  const uint32_t mode_bit = 1u << mode;
  const int kmax = pick([](const MatchParams& q) { return q.kmax; });
  const double plat = b.lat[probe], plon = b.lon[probe];
  const double a = (b.acc && b.acc[probe] >= 0.f) ? (double)b.acc[probe]
                                                  : pick([](const MatchParams& q) { return q.gps_accuracy; });
  const double sr0 = pick([](const MatchParams& q) { return q.search_radius; });
  const double srmax = pick([](const MatchParams& q) { return q.max_search_radius; });
  double radius = sr0 > a ? sr0 : a;
  if (radius > srmax) radius = srmax;
  const double mpl = kMetersPerDeg * cos_deg(plat);
  const double cd = g.grid_cell_deg;
  const double dlat = radius / kMetersPerDeg, dlon = radius / mpl;
  int64_t r0 = (int64_t)floor((plat - dlat - OTR_GRID_PAD_DEG - g.grid_min_lat) / cd);
  int64_t r1 = (int64_t)floor((plat + dlat + OTR_GRID_PAD_DEG - g.grid_min_lat) / cd);
  int64_t c0 = (int64_t)floor((plon - dlon - OTR_GRID_PAD_DEG - g.grid_min_lon) / cd);
  int64_t c1 = (int64_t)floor((plon + dlon + OTR_GRID_PAD_DEG - g.grid_min_lon) / cd);
  if (r0 < 0) r0 = 0;
  if (c0 < 0) c0 = 0;
  if (r1 > (int64_t)g.grid_rows - 1) r1 = (int64_t)g.grid_rows - 1;
  if (c1 > (int64_t)g.grid_cols - 1) c1 = (int64_t)g.grid_cols - 1;
  const double r2 = radius * radius;
  int n = 0;
  unsigned long long tests = 0;
  double* L_d2 = s_d2[gi];
  double* L_p = s_p[gi];
  uint32_t* L_e = s_e[gi];
  // merge one pass's qualifying candidates into the group's LDS top-K list (every lane of
  // the wave calls it: the barriers are the wave's)
  auto merge = [&](bool ok, double d2, double frac, uint32_t e) {
    const unsigned long long mask = __ballot(ok);
    if (!mask) return;
    if (ok) {
      const int pos = n + Gr::prefix(mask);
      L_d2[pos] = d2;
      L_p[pos] = frac;
      L_e[pos] = e;
    }
    n += Gr::count(mask);
    __syncthreads();
    if (Gr::umax(n > kmax ? 1 : 0)) {  // rank-compact to the kmax best (all (d2, edge) keys distinct)
      double dv[2], pv[2];
      uint32_t ev[2];
      int rk[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int idx = lane + h * GL;
        rk[h] = OTR_KMAX * 2;
        if (n > kmax && idx < n) {
          dv[h] = L_d2[idx];
          pv[h] = L_p[idx];
          ev[h] = L_e[idx];
          int rank = 0;
          for (int m = 0; m < n; ++m) rank += cand_less(L_d2[m], L_e[m], dv[h], ev[h]);
          rk[h] = rank;
        }
      }
      __syncthreads();
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (rk[h] < kmax) {
          L_d2[rk[h]] = dv[h];
          L_p[rk[h]] = pv[h];
          L_e[rk[h]] = ev[h];
        }
      __syncthreads();
      n = n > kmax ? kmax : n;
    }
  };
  const int nr = (int)(r1 - r0 + 1), nc = (int)(c1 - c0 + 1);
  const bool win = have && nr >= 1 && nc >= 1 && nr <= kWin && nc <= kWin;
  const bool slow = have && !win && nr >= 1 && nc >= 1;  // (a window past kWin cells: cell by cell)
  if (Gr::umax(win ? 1 : 0)) {
    // The cells of one grid row are contiguous in cell_edge: flatten the window into
    // one entry range per row and sweep all rows with full lane groups.
    const int nb = win ? nr * (nc + 1) : 0;
    const int nbx = Gr::umax(nb);
    for (int idx = lane; idx < nbx; idx += GL) {
      if (idx < nb) {
        const int rr = idx / (nc + 1), cc = idx % (nc + 1);
        s_bnd[gi][rr][cc] = g.cell_row[(r0 + rr) * (int64_t)g.grid_cols + c0 + cc];
      }
    }
    __syncthreads();
    if (win && lane == 0) {
      uint32_t acc = 0;
      for (int rr = 0; rr < nr; ++rr) {
        s_pre[gi][rr] = acc;
        acc += s_bnd[gi][rr][nc] - s_bnd[gi][rr][0];
      }
      s_pre[gi][nr] = acc;
    }
    __syncthreads();
#ifdef OTR_STAMPS_CAND
    cs1 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t total = win ? s_pre[gi][nr] : 0u;
    const uint32_t totx = (uint32_t)Gr::umax((int)total);
    for (uint32_t base = 0; base < totx; base += GL) {
      const uint32_t k = base + lane;
      bool ok = false;
      double d2 = 0, frac = 0;
      uint4 rec = make_uint4(0u, 0u, 0u, 0u);
      if (k < total) {
        int rr = 0;
        while (rr + 1 < nr && s_pre[gi][rr + 1] <= k) ++rr;
        const uint32_t q = s_bnd[gi][rr][0] + (k - s_pre[gi][rr]);
        rec = ld16(g.cell_rec + 3 * (size_t)q);
        const uint4 p01 = ld16(g.cell_rec + 3 * (size_t)q + 1), p23 = ld16(g.cell_rec + 3 * (size_t)q + 2);
        int64_t sr, sc;
        ok = project_edge(g, rec, p01, p23, mode_bit, plat, plon, mpl, r2, &sr, &sc, &d2, &frac, &tests);
        // owned by the cell holding the snapped point: entry q lies in that cell's range
        if (ok) {
          const int64_t wr = sr - r0, wc = sc - c0;
          ok = wr >= 0 && wr < nr && wc >= 0 && wc < nc && s_bnd[gi][wr][wc] <= q && q < s_bnd[gi][wr][wc + 1];
        }
      }
      merge(ok, d2, frac, rec.x);
    }
#ifdef OTR_STAMPS_CAND
    cs2 = __builtin_amdgcn_s_memtime();
#endif
  }
  if (Gr::umax(slow ? 1 : 0)) {
    // cell by cell (the longer group's cell count; entries of a cell by passes of GL lanes)
    const int ncell = slow ? nr * nc : 0;
    const int ncx = Gr::umax(ncell);
    for (int ci = 0; ci < ncx; ++ci) {
      const bool act = ci < ncell;
      const int64_t r = r0 + (act ? ci / nc : 0), c = c0 + (act ? ci % nc : 0);
      const uint32_t cell = (uint32_t)(r * g.grid_cols + c);
      const uint32_t beg = act ? g.cell_row[cell] : 0u, end = act ? g.cell_row[cell + 1] : 0u;
      const int cnt = (int)(end - beg), cntx = Gr::umax(cnt);
      for (int base = 0; base < cntx; base += GL) {
        const uint32_t q = beg + (uint32_t)(base + lane);
        bool ok = false;
        double d2 = 0, frac = 0;
        uint4 rec = make_uint4(0u, 0u, 0u, 0u);
        if (base + lane < cnt) {
          rec = ld16(g.cell_rec + 3 * (size_t)q);
          const uint4 p01 = ld16(g.cell_rec + 3 * (size_t)q + 1), p23 = ld16(g.cell_rec + 3 * (size_t)q + 2);
          int64_t sr, sc;
          ok = project_edge(g, rec, p01, p23, mode_bit, plat, plon, mpl, r2, &sr, &sc, &d2, &frac, &tests) &&
               sr == r && sc == c;
        }
        merge(ok, d2, frac, rec.x);
      }
    }
  }
  // final ordering
  if (have) {
    const size_t o = (size_t)s * OTR_KMAX;
    for (int idx = lane; idx < n; idx += GL) {
      const double d = L_d2[idx];
      const uint32_t ee = L_e[idx];
      int rank = 0;
      for (int m = 0; m < n; ++m) rank += cand_less(L_d2[m], L_e[m], d, ee);
      out.edge[o + rank] = ee;
      out.p[o + rank] = L_p[idx];
      out.sqd[o + rank] = d;
    }
    if (lane == 0) {
      out.count[s] = n;
      out.radius[s] = radius;
    }
  }
  for (int off = GL / 2; off > 0; off >>= 1) tests += __shfl_xor(tests, off);  // (within the group)
#ifdef OTR_STAMPS_CAND
  if (threadIdx.x == 0 && counters) {
    const unsigned long long cs3 = __builtin_amdgcn_s_memtime();
    const int sh = cshard();
    atomicAdd(&counters[16 * kCShards + sh], cs1 - cs0);
    atomicAdd(&counters[17 * kCShards + sh], cs2 - cs1);
    atomicAdd(&counters[18 * kCShards + sh], cs3 - cs2);
  }
#endif
  if (have && lane == 0 && counters) {
    const int sh = cshard();
    atomicAdd(&counters[0 * kCShards + sh], (unsigned long long)((r1 - r0 + 1) * (c1 - c0 + 1)));
    atomicAdd(&counters[1 * kCShards + sh], tests);
    atomicAdd(&counters[2 * kCShards + sh], (unsigned long long)n);
  }
}

// ------------------------------------------------------------------------------
// K_link: per trace, chain active states (K>0) into steps.
// ------------------------------------------------------------------------------
struct StepBuf {
  int64_t* prev;      // previous active state of the same trace, -1 none, -2 inactive
  double* g;          // great-circle distance prev→s
  double* bound;      // route bound
  uint8_t* forced;    // g > breakage_distance
  int32_t* bt;        // time bound of the step, 0.1 s (max_route_time_factor * dt), -1 none
  int64_t* ntask;     // search tasks of the step (k_tasks)
  int64_t* ntrans;    // K[prev]*K[s]
};

// One wave per trace, lane = state within a chunk of 64: the previous active state is
// the highest active lane below (ballot), or the last active state of earlier chunks —
// the trace's serial chain becomes one step per 64 states.
__global__ __launch_bounds__(256) void k_link(BatchDev b, ModeParams mp, const int64_t* trace_state_off,
                                              const int64_t* state_probe, const int32_t* cand_count, StepBuf st) {
  const int64_t t = (int64_t)blockIdx.x * (blockDim.x / OTR_WAVE) + threadIdx.x / OTR_WAVE;
  const int lane = threadIdx.x % OTR_WAVE;
  if (t >= b.n_traces) return;
  const MatchParams& P = mp.m[b.mode[t] < OTR_MODES ? b.mode[t] : 0];
  const int64_t so = trace_state_off[t], eo = trace_state_off[t + 1];
  int64_t last = -1;  // wave-uniform: last active state of the chunks before
  for (int64_t base = so; base < eo; base += OTR_WAVE) {
    const int64_t s = base + lane;
    const bool in = s < eo;
    const int K = in ? cand_count[s] : 0;
    const unsigned long long am = __ballot(K > 0);
    const unsigned long long below = am & ((1ull << lane) - 1ull);
    const int64_t pv = below ? base + (63 - __clzll((long long)below)) : last;
    if (in) {
      st.ntrans[s] = 0;
      st.bt[s] = -1;
      if (K <= 0) {
        st.prev[s] = -2;
      } else {
        st.prev[s] = pv;
        if (pv >= 0) {
          const int64_t ia = state_probe[pv], ib = state_probe[s];
          const double gcd = gc_dist(b.lat[ia], b.lon[ia], b.lat[ib], b.lon[ib]);
          st.g[s] = gcd;
          st.forced[s] = gcd > P.breakage_distance;
          st.bound[s] = route_bound(P, gcd);
          st.bt[s] = time_bound_ds(P, b.time[ib] - b.time[ia]);
          st.ntrans[s] = (int64_t)cand_count[pv] * K;
        }
      }
    }
    if (am) last = base + (63 - __clzll((long long)am));
  }
}

// One search task per (step, distinct search root).  Labels are rooted (label 0) at
// dst(e_i), so every source candidate whose edge ends at the same node shares the
// search; the task carries the bit mask of those sources.  The counts come from k_prep
// (PrepArgs::nroot, per state) through k_ntask; task_off == null counts here instead (the
// same number, a pass of its own).
// my lane group's bits of a wave ballot, for kernels whose blocks hold several waves
// (Grp<G> assumes one wave per block)
template <int G>
__device__ inline unsigned long long group_bits(unsigned long long m) {
  if (G == 1) return m;
  constexpr int GL = OTR_WAVE / G;
  const int gi = (int)(threadIdx.x % OTR_WAVE) / GL;
  return (m >> (GL * gi)) & ((1ull << GL) - 1ull);
}

// ------------------------------------------------------------------------------
// Bounded one-to-many search, one wave, node labels in an LDS hash table.
//
// The oracle's search is label-setting with pruning: a label is the
// minimum over the feasible offers of its predecessors' FINAL labels, and a time-pruned
// offer from a label that later improves would leave a withdrawn label behind, so the
// GPU search only ever relaxes final labels.  Rounds settle, in parallel, every pending
// node u whose label is provably final by the IN criterion: any later offer to u comes
// from a pending node (length >= kmin, the smallest pending length) through an in-edge
// of u (length >= minin(u)), so d(u) < kmin + max(1, minin(u)) makes (d, t) final.
// Lane = (settled node, adjacency slot); relaxation = LDS atomicMin.  Every offer comes
// from a final label, so labels, pruning and the predecessor rule equal the oracle's
// label-setting search whatever the round sizes.  With PRED the label word is
// (label << 32 | edge id) so the minimum also records the smallest-id predecessor
// edge among those achieving the label (the oracle's walk_path rule).
// ------------------------------------------------------------------------------
// Label word of a search table, by label mode LM: 0 the packed (length << sh | time) word
// in 32 bits; 1 (PRED) that word << 32 | the smallest predecessor edge; 2 (WIDE) the
// packed word in 64 bits, for steps whose length and time bits exceed 32 (long gaps
// between states).  W: the packed word as label() returns it.
template <int LM>
struct LabelT {
  using T = uint32_t;
  using W = uint32_t;
  static constexpr T kInf = 0xFFFFFFFFu;
  static constexpr W kNone = 0xFFFFFFFFu;
  __device__ static W label(T x) { return x; }
  __device__ static T make(W l, uint32_t) { return l; }
};
template <>
struct LabelT<1> {
  using T = unsigned long long;
  using W = uint32_t;
  static constexpr T kInf = 0xFFFFFFFFFFFFFFFFull;
  static constexpr W kNone = 0xFFFFFFFFu;
  __device__ static W label(T x) { return (uint32_t)(x >> 32); }
  __device__ static T make(W l, uint32_t e) { return ((unsigned long long)l << 32) | e; }
};
template <>
struct LabelT<2> {
  using T = unsigned long long;
  using W = unsigned long long;
  static constexpr T kInf = 0xFFFFFFFFFFFFFFFFull;
  static constexpr W kNone = 0xFFFFFFFFFFFFFFFFull;
  __device__ static W label(T x) { return x; }
  __device__ static T make(W l, uint32_t) { return l; }
};

// a settled node of this round: its id and the packed label it was settled with
template <class W>
struct WorkE {
  uint32_t node;
  W lab;
};


#ifndef OTR_PCAP1024
#define OTR_PCAP1024 512
#endif
#ifndef OTR_PCAP2048
#define OTR_PCAP2048 512
#endif
#ifndef OTR_PCAP448
#define OTR_PCAP448 448
#endif
#ifndef OTR_WCAP1024
#define OTR_WCAP1024 120
#endif
// settles per round of the small tier's 80-slot tables (four tables per wave in 32 waves'
// LDS: at most 28)
#ifndef OTR_WCAP4
#define OTR_WCAP4 16
#endif
template <int CAP, int LM>
struct SearchLds {
  static constexpr bool PRED = LM == 1;
  // one-byte minin codes (mf8) in the retry tables of 384..1024 slots: 11 B per slot
  // instead of 12 (C4: the 1024-slot tier 13 waves per CU instead of 12, 263.9 -> 257.0 ms;
  // 448x2 14 instead of 13, 21.5 -> 19.6 ms; the 2048-slot table keeps its 6 waves either
  // way and the 2-byte codes)
  static constexpr bool MI8 = CAP >= 384 && CAP <= 1024 && !PRED;
  using MiT = typename std::conditional<MI8, uint8_t, uint16_t>::type;
  __device__ static MiT code(uint32_t m) {
    if constexpr (MI8) return mf8_of(m);
    else return mi_of(m);
  }
  __device__ static uint32_t gap(MiT c) {
    if constexpr (MI8) return mf8_gap(c);
    else return in_gap(c);
  }
  using W = typename LabelT<LM>::W;
  typename LabelT<LM>::T lab[CAP];  // label (| pred edge)
  uint32_t key[CAP];                  // node id | INQ / REL bits, 0xFFFFFFFF empty
  MiT mi[CAP];                        // minin(node) code (mi_of, or mf8_of): the IN criterion's gap
  using Idx = typename std::conditional<(CAP <= 256 && !PRED), uint8_t, uint16_t>::type;
  // nodes settled per round (at most); k_paths (PRED) reuses pend + work as CAP u32 words
  // (1024 slots: 120, the 1-B codes' table then fits 13 waves per CU's LDS)
  // (the small tier's 80-slot tables: 16, so four tables fit 32 waves per CU: 4.5 KB per wave)
  static constexpr int WCAP = CAP <= 48 ? 8 : CAP <= 96 ? (PRED ? 20 : OTR_WCAP4) : CAP <= 160 ? 48 : (PRED ? CAP / 4 : (CAP <= 512 ? 64 : (CAP <= 1024 ? OTR_WCAP1024 : 128)));
  // pending list capacity: the 1024-slot table's may be shorter (OTR_PCAP1024: LDS for
  // more resident waves; a search whose frontier outgrows it restarts in the next table)
  static constexpr int PCAP = PRED ? CAP
                                    : (CAP == 1024 ? OTR_PCAP1024 : (CAP == 2048 ? OTR_PCAP2048 : (CAP == 448 ? OTR_PCAP448 : CAP)));
  Idx pend[PCAP];                     // pending slots (k_paths reuses pend+work as CAP u32)
  WorkE<W> work[WCAP];                // this round's settled nodes: {node, label}
  int n_pend, n_keys, overflow;
};

constexpr uint32_t kEmpty = 0xFFFFFFFFu;

constexpr uint32_t kInq = 0x80000000u;   // key bit: the node is on the pending list
constexpr uint32_t kRel = 0x40000000u;   // key bit: the node is settled (its label is final)
constexpr uint32_t kNodeMask = 0x0FFFFFFFu;
constexpr uint32_t kNoLabel = 0xFFFFFFFFu;
constexpr uint32_t kNoRoute = 0xFFFFFFFFu;  // transition array: no valid route within the bound

// Diagnostic build only (-DOTR_STAMPS): shader-clock stamps per search phase, summed
// into counter kinds 16..19.  The production build compiles them out.
#ifdef OTR_STAMPS
#define OTR_STAMP(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define OTR_STAMP(v) const unsigned long long v = 0
#endif

// routing bound and partial edge lengths in whole mm (shared with the oracle)
__device__ inline int64_t bound_mm_of(double bound) { return (int64_t)floor(bound * 1000.0); }
__device__ inline int64_t part_mm(double frac, uint32_t len_mm) { return (int64_t)llround(frac * (double)len_mm); }

// home slot: multiplicative hashing of the id's low 24 bits (the ids of one search are
// spatially clustered, nearly consecutive): bits 8..23 of id x 0x9E3779 step by 0.618 of
// their range per consecutive id (Fibonacci spreading), scaled to CAP by a multiply, so
// CAP need not be a power of two.  24-bit multiplies are full-rate VALU ops (32-bit ones
// take four passes), and every relaxation hashes its head.
template <int CAP>
__device__ inline uint32_t hslot(uint32_t node) {
  static_assert(CAP < (1 << 16), "table size fits the 16-bit scale");
  // v_mul_u32_u24 spelled out: only product bits 8..23 are used, which a 32-bit multiply
  // gives as well, so the compiler otherwise picks the quarter-rate v_mul_lo_u32
  uint32_t p;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(p) : "s"(0x9E3779u), "v"(node));
  const uint32_t h = (p >> 8) & 0xFFFFu;
  return __umul24(h, (uint32_t)CAP) >> 16;  // h * CAP / 2^16 < CAP
}

template <int CAP, int LM>
__device__ inline int lds_find(const SearchLds<CAP, LM>& L, uint32_t node) {
  uint32_t h = hslot<CAP>(node);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = L.key[h];
    if (k == kEmpty) return -1;
    if ((k & kNodeMask) == node) return (int)h;
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  return -1;
}

// COUNT: add new keys to L.n_keys; the main relax loop instead counts them by ballot in a
// register (one LDS atomic less per new key, and no same-address atomic serialisation)
template <int CAP, int LM, bool COUNT = true>
__device__ inline int lds_insert(SearchLds<CAP, LM>& L, uint32_t node, bool* isnew) {
  uint32_t h = hslot<CAP>(node);
  for (int probe = 0; probe < CAP; ++probe) {
    // CAS first: one LDS round trip both claims an empty slot and reads an occupied one
    const uint32_t k = atomicCAS(&L.key[h], kEmpty, node);
    if (k == kEmpty) {
      if (COUNT) atomicAdd(&L.n_keys, 1);  // load factor checked once per round (search_run)
      *isnew = true;
      return (int)h;
    }
    if ((k & kNodeMask) == node) {
      *isnew = false;
      return (int)h;
    }
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  L.overflow = 1;
  *isnew = false;
  return -1;
}

template <int CAP, int LM, int G = 1>
__device__ inline void search_init(SearchLds<CAP, LM>* Ls) {
  for (int q = 0; q < G; ++q) {
    SearchLds<CAP, LM>& L = Ls[q];
    for (int k = threadIdx.x; k < CAP; k += OTR_WAVE) {
      L.key[k] = kEmpty;
      L.lab[k] = LabelT<LM>::kInf;
    }
    if (threadIdx.x == 0) {
      L.n_pend = 0;
      L.n_keys = 0;
      L.overflow = 0;
    }
  }
  __syncthreads();
}

// Route-label packing of the LDS search: a node label is the 32-bit
// word (length mm << sh) | time, time in 0.1 s saturating at tcap = 2^sh - 1 >= bound + 1
// (sh = 0: no time bound, the word is the length).  The word order is the
// lexicographic (length, time) order, so one atomicMin keeps the exact minimum.
struct Pack {
  uint32_t sh;
  __device__ uint32_t tcap() const { return (1u << sh) - 1u; }
  template <class W>
  __device__ uint32_t d(W w) const { return (uint32_t)(w >> sh); }
  template <class W>
  __device__ uint32_t t(W w) const { return (uint32_t)(w & (W)tcap()); }
};
// the step's shift: the smallest sh with 2^sh - 1 >= bt + 1; 0 without a time bound
__host__ __device__ inline uint32_t pack_shift(int32_t bt) {
  if (bt < 0) return 0u;
  uint32_t sh = 0;
  while (((1u << sh) - 1u) < (uint32_t)bt + 1u) ++sh;
  return sh;
}
// the largest packed word of the step stays below kNoLabel
__host__ __device__ inline bool pack_fits(uint32_t bmm, uint32_t sh) {
  return (((uint64_t)bmm << sh) | ((1ull << sh) - 1ull)) < 0xFFFFFFFFull;
}

// Target (lane) resolved?  Every later offer to the target node T has length >= kmin +
// minin(T) (IN criterion), so L(T) below that — or T settled — makes T's (length, time)
// final; if even min(L(T), kmin + minin(T)) cannot make L + tpart fit the relative bound
// pd (= B - the sources' smallest exit part), T is unreachable for every source.
// (branch-free: the slot's words are read unconditionally, slot 0 for a lane without one)
// Measured and dropped: a time rule (T unreachable once it has no feasible
// label and the smallest pending time + its entry time breaks the time bound) settled
// 3.2 % fewer nodes at C2 and made the first tier 2.5 % slower (the per-round minimum,
// six more registers).
template <int CAP, int LM>
__device__ inline bool target_resolved(const SearchLds<CAP, LM>& L, const Pack& K, int tslot, uint32_t tpart,
                                       uint32_t gapT, uint32_t pd, uint32_t kmin, bool pend_empty) {
  const int ts = tslot < 0 ? 0 : tslot;
  const uint32_t key = L.key[ts];
  const typename LabelT<LM>::W lw = LabelT<LM>::label(L.lab[ts]);
  const int64_t lab = lw == LabelT<LM>::kNone ? INT64_MAX / 4 : (int64_t)K.d(lw);
  const int64_t next = (int64_t)kmin + (int64_t)gapT;
  const bool unreach = (lab < next ? lab : next) + (int64_t)tpart > (int64_t)pd;
  return (tslot < 0) | pend_empty | ((key & kRel) != 0u) | (lab < next) | unreach;
}

// Relax edge (u → dw) with u's FINAL packed label pu: the offer (length nd, time tt) is
// pruned when it breaks a bound (pd / pt: B and bt relative to the root),
// else it is inserted and kept by atomicMin.  A label improves when its packed word does
// (a shorter length, or the same length sooner): the node is then pending (again).  The
// improvement's length enters the next round's kmin.  mq: minin(head) in 16-mm units
// (the adjacency record carries it), stored with a new key.  Returns the slot when it
// became newly pending.
template <int CAP, int LM, bool COUNT = true>
__device__ inline int relax_one(SearchLds<CAP, LM>& L, const Pack& K, uint32_t dw, uint32_t len_mm,
                                uint32_t time_ds, uint32_t minin, typename LabelT<LM>::W pu, uint32_t edge,
                                uint32_t pd, uint32_t pt, uint32_t mode_bit, uint32_t& relaxed, uint32_t& knext,
                                bool& isnew) {
  using W = typename LabelT<LM>::W;
  isnew = false;
  if (!(((dw >> 28) & 7u) & mode_bit)) return -1;
  ++relaxed;
  const uint32_t nd = K.d(pu) + len_mm;  // d <= bound < 2^31, len_mm < 2^31: no wrap
  if (nd > pd) return -1;
  const uint32_t tt = K.t(pu) + time_ds;  // both < 2^31
  if (tt > pt) return -1;
  const W nw = ((W)nd << K.sh) | (W)tt;  // tt <= pt <= bt < 2^sh - 1
  const int sl = lds_insert<CAP, LM, COUNT>(L, dw & kAdjDstMask, &isnew);
  if (sl < 0) return -1;
  if (isnew) L.mi[sl] = SearchLds<CAP, LM>::code(minin);
  const typename LabelT<LM>::T nb = LabelT<LM>::make(nw, edge);
  const typename LabelT<LM>::T old = atomicMin(&L.lab[sl], nb);
  if (LabelT<LM>::label(nb) < LabelT<LM>::label(old)) {
    knext = nd < knext ? nd : knext;
    const uint32_t ok = atomicOr(&L.key[sl], kInq);
    if (!(ok & kInq)) return sl;  // newly pending: the caller appends it
  }
  return -1;
}

// relax_one for the plain (non-PRED) tables with its common path branch-free: the
// group's lanes all issue the insert, label and pending-bit atomics, a lane with nothing
// to do aiming them at its own word of `sink` (a per-wave scratch row in LDS whose values
// are never read), so the exec-mask bookkeeping of the nested ifs is gone — the scalar
// unit, which carries it, was the search's busiest issue port.  Only a
// probe chain past the home slot takes a branch (wave-uniform, rare).  Same slots, labels
// and pending list as relax_one.
template <int CAP>
__device__ inline int relax_sink(SearchLds<CAP, 0>& L, uint32_t* sink, const Pack& K, uint32_t dw, uint32_t len_mm,
                                 uint32_t time_ds, uint32_t minin, uint32_t pu, uint32_t pd, uint32_t pt,
                                 uint32_t mode_bit, uint32_t& relaxed, uint32_t& knext, bool& isnew) {
  const bool mode_ok = (((dw >> 28) & 7u) & mode_bit) != 0u;
  relaxed += mode_ok ? 1u : 0u;
  const uint32_t nd = K.d(pu) + len_mm;  // d <= bound < 2^31, len_mm < 2^31: no wrap
  const uint32_t tt = K.t(pu) + time_ds;
  const uint32_t nw = (nd << K.sh) | tt;  // read only where tt <= pt < 2^sh - 1
  const uint32_t node = dw & kAdjDstMask;
  bool go = mode_ok && nd <= pd && tt <= pt;
  uint32_t* mine = sink + lane_id();
  const uint32_t h0 = hslot<CAP>(node);
  const uint32_t k0 = atomicCAS(go ? &L.key[h0] : mine, kEmpty, node);
  isnew = go && k0 == kEmpty;
  int sl = (go && (k0 == kEmpty || (k0 & kNodeMask) == node)) ? (int)h0 : -1;
  const bool coll = go && sl < 0;
  if (__ballot(coll) != 0ull) {  // the home slot holds another node: linear probing
    if (coll) {
      uint32_t hh = h0;
      for (int probe = 1; probe < CAP; ++probe) {
        hh = hh + 1 == (uint32_t)CAP ? 0u : hh + 1;
        const uint32_t k = atomicCAS(&L.key[hh], kEmpty, node);
        if (k == kEmpty) {
          isnew = true;
          sl = (int)hh;
          break;
        }
        if ((k & kNodeMask) == node) {
          sl = (int)hh;
          break;
        }
      }
      if (sl < 0) L.overflow = 1;
    }
  }
  go = go && sl >= 0;
  using MiT = typename SearchLds<CAP, 0>::MiT;
  *((go && isnew) ? &L.mi[sl] : reinterpret_cast<MiT*>(mine)) = SearchLds<CAP, 0>::code(minin);
  const uint32_t old = atomicMin(go ? &L.lab[sl] : mine, nw);
  const bool imp = go && nw < old;
  knext = (imp && nd < knext) ? nd : knext;
  const uint32_t was = atomicOr(imp ? &L.key[sl] : mine, kInq);
  return (imp && !(was & kInq)) ? sl : -1;  // newly pending: the caller appends it
}

// Resuming an outgrown node search in the next retry table (as otr_edge1.h does for the
// edge-state tiers): a search that passes its table's load limit stops between two rounds
// (no relaxation lost) and its table goes to a dump slot in HBM — every key with its label
// and minin code (settled nodes too, whose final labels keep rejecting later offers; the
// pending ones carry kInq), and the round's kmin; the next table re-inserts the keys,
// rebuilds the pending list and goes on with the next round: the same rounds as one big
// table, so the same labels.  32-bit labels only (the retry tiers).  Slot (u64 words):
// [0] entries n, [1] kmin, [2, 2 + n) label | key << 32, then the n IN gaps (u32 mm: the
// tables' codes differ, SearchLds::code / gap; re-encoding a gap keeps a lower bound).
struct NDump {
  const unsigned long long* in;  // the dump this group's search resumes (null: a fresh search)
  unsigned long long* base;      // this tier's dump slots (null: an outgrown search restarts)
  unsigned long long* ctr;       // slots taken (zeroed per batch)
  uint32_t words, slots;
#ifdef OTR_FORCE_RETRY
  int stop_rounds;  // test build: a search with dump slots stops after this many rounds (0: off)
#endif
};
__host__ __device__ constexpr uint32_t nd_words(int cap) { return 2u + (uint32_t)cap + ((uint32_t)cap + 1u) / 2u; }
// which retry tables carry the resume code (compile time: the code costs the hot tiers ~2 %
// even unused): tables of at least OTR_ND_IN_MIN slots resume, of at least OTR_ND_OUT_MIN
// slots dump (C4: the 1024-slot tier's 4 % outgrowers; the smaller tiers' overflows are few)
#ifndef OTR_ND_IN_MIN
#define OTR_ND_IN_MIN 2048
#endif
#ifndef OTR_ND_OUT_MIN
#define OTR_ND_OUT_MIN 1024
#endif

// G searches per wave, one per lane group, each in its own table Ls[g]: search g is
// rooted at `start` (label 0); lanes gl < n_tgt of the group hold a target node tnode,
// its minin gapT (in_gap units: mm, >= 1) and partial length tpart (mm).  active = false:
// the group idles.  K packs the labels (route time tracked when K.sh > 0, from adj_t /
// edge_t: the mode's times).  pd / pt prune the relaxations (relative length and time
// bounds, relax_one); pd also decides when a target is unreachable.  Returns false (per
// lane, group-uniform) on an LDS-table overflow.  nd (retry tiers): the group's dump to
// resume, and this tier's dump slots; *dslot: the slot an outgrown search went to (-1: none).
template <int CAP, int LM, int G = 1, bool RIN = false, bool ROUT = false>
__device__ bool search_run(SearchLds<CAP, LM>* Ls, const DevGraph& g, const Pack& K, uint32_t mode_bit, bool active,
                           uint32_t start, uint32_t pd, uint32_t pt, uint32_t tnode, uint32_t tpart, uint32_t gapT,
                           int n_tgt, unsigned long long* settled, unsigned long long* relaxed,
                           unsigned long long* rounds, unsigned long long* stamps = nullptr, uint32_t* sink = nullptr,
                           const NDump* nd = nullptr, int* dslot = nullptr) {
  using Gr = Grp<G>;
  // load-factor limit (probe chains stay short): 7/8 (the exact searches run to the
  // bounds, so a fuller first-tier table keeps more of them out of the retry tiers: C2
  // 32.5M -> 33.1M probes/s against 3/4, profiles/r03_ab_load7_bench_c2.json)
  constexpr int kMaxKeys = (CAP <= 128 || CAP >= 256) ? (CAP * 7) / 8 : (CAP * OTR_LOAD1) / 8;
  const int gl = Gr::gl();
  using W = typename LabelT<LM>::W;
  SearchLds<CAP, LM>& L = Ls[Gr::g()];
  using Idx = typename SearchLds<CAP, LM>::Idx;
  constexpr int WCAP = SearchLds<CAP, LM>::WCAP;
  const bool timed = K.sh != 0u;  // group-uniform
  const uint32_t* adjt = g.adj_t + (size_t)__builtin_ctz(mode_bit) * g.adj_t_stride;
  uint32_t kmin = 0;           // the smallest pending length (0xFFFFFFFF: nothing pending)
  int npend = active ? 1 : 0;  // pending-list length (group-uniform register)
  // resume: the outgrown search's table, keys re-inserted (distinct: every CAS lands)
  const bool resume = RIN && LM == 0 && active && nd->in != nullptr;  // (group-uniform)
  const int nres = resume ? (int)nd->in[0] : 0;
  const int nrx = RIN ? Gr::umax(nres) : 0;
  if (RIN && nrx > 0) {
    const unsigned long long* D = nd->in;
    const uint32_t* M = (const uint32_t*)(D + 2 + nres);
    int np = 0;
    for (int base = 0; base < nrx; base += Gr::GL) {
      const int k = base + gl;
      bool pend = false;
      int sl = 0;
      if (k < nres) {
        const unsigned long long e = D[2 + k];
        const uint32_t key = (uint32_t)(e >> 32), node = key & kNodeMask;
        uint32_t h = hslot<CAP>(node);
        for (int probe = 0; probe < CAP; ++probe) {
          if (atomicCAS(&L.key[h], kEmpty, node) == kEmpty) break;
          h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
        }
        sl = (int)h;
        L.key[sl] = key;
        L.lab[sl] = (typename LabelT<LM>::T)(uint32_t)e;
        L.mi[sl] = SearchLds<CAP, LM>::code(M[k]);
        pend = (key & kInq) != 0u;
      }
      const unsigned long long mp = __ballot(pend);
      if (pend && np + Gr::prefix(mp) < SearchLds<CAP, LM>::PCAP) L.pend[np + Gr::prefix(mp)] = (Idx)sl;
      np += Gr::count(mp);
    }
    if (resume && np > SearchLds<CAP, LM>::PCAP) {  // (a frontier past the pending list: restart)
      if (gl == 0) L.overflow = 1;
      np = SearchLds<CAP, LM>::PCAP;
    }
    if (resume) {
      npend = np;
      kmin = (uint32_t)D[1];
      if (gl == 0) L.n_keys = nres;
    }
  }
  if (!resume && active && gl == 0) {
    bool isnew;
    const int sl = lds_insert(L, start, &isnew);
    L.mi[sl] = 0;
    L.lab[sl] = LabelT<LM>::make(0u, kEmpty);
    L.key[sl] |= kInq;
    L.pend[0] = (Idx)sl;
  }
  __syncthreads();
  // targets are pre-inserted (no label) so every round reads their label from a known slot
  int tslot = -1;
  if (active && gl < n_tgt && tnode != kEmpty) {
    bool isnew;
    tslot = lds_insert(L, tnode, &isnew);
    if (tslot >= 0 && isnew) L.mi[tslot] = SearchLds<CAP, LM>::code(gapT);
  }
  __syncthreads();
  uint32_t my_settled = 0, my_relaxed = 0, my_rounds = 0;
  unsigned long long cyc[4] = {0, 0, 0, 0};
  bool done = !active, grew = false;  // grew: stopped between rounds at the load limit
#ifdef OTR_FORCE_RETRY
  int force_round = 0;
#endif
  int nkeys = 0;               // keys the main relax loop added (group-uniform; L.n_keys has the rest)
  for (;;) {
    OTR_STAMP(t0);
    const int np = done ? 0 : npend;
    OTR_STAMP(t1);
    const bool res = done | (gl >= n_tgt) | target_resolved(L, K, tslot, tpart, gapT, pd, kmin, np == 0);
    done = done || Gr::mine(__ballot(!res)) == 0ull || np == 0;
    OTR_STAMP(t2);
    cyc[0] += t1 - t0;
    cyc[1] += t2 - t1;
    if (Gr::all(done)) break;
    if (!done && gl == 0) ++my_rounds;
    uint32_t knext = 0xFFFFFFFFu;
    int kept = 0, nw = 0;
    const int npx = Gr::umax(np);
    for (int base = 0; base < npx; base += Gr::GL) {
      const int k = base + gl;
      const bool in = k < np;
      // unconditional reads (k < CAP; a lane past its group's list reads slot 0), so no
      // exec-mask branch around them
      const int sl = in ? (int)L.pend[k] : 0;
      const W lb = LabelT<LM>::label(L.lab[sl]);
      const uint32_t key = L.key[sl];
      const uint32_t d = K.d(lb);
      bool take = in && (uint64_t)d < (uint64_t)kmin + SearchLds<CAP, LM>::gap(L.mi[sl]);  // final (IN criterion)
      // at most WCAP settles per round; the rest stay pending (still final later)
      take = take && nw + Gr::prefix(__ballot(take)) < WCAP;
      const unsigned long long mt = __ballot(take), mk = __ballot(in && !take);
      __syncthreads();
      if (take) {
        // off the pending list and marked settled; the relax phase's atomics on this key
        // come after the barrier below, so a plain store suffices
        const uint32_t node = key & kNodeMask;
        L.work[nw + Gr::prefix(mt)] = WorkE<W>{node, lb};
        L.key[sl] = node | kRel;
      }
      const bool keep = in && !take;
      if (keep) L.pend[kept + Gr::prefix(mk)] = (Idx)sl;
      knext = (keep && d < knext) ? d : knext;
      nw += Gr::count(mt);
      kept += Gr::count(mk);
      __syncthreads();
    }
    npend = kept;
    OTR_STAMP(t3);
    cyc[2] += t3 - t2;
    // relax: lane = (work node, adjacency slot), so a round's dependent chain is a single
    // relaxation; slot 3 of a node with more than 4 out-edges also walks the CSR tail
    const int nwx = Gr::umax(4 * nw);
    uint32_t tail = 0u;  // (a lane word, not a lane mask: VALU ors instead of scalar mask updates)
    for (int base = 0; base < nwx; base += Gr::GL) {
      const int k = base + gl;
      int psl = -1;
      bool isnew = false;
      if (k < 4 * nw) {
        const WorkE<W> wk = L.work[k >> 2];
        const uint32_t wnode = wk.node;
        const int slot = k & 3;
        if (slot == 0) ++my_settled;
        // the mode's route time of the slot (DevGraph::adj_t, one block per mode), loaded
        // beside the adjacency record and unconditionally: both loads in flight together
        const uint32_t tq = adjt[4 * (size_t)wnode + slot];
        const uint4 r = ld16(g.adj + 4 * (size_t)wnode + slot);
        const uint32_t tt = timed ? tq : 0u;
        if constexpr (LM == 0) {
#ifdef OTR_NO_SINK  // (A/B build: the branching relax_one)
          psl = relax_one<CAP, LM, false>(L, K, r.x & ~kAdjMore, r.y, tt, r.z, wk.lab, 0u, pd, pt, mode_bit,
                                          my_relaxed, knext, isnew);
#else  // (every 32-bit table has its scratch row: no run-time test of `sink`)
          psl = relax_sink<CAP>(L, sink, K, r.x & ~kAdjMore, r.y, tt, r.z, wk.lab, pd, pt, mode_bit, my_relaxed,
                                knext, isnew);
#endif
        } else {
          const uint32_t e0 = LM == 1 ? g.node_row[wnode] : 0u;  // edge id = CSR row start + slot
          psl = relax_one<CAP, LM, false>(L, K, r.x & ~kAdjMore, r.y, tt, r.z, wk.lab, e0 + slot, pd, pt, mode_bit,
                                          my_relaxed, knext, isnew);
        }
        tail |= slot == 3 ? (r.x & kAdjMore) : 0u;
      }
      nkeys += Gr::count(__ballot(isnew));
      // append newly pending nodes by ballot (no shared counter)
      const unsigned long long mp = __ballot(psl >= 0);
#ifndef OTR_NO_SINK
      if constexpr (LM == 0 && G == 1) {
        // branch-free (the one-search retry tables: C4's 1024-slot tier 240.1 -> 237.0 ms;
        // the two-search first tier is faster with the branch): a lane with nothing to
        // append writes its scratch word (< CAP: the pending nodes are distinct keys of the
        // table; clamped)
        const int p = npend + Gr::prefix(mp);
        constexpr int PC = SearchLds<CAP, LM>::PCAP;
        *(psl >= 0 ? &L.pend[p < PC ? p : PC - 1] : reinterpret_cast<Idx*>(sink + lane_id())) = (Idx)psl;
      } else
#endif
      if (psl >= 0) {
        // (< CAP: the pending nodes are distinct keys of the table; clamped, not branched)
        const int p = npend + Gr::prefix(mp);
        L.pend[p < SearchLds<CAP, LM>::PCAP ? p : SearchLds<CAP, LM>::PCAP - 1] = (Idx)psl;
      }
      npend += Gr::count(mp);
    }
    // (a pending list past its capacity lost appends: the search restarts in the next table)
    if (SearchLds<CAP, LM>::PCAP < CAP && npend > SearchLds<CAP, LM>::PCAP) {
      if (gl == 0) L.overflow = 1;
      npend = SearchLds<CAP, LM>::PCAP;
    }
    if (__ballot(tail != 0u) != 0ull) {
      // rare: slot 3 of a node with more than 4 out-edges walks the CSR tail; appends
      // through the shared counter
      if (gl == 0) L.n_pend = npend;
      __syncthreads();
      for (int base = 0; base < nwx; base += Gr::GL) {
        const int k = base + gl;
        if (k < 4 * nw && (k & 3) == 3) {
          const WorkE<W> wk = L.work[k >> 2];
          const uint32_t wnode = wk.node;
          if (g.adj[4 * (size_t)wnode + 3].x & kAdjMore)
            for (uint32_t e = g.node_row[wnode] + 4; e < g.node_row[wnode + 1]; ++e) {
              const uint4 pk = ld16(g.edge_pack + e);  // {dst, len_mm, attr, minin(dst)}
              const uint32_t tt = timed ? g.et(__builtin_ctz(mode_bit))[e] : 0u;
              bool isnew;
              const int psl = relax_one(L, K, pk.x | ((pk.z & 7u) << 28), pk.y, tt, pk.w, wk.lab, e, pd, pt, mode_bit,
                                        my_relaxed, knext, isnew);
              if (psl >= 0) {
                const int p = atomicAdd(&L.n_pend, 1);
                if (p < SearchLds<CAP, LM>::PCAP) L.pend[p] = (Idx)psl;
                else L.overflow = 1;
              }
            }
        }
      }
      __syncthreads();
      npend = L.n_pend;
      if (npend > SearchLds<CAP, LM>::PCAP) npend = SearchLds<CAP, LM>::PCAP;
    }
    __syncthreads();
    OTR_STAMP(t4);
    cyc[3] += t4 - t3;
    // a finished group's kmin stays that of its last round (G = 2: the other group may run
    // on; an outgrown search's dump needs the kmin it stopped with)
    const uint32_t km = Gr::min_u32(knext);
    if (!done) kmin = km;
    const int keys = L.n_keys + nkeys;
    if (!done && (L.overflow || keys > kMaxKeys)) {
      grew = !L.overflow && keys > kMaxKeys;
      done = true;
    }
#ifdef OTR_FORCE_RETRY
    ++force_round;
    if (ROUT && !done && nd->base != nullptr && nd->stop_rounds > 0 && force_round >= nd->stop_rounds &&
        !L.overflow) {
      grew = true;
      done = true;
    }
#endif
    __syncthreads();
    if (done && active && gl == 0 && (keys > kMaxKeys || grew)) L.overflow = 1;
  }
  if (gl == 0) L.n_keys += nkeys;  // the table's key count, for the caller
  if (ROUT) *dslot = -1;
  if (ROUT && LM == 0 && __ballot(grew && active && nd->base != nullptr) != 0ull) {
    // dump the outgrown tables to claimed slots: keys in slot order, compacted by ballot
    int v = 0;
    if (grew && active && nd->base != nullptr && gl == 0) v = (int)atomicAdd(nd->ctr, 1ull);
    v = __shfl(v, 0, Gr::GL);  // (the group's lane 0)
    const bool dump = grew && active && nd->base != nullptr && (uint32_t)v < nd->slots;  // (group-uniform)
    unsigned long long* D = dump ? nd->base + (size_t)v * nd->words : nullptr;
    int n = 0;
    for (int base = 0; base < CAP; base += Gr::GL) {
      const int k = base + gl;
      const uint32_t key = (dump && k < CAP) ? L.key[k] : kEmpty;
      const bool has = key != kEmpty;
      const unsigned long long m = __ballot(has);
      if (has) D[2 + n + Gr::prefix(m)] = (unsigned long long)(uint32_t)L.lab[k] | ((unsigned long long)key << 32);
      n += Gr::count(m);
    }
    uint32_t* M = dump ? (uint32_t*)(D + 2 + n) : nullptr;
    int q = 0;
    for (int base = 0; base < CAP; base += Gr::GL) {
      const int k = base + gl;
      const bool has = dump && k < CAP && L.key[k] != kEmpty;
      const unsigned long long m = __ballot(has);
      if (has) M[q + Gr::prefix(m)] = SearchLds<CAP, LM>::gap(L.mi[k]);
      q += Gr::count(m);
    }
    if (dump && gl == 0) {
      D[0] = (unsigned long long)(uint32_t)n;
      D[1] = kmin;
    }
    *dslot = dump ? v : -1;
  }
#ifdef OTR_STAMPS
  if (stamps && threadIdx.x == 0)
    for (int q = 0; q < 4; ++q) atomicAdd(&stamps[q * kCShards + cshard()], cyc[q]);
#endif
  if (settled) *settled += my_settled;
  if (relaxed) *relaxed += my_relaxed;
  if (rounds) *rounds += my_rounds;
  __syncthreads();
  return !L.overflow;
}

// ------------------------------------------------------------------------------
// K2b: per-state search inputs, computed once per state instead of once per search
// task (a step has ~9 tasks): per candidate j {entry part mm, source node, minin(source
// node) (the IN criterion's gap of a target; turn modes: the begin heading of the edge,
// which the edge-state search's target turn needs), exit part mm}.
// ------------------------------------------------------------------------------
struct PrepArgs {
  int64_t n_states;
  const int64_t* prev;
  const double* bound;
  const int32_t* cand_count;
  const uint32_t* cand_edge;
  const double* cand_p;
  const int32_t* state_trace;
  const uint8_t* mode;
  uint4* cprep;   // [S][OTR_KMAX]: {part(p), src(e), minin(src(e)) | turn modes: heading(e), part(1 - p)}
  uint2* cprep_t; // [S][OTR_KMAX]: {part_t(p), part_t(1 - p)}: the same parts of the edge's route time
  uint2* clen;    // [S][OTR_KMAX]: {len_mm(e), route time(e)}: a same-edge transition's whole-edge terms
  int32_t* nroot; // [S]: the search tasks of the step leaving the state (k_tasks' grouping)
  uint32_t turn_modes;  // bit m: mode m has turn costs (edge-based searches, one per source)
};

// G states per wave (G = 2 when every mode keeps <= 32 candidates: lane groups of 32;
// the kernel waits on dependent loads, so half the waves take about half the time)
template <int G>
__global__ __launch_bounds__(256) void k_prep(DevGraph g, PrepArgs a) {
  constexpr int GL = OTR_WAVE / G;
  const int64_t s = ((int64_t)blockIdx.x * (blockDim.x / OTR_WAVE) + threadIdx.x / OTR_WAVE) * G +
                    (threadIdx.x % OTR_WAVE) / GL;
  const int lane = threadIdx.x % GL;
  if (s >= a.n_states) return;
  const int K = a.cand_count[s];
  if (K <= 0) return;
  const int md = a.mode[a.state_trace[s]] < OTR_MODES ? a.mode[a.state_trace[s]] : 0;
  const bool turn = (a.turn_modes >> md) & 1u;
  // distinct search tasks (K <= OTR_KMAX: one candidate per lane): a lane is its task's
  // first holder when no lower lane has the same key (root, exit time) (k_tasks' rule)
  uint32_t root = 0xFFFFFFFFu, t0 = 0u;
  if (lane < K) {
    const uint32_t e = a.cand_edge[s * OTR_KMAX + lane];
    const double p = a.cand_p[s * OTR_KMAX + lane];
    const uint4 ep = g.eprep[e];  // {len_mm, src, minin(src), dst}: one gather beside the time's
    const uint32_t et = g.et(md)[e];
    const uint32_t len = ep.x, tn = ep.y;
    const uint32_t z = turn ? (uint32_t)(uint16_t)g.edge_head[e].x : ep.z;
    const uint32_t x1 = (uint32_t)part_mm(1.0 - p, len), t1 = (uint32_t)part_mm(1.0 - p, et);
    a.cprep[s * OTR_KMAX + lane] = make_uint4((uint32_t)part_mm(p, len), tn, z, x1);
    a.cprep_t[s * OTR_KMAX + lane] = make_uint2((uint32_t)part_mm(p, et), t1);
    a.clen[s * OTR_KMAX + lane] = make_uint2(len, et);
    root = turn ? e : ep.w;
    if (!turn) t0 = t1;
  }
  bool first = lane < K;
  for (int k = 0; k < K; ++k) {
    const uint32_t rk = (uint32_t)__shfl((int)root, k, GL);  // every lane of the group takes part
    const uint32_t tk = (uint32_t)__shfl((int)t0, k, GL);
    if (k < lane && rk == root && tk == t0) first = false;
  }
  const int nr = __popcll(group_bits<G>(__ballot(first)));
  if (lane == 0) a.nroot[s] = nr;
}

// the small-search first tier (k_route<OTR_CAP4, 4>): which steps' tasks it takes
// (SmallArgs::ntask4 null: none, every task in the two-search tier)
#ifndef OTR_CAP4
#define OTR_CAP4 80
#endif
// the tiny-search tier (k_route<OTR_CAP8, 8>: eight searches per wave, 8 lanes each)
#ifndef OTR_CAP8
#define OTR_CAP8 40
#endif
struct SmallArgs {
  int64_t* ntask4;            // per state: the step's tasks when they go to the small tier, else 0
  int64_t* ntask8;            // per state: ... to the tiny tier (null: none)
  float tiny_keys;            // a step of at most 8 targets whose estimate is at most this is tiny
  const double* bound;
  const int32_t* bt;
  const uint8_t* forced;
  const int32_t* cand_count;
  const int32_t* state_trace;
  const uint8_t* mode;
  uint32_t turn_modes;
  float est_k;                // k_tasks' size estimate (keys = est_k * reach^2)
  float est_v[OTR_MODES];
  float small_keys;           // a step whose estimate is at most this many keys is small
};

// search tasks of each step: one per distinct root among the previous state's candidates.
// With the small tier on, a step goes to it (ntask4) or to the two-search tier (ntask):
// node mode, 32-bit labels, not forced, at most 16 targets (a lane group of 16) and a
// size estimate (k_tasks' rule) of at most small_keys keys; the two classes get separate
// task ranges (small first), so each first-tier kernel runs over a contiguous range.
__global__ void k_ntask(int64_t n_states, const int64_t* prev, const int32_t* nroot, int64_t* ntask, SmallArgs sa) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_states) return;
  const int64_t sp = prev[s];  // -1: first state of a sub-trace, -2: no candidates (k_link)
  const int64_t n = sp >= 0 ? nroot[sp] : 0;
  bool small = false, tiny = false;
  if (sa.ntask4 != nullptr && n > 0 && sa.cand_count[s] <= OTR_WAVE / 4 && !sa.forced[s]) {
    const int md = sa.mode[sa.state_trace[s]] < OTR_MODES ? sa.mode[sa.state_trace[s]] : 0;
    const uint32_t bmm = (uint32_t)bound_mm_of(sa.bound[s]);
    const int32_t bt = sa.bt[s];
#ifdef OTR_FORCE_GENERAL
    const bool general = true;  // (test build: every search in k_general)
#else
    const bool general = !pack_fits(bmm, pack_shift(bt)) || ((sa.turn_modes >> md) & 1u);
#endif
    if (!general) {
      float reach = (float)bmm * 1e-3f;
      if (bt >= 0) reach = fminf(reach, (float)bt * 0.1f * sa.est_v[md]);
      const float est = sa.est_k * reach * reach;
      small = est <= sa.small_keys;
      tiny = sa.ntask8 != nullptr && sa.cand_count[s] <= OTR_WAVE / 8 && est <= sa.tiny_keys;
    }
  }
  if (sa.ntask8 != nullptr) sa.ntask8[s] = tiny ? n : 0;
  if (sa.ntask4 != nullptr) sa.ntask4[s] = small && !tiny ? n : 0;
  ntask[s] = small || tiny ? 0 : n;
}

// ------------------------------------------------------------------------------
// K3 + K4: one wave per (step, search root): search, then transition costs for
// every source candidate sharing the root.
// ------------------------------------------------------------------------------
struct RouteArgs {
  const int64_t* task_list;   // optional indirection (overflow retry), else null
  int64_t n_tasks;
  const int64_t* prev;
  const double* g;
  const double* bound;
  const uint8_t* forced;
  const int64_t* trans_off;
  uint32_t* trans;            // route length (mm) per transition, kNoRoute when invalid
  const int32_t* cand_count;
  const uint32_t* cand_edge;
  const double* cand_p;
  const int32_t* state_trace;
  const uint8_t* mode;
  const uint4* cprep;         // per state candidate (k_prep)
  const uint2* cprep_t;       // per state candidate: route-time parts (k_prep)
  const uint2* clen;          // per state candidate: {len_mm(e), route time(e)} (k_prep)
  const int32_t* bt;          // per state: the step's time bound (0.1 s), -1 none
  const uint4* rec;           // per task, 3 x uint4 (k_tasks)
  const unsigned long long* list_count;  // retry tiers: length of task_list, on the device
  const int32_t* turn;        // [OTR_MODES][181] turn cost tables (mm), turn modes only
  uint32_t* trans_tc;         // turn cost (mm) per transition, turn modes only
  double inv_beta[OTR_MODES];
  int32_t* overflow_flag;     // per task: 1/2 retry in a larger LDS table, 3 the global-memory search,
                              // 5 / 6 the edge-state tiers
  // first tier: a search whose expected size (keys) exceeds its table starts in the first
  // retry tier that holds it (flag 16 + tier): expected keys = est_k * r^2 with r = the
  // step's reach, min(length bound, time bound x est_v[mode])
  float est_k;                // keys per m^2 of reach (calibrated on the graph's node density)
  float est_v[OTR_MODES];     // m/s: the mode's typical speed (50 km/h, capped by the mode's)
  uint32_t tier_keys[8];      // key capacity of each retry tier, in order
  int n_tiers;
  int64_t unit_base;          // first tier: the launch's first unit (launches of < 2^32 work-items)
  int64_t task_base;          // first tier: its first task (the small tier's tasks come first)
  unsigned long long* queue;  // list tiers: this launch's 8 per-XCD unit counters (XcdQueue), zeroed
  unsigned long long* stamps;  // diagnostic build (OTR_STAMPS): bank 0 of the work counters (phase cycles)
  int force_edge;             // test build only (OTR_FORCE_RETRY, env OTR_FORCE_EDGE): bits 0 / 1 / 2 fail
                              // every OTR_E1CAP (360) / 512 / 1024-state edge-state route search (the
                              // next tier takes it), bits 3 / 4 every 384 / 2048-state winner path;
                              // bits 5 / 6 stop every OTR_E1CAP / 512-state search after 2 / 4 rounds
                              // and resume it in the next table (otr_edge1.h e1_dump / e1_restore);
                              // bit 7 stops every node retry-tier search that has dump slots after 2
                              // rounds (search_run, NDump): resumed tier after tier to the last
  // retry tiers (node and edge-state): a search that outgrows its table is dumped between
  // two rounds and resumed in the next table (search_run NDump, otr_edge1.h e1_dump)
  const unsigned long long* dump_in;  // the previous tier's dumps (null: every search starts afresh)
  uint32_t dump_in_words, dump_in_cap;  // u64 words per dump slot, the table size that wrote them
  unsigned long long* dump_out;       // this tier's dump slots (null: outgrown searches restart)
  unsigned long long* dump_ctr;       // slots taken (device counter, zeroed per batch)
  uint32_t dump_out_words, dump_out_slots;
  int32_t* task_dump;                 // per task: its slot in the next tier's input, -1: restart
};

// k_tasks' inputs and outputs
struct TaskArgs {
  int64_t n_states;
  const int64_t* prev;
  const int32_t* cand_count;
  const uint32_t* cand_edge;
  const uint32_t* edge_dst;
  const int64_t* task_off;    // exclusive offsets of each step's tasks (scan of k_ntask's counts)
  const double* bound;
  const uint8_t* forced;
  const int32_t* bt;
  const int32_t* state_trace;
  const uint8_t* mode;
  const uint4* cprep;         // k_prep
  const uint2* cprep_t;       // k_prep
  const int64_t* trans_off;
  uint32_t turn_modes;
  uint4* rec;                 // 3 per task (the K2c record, below; the state and source mask of a task
                              // are read from it everywhere: no separate per-task arrays)
  const int64_t* ntask4;      // small-tier steps' task counts (k_ntask), or null
  const int64_t* task4_off;   // their exclusive offsets: small-tier tasks are [nt8, nt8 + nt4)
  int64_t nt4;                // two-search tasks are nt8 + nt4 + task_off[s]
  const int64_t* ntask8;      // tiny-tier steps' task counts, or null
  const int64_t* task8_off;   // their exclusive offsets: tiny-tier tasks are [0, nt8)
  int64_t nt8;
  int32_t* flag_turn;         // per task: 5 for a turn-mode task (the first edge-state tier's list), or null
  // the two-search first tier's size estimate (RouteArgs est_*): a node-mode step whose
  // estimated keys exceed est_first_keys (0: no estimate) starts in a retry tier
  int est_first_keys;
  float est_k;
  float est_v[OTR_MODES];
  uint32_t tier_keys[8];
  int n_tiers;
};

// One lane group per step s (G states per wave: G = 2 when every mode keeps <= 32
// candidates), lane i = source candidate i of the previous state.  Node mode: the sources
// whose edges end at the same node and whose exit parts take the same route time share a
// task: one search rooted at that node, pruned at bt - that time and at B - the smallest
// exit part — length pruning is monotone in the label order, so each source's labels
// within its own length bound are the shared ones.  Turn modes: every
// source edge is its own task (the edge-state search).  The task's representative (its lowest source) writes the task
// record every route kernel reads (its state and source mask included):
//   rec[3t]   = {s, sp, root, bound_mm}
//   rec[3t+1] = {d0min, Kb | mode << 8 | forced << 10 | sh << 11 | general << 16 | turn << 17 | pre << 18,
//                mask lo, mask hi}
//   rec[3t+2] = {0, time bound bt, trans_off[s] lo, hi}
// general: the task runs in the global-memory search (a bound whose packed labels would
// not fit 32 bits, or a turn mode: edge-based labels).  pre (4 bits): 1 | the retry tier
// << 1 of a step whose size estimate exceeds the first tier's table (the first tier flags
// it 16 + tier without loading its step); the estimate is per step (bound, time bound, mode).
template <int G>
__global__ __launch_bounds__(256) void k_tasks(TaskArgs a) {
  constexpr int GL = OTR_WAVE / G;
  const int64_t s = ((int64_t)blockIdx.x * (blockDim.x / OTR_WAVE) + threadIdx.x / OTR_WAVE) * G +
                    (threadIdx.x % OTR_WAVE) / GL;
  const int lane = threadIdx.x % GL;
  if (s >= a.n_states) return;
  const int64_t sp = a.prev[s];
  if (sp < 0 || a.cand_count[s] <= 0) return;
  const int Ka = a.cand_count[sp];
  const int md = a.mode[a.state_trace[s]] < OTR_MODES ? a.mode[a.state_trace[s]] : 0;
  const uint32_t turn = (a.turn_modes >> md) & 1u;
  const uint32_t ce = lane < Ka ? a.cand_edge[sp * OTR_KMAX + lane] : 0xFFFFFFFFu;
  const uint32_t root = lane < Ka ? (turn ? ce : a.edge_dst[ce]) : 0xFFFFFFFFu;
  const uint32_t w = lane < Ka ? a.cprep[sp * OTR_KMAX + lane].w : 0xFFFFFFFFu;  // exit part mm
  const uint32_t t0 = (lane < Ka && !turn) ? a.cprep_t[sp * OTR_KMAX + lane].y : 0u;  // exit part time
  // sources sharing my task (root, exit time), their smallest exit part, then: am I the
  // lowest of them?
  unsigned long long same = 0;
  uint32_t d0min = 0xFFFFFFFFu;
  for (int k = 0; k < Ka; ++k) {
    const uint32_t rk = (uint32_t)__shfl((int)root, k, GL), wk = (uint32_t)__shfl((int)w, k, GL);
    const uint32_t tk = (uint32_t)__shfl((int)t0, k, GL);
    if (rk == root && tk == t0) {
      same |= 1ull << k;
      d0min = wk < d0min ? wk : d0min;
    }
  }
  const bool rep = lane < Ka && (__ffsll((long long)same) - 1) == lane;
  const unsigned long long reps = group_bits<G>(__ballot(rep));
  if (!rep) return;
  // the step's task range: the small tier's first, then the two-search tier's (k_ntask)
  const int64_t n4 = a.ntask4 != nullptr ? a.ntask4[s] : 0;
  const int64_t n8 = a.ntask8 != nullptr ? a.ntask8[s] : 0;
  const int64_t tbase = n8 > 0 ? a.task8_off[s] : (n4 > 0 ? a.nt8 + a.task4_off[s] : a.nt8 + a.nt4 + a.task_off[s]);
  const int64_t tend = n8 > 0 ? tbase + n8 : (n4 > 0 ? tbase + n4 : a.nt8 + a.nt4 + a.task_off[s + 1]);
  const int64_t o = tbase + __popcll(reps & ((1ull << lane) - 1ull));
  if (o >= tend) return;  // the count (k_prep's nroot) and this rule agree; never write past it
  const uint32_t bmm = (uint32_t)bound_mm_of(a.bound[s]);
  const int32_t bt = a.bt[s];
  const uint32_t sh = pack_shift(bt);
#ifdef OTR_FORCE_GENERAL
  const bool general = true;  // test build: every search in k_general (tests/test_gpu_tiers.py)
#else
  const bool general = !pack_fits(bmm, sh) || turn;
#endif
  uint32_t pre = 0u;
  if (a.est_first_keys > 0 && !general && !turn && !a.forced[s]) {
    float reach = (float)bmm * 1e-3f;
    if (bt >= 0) reach = fminf(reach, (float)bt * 0.1f * a.est_v[md]);
    const float est = a.est_k * reach * reach;
    if (est > (float)a.est_first_keys) {
      uint32_t st = 0;
      while ((int)st + 1 < a.n_tiers && (float)a.tier_keys[st] < est) ++st;
      pre = 1u | (st << 1);
    }
  }
  const uint32_t meta = (uint32_t)a.cand_count[s] | ((uint32_t)md << 8) | ((a.forced[s] ? 1u : 0u) << 10) |
                        (sh << 11) | ((general ? 1u : 0u) << 16) | (turn << 17) | (pre << 18);
  const int64_t to = a.trans_off[s];
  if (turn && a.flag_turn) a.flag_turn[o] = 5;  // the edge-state tiers (otr_edge1.h)
  a.rec[3 * o] = make_uint4((uint32_t)s, (uint32_t)sp, root, bmm);
  a.rec[3 * o + 1] = make_uint4(d0min, meta, (uint32_t)same, (uint32_t)(same >> 32));
  a.rec[3 * o + 2] = make_uint4(0u, (uint32_t)bt, (uint32_t)to, (uint32_t)((uint64_t)to >> 32));
}

// waves per SIMD of the first tier (two searches per wave): 8 = 32 waves per CU, whose
// 4.7 KB tables fill 150 of the CU's 160 KB of LDS; the search waits on LDS and L2 round
// trips, so the eighth wave pays (20.2 ms against 21.5 at 7, profiles/r03_abw8_*)
#ifndef OTR_ROUTE2_WAVES
#define OTR_ROUTE2_WAVES 8
#endif

// index of the q-th set bit of m (q < popcount(m))
__device__ inline int nth_set_bit(unsigned long long m, int q) {
  for (int j = 0; j < q; ++j) m &= m - 1;
  return __ffsll((long long)m) - 1;
}

// one unit = G search tasks of the wave (ordinal w of the task range or list).  LIST =
// false: the first tier, one unit per block over all tasks (XCD-mapped); LIST = true: a
// retry tier, a fixed grid whose waves claim units of the device-side task list from
// per-XCD queues (its length never crosses to the host).  WIDE: the table keeps 64-bit
// packed words and takes the tasks whose (length << sh | time) words do not fit 32 bits
// (`general` in the record).  The LDS tiers run node-mode tasks; turn-mode (edge-state)
// tasks carry flag 5 from k_tasks and run in the edge-state tiers (otr_edge1.h), then
// k_general.
template <int CAP, int G, bool LIST, bool WIDE = false, bool CNT = true>
__device__ __forceinline__ void route_unit(const DevGraph& gr, const RouteArgs& a, unsigned long long* counters,
                                           SearchLds<CAP, WIDE ? 2 : 0>* Ls, int64_t w, int64_t n_tasks,
                                           uint32_t* sink, uint4 (*trec)[3]) {
  constexpr int LM = WIDE ? 2 : 0;
  using Gr = Grp<G>;
  const int lane = Gr::gl();
  const int64_t tw = (LIST ? 0 : a.task_base) + w * G + Gr::g();
  const bool have = tw < n_tasks;
  const int64_t task = have ? (LIST ? a.task_list[tw] : tw) : 0;
  OTR_STAMP(ts_in);
  // ---- search inputs (only these stay live through the search)
  bool search, fits, forced;
  int start_tier = -1;  // >= 0: the retry tier this (first-tier) task starts in
  uint32_t tnode = kEmpty, tpart = 0, gapT = 1, d0min = 0xFFFFFFFFu, root = 0, bmm = 0, mode_bit = 1;
  uint32_t pd = 0, pt = 0xFFFFFFFFu;  // pruning bounds relative to the root (length, time)
  int Kb;
  Pack K;
  {
    const uint4 r0 = have ? a.rec[3 * task] : make_uint4(0u, 0u, 0u, 0u);
    const uint4 r1 = have ? a.rec[3 * task + 1] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
    const uint4 r2 = have ? a.rec[3 * task + 2] : make_uint4(0u, 0u, 0u, 0u);
    // the record, stashed in LDS for the transition rows (one LDS read after the search
    // instead of an L2 round trip ahead of the rows' own loads)
    if (lane == 0) {
      trec[Gr::g()][0] = r0;
      trec[Gr::g()][1] = r1;
      trec[Gr::g()][2] = r2;
    }
    const int64_t s = r0.x;
    const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
    const int64_t sp = r0.y;
    Kb = (int)(r1.y & 0xFFu);
    K.sh = (r1.y >> 11) & 31u;
    const bool general = (r1.y >> 16) & 1u;  // re-read after the search
    // targets are lanes of the group (wider steps go to a G = 1 tier); 32-bit tables leave
    // the tasks whose packed words need 64 bits to the WIDE tier
    fits = Kb <= Gr::GL && (WIDE || !general) && !((r1.y >> 17) & 1u);
    // a step too big for this table starts in a retry tier (k_tasks' estimate): no load of it
    const bool pre = G >= 2 && !LIST && have && ((r1.y >> 18) & 1u);
    if (pre) {
      start_tier = (int)((r1.y >> 19) & 7u);
      fits = false;
    }
    mode_bit = 1u << ((r1.y >> 8) & 3u);
    bmm = r0.w;
    root = r0.z;
    d0min = r1.x;
    const int32_t bt = (int32_t)r2.y;
    uint32_t ej = 0;
    double pj = 0;
    bool needed = false;
    uint4 cq = make_uint4(0u, 0u, 0u, 0u);
    if (have && !pre && lane < Kb) {
      ej = a.cand_edge[s * OTR_KMAX + lane];
      pj = a.cand_p[s * OTR_KMAX + lane];
      cq = a.cprep[s * OTR_KMAX + lane];
      tpart = cq.x;
    }
    // the task's sources staged one per lane (lane q: the q-th set bit of mask), read in
    // the loop by group shuffles: one parallel load instead of a dependent one per source
    const int nsrc = have && !pre ? __popcll(mask) : 0;
    const int iq = lane < nsrc ? nth_set_bit(mask, lane) : 0;
    uint32_t e_q = 0, t_q = 0;
    double p_q = 0;
    if (lane < nsrc) {
      e_q = a.cand_edge[sp * OTR_KMAX + iq];
      p_q = a.cand_p[sp * OTR_KMAX + iq];
      if (bt >= 0) t_q = a.cprep_t[sp * OTR_KMAX + iq].y;  // the task's common exit time
    }
    for (int q = 0; q < nsrc; ++q) {  // group-uniform trip count
      uint32_t ei;
      double pi;
      if (q < Gr::GL) {
        ei = (uint32_t)__shfl((int)e_q, q, Gr::GL);
        pi = __shfl(p_q, q, Gr::GL);
      } else {  // more sources than lanes (K > 32 at G = 2): direct loads
        const int i = nth_set_bit(mask, q);
        ei = a.cand_edge[sp * OTR_KMAX + i];
        pi = a.cand_p[sp * OTR_KMAX + i];
      }
      if (lane < Kb && !(ej == ei && pj >= pi)) needed = true;
    }
    // the bounds relative to the root: B - (smallest exit part) and bt - (the task's exit
    // time); a task whose exit parts alone break a bound has no route through the graph
    const uint32_t t0 = (uint32_t)__shfl((int)t_q, 0, Gr::GL);
    bool feasible_root = d0min <= bmm;
    pd = feasible_root ? bmm - d0min : 0u;
    if (bt >= 0) {
      feasible_root = feasible_root && t0 <= (uint32_t)bt;
      pt = t0 <= (uint32_t)bt ? (uint32_t)bt - t0 : 0u;
    }
    forced = have && ((r1.y >> 10) & 1u);
    const unsigned long long need_mask = __ballot(needed);
    search = have && fits && !forced && feasible_root && Gr::mine(need_mask) != 0ull;
    if (needed) {
      tnode = cq.y;
      gapT = cq.z ? cq.z : 1u;  // minin(target node), >= 1 mm
    }
  }
  unsigned long long settled = 0, relaxed = 0, rounds = 0;
  OTR_STAMP(ts_set);
  // a retry tier resumes the search the previous tier outgrew (its dump slot, task_dump)
  // and dumps what outgrows this table for the next one (NDump)
  NDump nd{};
  int dslot = -1;
  constexpr bool kIn = LIST && !WIDE && CAP >= OTR_ND_IN_MIN, kOut = LIST && !WIDE && CAP >= OTR_ND_OUT_MIN;
  constexpr bool kDumps = kIn || kOut;
  if (kIn) {
    const int32_t rs = (a.dump_in != nullptr && search) ? a.task_dump[task] : -1;
    nd.in = rs >= 0 ? a.dump_in + (size_t)rs * a.dump_in_words : nullptr;
  }
  if (kOut) {
    nd.base = a.dump_out;
    nd.ctr = a.dump_ctr;
    nd.words = a.dump_out_words;
    nd.slots = a.dump_out_slots;
#ifdef OTR_FORCE_RETRY
    nd.stop_rounds = (a.force_edge >> 7) & 1 ? 2 + Gr::g() : 0;  // (G = 2: the groups stop in different rounds)
#endif
  }
  search_init<CAP, LM, G>(Ls);
  bool ok = search_run<CAP, LM, G, kIn, kOut>(Ls, gr, K, mode_bit, search, root, pd, pt, tnode, tpart, gapT, Kb, &settled,
                                   &relaxed, &rounds, counters ? counters + 16 * kCShards : nullptr, sink,
                                   kDumps ? &nd : nullptr, kDumps ? &dslot : nullptr) &&
            fits;
#ifdef OTR_FORCE_RETRY
  if (G >= 2 && !LIST) ok = false;  // test build: every first-tier task takes the retry tiers
#endif
  OTR_STAMP(ts_srch);
  SearchLds<CAP, LM>& L = Ls[Gr::g()];
  int64_t lab = -1;
  if (ok && search && tnode != kEmpty && !forced) {
    const int sl = lds_find(L, tnode);
    if (sl >= 0 && LabelT<LM>::label(L.lab[sl]) != LabelT<LM>::kNone) lab = (int64_t)LabelT<LM>::label(L.lab[sl]);
  }
  // ---- transition rows: re-read the step (cached) rather than hold it live through the search
  asm volatile("" ::: "memory");
  uint32_t ntr = 0;  // transition entries this search wrote (K4), for the work counters
  if (have && forced && Kb > Gr::GL) {
    // a step beyond the breakage distance with more targets than the group has lanes (a
    // mode keeping > 32 candidates, G = 2): no route for any of them, written by stride
    const uint4 r1 = trec[Gr::g()][1], r2 = trec[Gr::g()][2];
    const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
    uint32_t* trow = a.trans + (int64_t)(((uint64_t)r2.w << 32) | r2.z);
    for (int q = 0; q < __popcll(mask); ++q) {  // (group-uniform)
      const int i = nth_set_bit(mask, q);
      for (int j = lane; j < Kb; j += Gr::GL) trow[(int64_t)i * Kb + j] = kNoRoute;
    }
  } else if (have && (ok || forced)) {
    const uint4 r0 = trec[Gr::g()][0], r1 = trec[Gr::g()][1], r2 = trec[Gr::g()][2];
    const int64_t s = r0.x;
    const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
    if (search) ntr = (uint32_t)Kb * (uint32_t)__popcll(mask);
    const int64_t sp = r0.y;
    const int32_t bt = (int32_t)r2.y;
    uint32_t* trow = a.trans + (int64_t)(((uint64_t)r2.w << 32) | r2.z);
    // sources staged one per lane as in the setup: {index, edge, fraction, exit part mm,
    // exit part time, edge length mm, edge time}, read by group shuffles in the row loop
    const int nsrc = __popcll(mask);
    const int iq = lane < nsrc ? nth_set_bit(mask, lane) : 0;
    uint32_t e_q = 0, w_q = 0, t_q = 0;
    uint2 l_q = make_uint2(0u, 0u);
    double p_q = 0;
    if (lane < nsrc) {
      e_q = a.cand_edge[sp * OTR_KMAX + iq];
      p_q = a.cand_p[sp * OTR_KMAX + iq];
      w_q = a.cprep[sp * OTR_KMAX + iq].w;
      if (bt >= 0) t_q = a.cprep_t[sp * OTR_KMAX + iq].y;
      l_q = a.clen[sp * OTR_KMAX + iq];
    }
    uint32_t ej = 0, tpt = 0;
    double pj = 0;
    if (lane < Kb) {
      ej = a.cand_edge[s * OTR_KMAX + lane];
      pj = a.cand_p[s * OTR_KMAX + lane];
      tpt = bt >= 0 ? a.cprep_t[s * OTR_KMAX + lane].x : 0u;
    }
    for (int q = 0; q < nsrc; ++q) {  // group-uniform trip count
      int i;
      uint32_t ei, wi, ti, li, lti;
      double pi;
      if (q < Gr::GL) {
        i = __shfl(iq, q, Gr::GL);
        ei = (uint32_t)__shfl((int)e_q, q, Gr::GL);
        pi = __shfl(p_q, q, Gr::GL);
        wi = (uint32_t)__shfl((int)w_q, q, Gr::GL);
        ti = (uint32_t)__shfl((int)t_q, q, Gr::GL);
        li = (uint32_t)__shfl((int)l_q.x, q, Gr::GL);
        lti = (uint32_t)__shfl((int)l_q.y, q, Gr::GL);
      } else {  // more sources than lanes (K > 32 at G = 2): direct loads
        i = nth_set_bit(mask, q);
        ei = a.cand_edge[sp * OTR_KMAX + i];
        pi = a.cand_p[sp * OTR_KMAX + i];
        wi = a.cprep[sp * OTR_KMAX + i].w;
        ti = bt >= 0 ? a.cprep_t[sp * OTR_KMAX + i].y : 0u;
        const uint2 l = a.clen[sp * OTR_KMAX + i];
        li = l.x;
        lti = l.y;
      }
      if (lane < Kb) {
        int64_t r = -1, rt = 0;
        if (forced) {
          r = -1;
        } else if (ej == ei && pj >= pi) {
          r = part_mm(pj - pi, li);  // li = len_mm[ei], lti = et(md)[ei] (k_prep)
          if (bt >= 0) rt = part_mm(pj - pi, lti);
        } else if (lab >= 0) {
          // the target's offer: its node's label plus the entry part, within both bounds
          r = (int64_t)wi + K.d((uint64_t)lab) + tpart;
          if (bt >= 0) rt = (int64_t)ti + K.t((uint64_t)lab) + tpt;
        }
        const bool valid = r >= 0 && r <= (int64_t)bmm && (bt < 0 || rt <= (int64_t)bt);
        trow[(int64_t)i * Kb + lane] = valid ? (uint32_t)r : kNoRoute;
      }
    }
  }
  // general (flag 3): the global-memory search; overflow: retry with a bigger table (1); a
  // first-tier search expected beyond its table starts in retry tier t (16 + t); turn modes:
  // none here (k_tasks flagged them 5, for the edge-state tiers otr_edge1.h / otr_edge.h)
  if (have && !ok && !forced && lane == 0) {
    const uint32_t meta = a.rec[3 * task + 1].y;
    const bool general = ((meta >> 16) & 1u) != 0u, turn = ((meta >> 17) & 1u) != 0u;
#ifdef OTR_FORCE_GENERAL
    a.overflow_flag[task] = 3;  // test build: every search (edge-state ones too) in k_general
#else
    // (turn-mode tasks carry flag 5 from k_tasks: the edge-state tiers take them)
    if (!turn) a.overflow_flag[task] = general ? 3 : (start_tier >= 0 ? 16 + start_tier : 1);
#endif
    if (!WIDE && !turn && a.task_dump != nullptr) a.task_dump[task] = dslot;  // (-1: the next tier restarts it)
  }
#ifdef OTR_STAMPS
  if (G == 2 && counters && threadIdx.x == 0) {  // task setup and transition rows, wave cycles
    OTR_STAMP(ts_out);
    const int sh = cshard();
    atomicAdd(&counters[20 * kCShards + sh], ts_set - ts_in);
    atomicAdd(&counters[21 * kCShards + sh], ts_out - ts_srch);
  }
#endif
  if (CNT && counters) {
    // wave totals: lane sums by DPP, per-group values read from each group's lane 0
    settled = wave_sum_u32((uint32_t)settled);
    relaxed = wave_sum_u32((uint32_t)relaxed);
    rounds = wave_sum_u32((uint32_t)rounds);
    const int nk = have && search ? L.n_keys : 0;
    unsigned long long kk = 0, ntrw = 0, nsearch = 0, nres = 0, ndmp = 0;
    const int rd = (kDumps && nd.in != nullptr ? 1 : 0) | (dslot >= 0 ? 2 : 0);
    for (int q = 0; q < G; ++q) {
      kk += (unsigned long long)__builtin_amdgcn_readlane(nk, q * Gr::GL);
      ntrw += (unsigned long long)__builtin_amdgcn_readlane(ntr, q * Gr::GL);
      nsearch += (unsigned long long)__builtin_amdgcn_readlane((int)(have && search), q * Gr::GL);
      const int rdq = __builtin_amdgcn_readlane(rd, q * Gr::GL);
      nres += rdq & 1;
      ndmp += rdq >> 1;
    }
    if (threadIdx.x == 0) {
      const int sh = cshard();
      atomicAdd(&counters[3 * kCShards + sh], settled);
      atomicAdd(&counters[4 * kCShards + sh], relaxed);
      atomicAdd(&counters[5 * kCShards + sh], ntrw);
      atomicAdd(&counters[6 * kCShards + sh], nsearch);
      atomicAdd(&counters[13 * kCShards + sh], rounds);
      atomicAdd(&counters[14 * kCShards + sh], kk);
      if (nres) atomicAdd(&counters[11 * kCShards + sh], nres);  // resumed from a dump
      if (ndmp) atomicAdd(&counters[12 * kCShards + sh], ndmp);  // dumped for the next tier
    }
  }
}

// CNT = false: the timed launches, compiled without the work counting (the per-lane
// settled / relaxed / round tallies are dead code there: fewer registers and
// instructions in the search loop); CNT = true: the instrumented launches
// (OTR_BATCH_ROUTE_WORK) that fill the work counters
template <int CAP, int G, bool LIST, bool WIDE = false, bool CNT = true>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(G == 2 ? OTR_ROUTE2_WAVES : 8, G == 2 ? OTR_ROUTE2_WAVES : 8))) void k_route(DevGraph gr, RouteArgs a, unsigned long long* counters) {
  __shared__ SearchLds<CAP, WIDE ? 2 : 0> Ls[G];
  __shared__ uint4 trec[G][3];  // each group's task record, for its transition rows
#ifdef OTR_NO_SINK
  uint32_t* sink = nullptr;  // A/B build: the branching relax_one everywhere
#else
  __shared__ uint32_t sink_row[OTR_WAVE];  // relax_sink's per-lane scratch words (32-bit tables)
  uint32_t* sink = WIDE ? nullptr : sink_row;
#endif
  if (!LIST) {
    const int64_t n_units = (a.n_tasks - a.task_base + G - 1) / G;
    // the first tier (task-major; the default is k_route_step): one unit per block,
    // XCD-mapped (no loop: fewer live registers); units [unit_base, unit_base + gridDim.x):
    // a launch's grid stays below 2^32 work-items (the dispatch packet's grid size), so a
    // large batch is several launches
    const int64_t w = a.unit_base + xcd_remap(blockIdx.x, (int64_t)gridDim.x / 8);
    if (w < n_units) route_unit<CAP, G, LIST, WIDE, CNT>(gr, a, counters, Ls, w, a.n_tasks, sink, trec);
    return;
  }
  const int64_t n_tasks = (int64_t)*a.list_count;
  const int64_t n_units = (n_tasks + G - 1) / G;
  XcdQueue q(a.queue, n_units);
  for (int64_t w = q.next(); w < q.hi; w = q.next()) {
    route_unit<CAP, G, LIST, WIDE, CNT>(gr, a, counters, Ls, w, n_tasks, sink, trec);
    __syncthreads();  // the next unit re-initialises the tables
  }
}

// ------------------------------------------------------------------------------
// K5: fp64 Viterbi, one wave per trace, lane j = candidate of the current state.
// ------------------------------------------------------------------------------
struct ViterbiArgs {
  int32_t n_traces;
  const int64_t* trace_state_off;
  const int32_t* cand_count;
  const double* cand_sqd;
  const int64_t* prev;
  const int64_t* trans_off;
  const uint32_t* trans;   // route mm per transition (k_route), kNoRoute when invalid
  const uint32_t* trans_tc;  // turn cost mm per transition (modes with turn costs only)
  uint32_t turn_modes;     // bit m: mode m has turn costs
  const double* g;         // great-circle distance of the step ending at the state
  const uint8_t* mode;
  double inv2s2[OTR_MODES];
  double inv_beta[OTR_MODES];
  int8_t* bp;          // [n_states][OTR_KMAX]
  uint8_t* brk;        // sub-path starts here
  int32_t* end_win;    // winner of a state that ends a sub-path
  int32_t* winner;
  int32_t* subpath;
};

// x / 1000.0 for integral x in [0, 2^32), correctly rounded without a division: product
// with RN(1/1000), exact residual by fma, one fma correction.  Equal to the IEEE quotient
// for every such x (exhaustive check: tests/div1000_check.c, tests/test_div1000.py).
__device__ inline double div1000(double x) {
  const double q0 = x * 0.001;
  const double e = __builtin_fma(-q0, 1000.0, x);
  return __builtin_fma(e, 0.001, q0);
}

// lowest-index argmin over the GL lanes of my group (GL = 64 / G)
template <int G>
__device__ inline void argmin_lane(double c, int j, double* oc, int* oj) {
  for (int off = OTR_WAVE / G / 2; off > 0; off >>= 1) {
    const double c2 = __shfl_xor(c, off);
    const int j2 = __shfl_xor(j, off);
    if (c2 < c || (c2 == c && j2 < j)) {
      c = c2;
      j = j2;
    }
  }
  *oc = c;
  *oj = j;
}

// Back-pointers, break flags and sub-path-end winners of a trace's states are also kept
// in LDS (traces of up to VitLds<G>::N states, K <= 32) so the serial backtrack reads LDS
// instead of a chain of dependent global loads; other traces use the global copies.
// G = 2 (every mode's max_candidates <= 32): two traces per wave, 32 lanes each, and a
// table of 104 states per trace (7.6 KB per wave: five waves per SIMD, so a C2 batch's
// 5,000 waves are resident at once instead of 10,000 one-trace waves in two rounds).
template <int G>
struct VitLds {
  static constexpr int N = G == 1 ? 128 : 104;
};

// One Viterbi step's min-plus scan for lane j < K: 16 independent transition loads in
// flight per chunk, then ascending i (strict <: lowest index among equal minima).  The
// array holds route lengths (u32 mm, half the bytes of a cost); the transition cost
// (turn_cost + |route - gc|) / beta (K4) is evaluated here.  TURNS = false: no trace of
// the wave has turn costs, so the turn term (0) is not added; TURNS = true: turn costs
// are read where `turn` (my trace's mode has them) and are 0 otherwise (0 + x == x).
// Kw: a wave-uniform bound >= Kp (the larger Kp of the wave's traces): the loads run
// unconditionally at clamped rows (i < Kp), rows past Kp read as no route.  U loads in
// flight per chunk.
template <bool TURNS, int U = 16>
__device__ __forceinline__ void vit_scan(const uint32_t* tr, const uint32_t* tcr, const double* s_cost, int Kp, int Kw,
                                         int K, int lane, double gcd, double inv_beta, bool turn, double* best_io,
                                         int* bi_io) {
  double best = *best_io;
  int bi = *bi_io;
  for (int i0 = 0; i0 < Kw; i0 += U) {
    uint32_t tv[U], tc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u < Kp ? i0 + u : Kp - 1;
      tv[u] = tr[(int64_t)i * K + lane];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u < Kp ? i0 + u : Kp - 1;
      tc[u] = (TURNS && turn) ? tcr[(int64_t)i * K + lane] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + u >= Kp || tv[u] == kNoRoute) continue;
      const double dg = fabs(div1000((double)tv[u]) - gcd);
      const double ti = (TURNS ? div1000((double)tc[u]) + dg : dg) * inv_beta;
      const double ci = s_cost[i0 + u < Kp ? i0 + u : Kp - 1];
      if (ci == __builtin_huge_val()) continue;
      const double c = ci + ti;
      if (c < best) {
        best = c;
        bi = i0 + u;
      }
    }
  }
  *best_io = best;
  *bi_io = bi;
}

// vit_scan over the predecessors i = h, h + 2, ... only (SPLIT: the two halves of a wave
// scan the even and the odd predecessors of candidate j; vit_pair joins them)
template <bool TURNS, int U = 8>
__device__ __forceinline__ void vit_scan_half(const uint32_t* tr, const uint32_t* tcr, const double* s_cost, int Kp,
                                              int K, int j, int h, double gcd, double inv_beta, bool turn,
                                              double* best_io, int* bi_io) {
  double best = *best_io;
  int bi = *bi_io;
  for (int i0 = h; i0 < Kp; i0 += 2 * U) {
    uint32_t tv[U], tc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 2 * u < Kp ? i0 + 2 * u : Kp - 1;  // (rows past Kp: a valid row, skipped below)
      tv[u] = tr[(int64_t)i * K + j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 2 * u < Kp ? i0 + 2 * u : Kp - 1;
      tc[u] = (TURNS && turn) ? tcr[(int64_t)i * K + j] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i0 + 2 * u >= Kp || tv[u] == kNoRoute) continue;
      const double dg = fabs(div1000((double)tv[u]) - gcd);
      const double ti = (TURNS ? div1000((double)tc[u]) + dg : dg) * inv_beta;
      const double ci = s_cost[i0 + 2 * u];
      if (ci == __builtin_huge_val()) continue;
      const double c = ci + ti;
      if (c < best) {
        best = c;
        bi = i0 + 2 * u;
      }
    }
  }
  *best_io = best;
  *bi_io = bi;
}
// the lexicographic (cost, index) minimum of lane and lane ^ 32: the argmin the ascending
// scan over all predecessors finds (strict <: the lowest index among equal minima)
__device__ __forceinline__ void vit_pair(double* best, int* bi) {
  const double ob = __shfl_xor(*best, 32);
  const int obi = __shfl_xor(*bi, 32);
  if (obi >= 0 && (*bi < 0 || ob < *best || (ob == *best && obi < *bi))) {
    *best = ob;
    *bi = obi;
  }
}

// One wave per G traces (group g = lane / GL), lane j = candidate j of the current state.
// The state loop runs to the longer trace of the wave; every per-state decision is
// group-uniform and the LDS hand-over of the state costs sits between two wave-uniform
// barriers.
// SPLIT (G = 1, batches of few traces): a state with K <= 32 candidates scans its
// predecessors in two halves (lanes j and j + 32), halving the step's serial chain.
template <int G, bool SPLIT = false>
__global__ __launch_bounds__(64) void k_viterbi(ViterbiArgs a, unsigned long long* counters) {
  static_assert(!SPLIT || G == 1, "the split scan uses the second half of a one-trace wave");
  constexpr int GL = OTR_WAVE / G;
  constexpr int NL = VitLds<G>::N;
  __shared__ double s_cost[G][OTR_KMAX / G];
  __shared__ int8_t s_bp[G][NL][32];
  __shared__ int8_t s_brk[G][NL];  // 1 break, 0 no break, -1 no candidates
  __shared__ int8_t s_win[G][NL];  // end_win of the states that end a sub-path
  const int gi = G == 1 ? 0 : (int)threadIdx.x / GL;
  const int lane = G == 1 ? (int)threadIdx.x : (int)threadIdx.x % GL;
  double* const cst = s_cost[gi];
  for (int64_t tw = blockIdx.x; tw * G < a.n_traces; tw += gridDim.x) {
    const int64_t t = tw * G + gi;
    const bool have = t < a.n_traces;  // group-uniform
    const int md = have && a.mode[t] < OTR_MODES ? a.mode[t] : 0;
    const double inv2s2 = a.inv2s2[md], inv_beta = a.inv_beta[md];
    const bool turns = (a.turn_modes >> md) & 1u;  // group-uniform
    // wave-uniform: does any trace of the wave have turn costs (one scan variant per wave)
    const bool wturns = G == 1 ? turns : __ballot(turns) != 0ull;
    const int64_t so = have ? a.trace_state_off[t] : 0, eo = have ? a.trace_state_off[t + 1] : 0;
    int64_t len = eo - so;
    if (G == 2) {  // the wave runs to its longer trace
      const int64_t l0 = __builtin_amdgcn_readlane((int)len, 0), l1 = __builtin_amdgcn_readlane((int)len, 32);
      len = l0 > l1 ? l0 : l1;
    }
    int64_t prev_s = -1;
    int Kp = 0;
    bool lds_ok = eo - so <= NL;  // group-uniform: every state cached (and K <= 32, below)
    for (int64_t k = 0; k < len; ++k) {
      const int Kw = G == 1 ? Kp : max(__builtin_amdgcn_readlane(Kp, 0), __builtin_amdgcn_readlane(Kp, 32));
      const int64_t s = so + k;
      const bool in = s < eo;
      const int K = in ? a.cand_count[s] : 0;
      if (in && lds_ok && lane == 0) s_brk[gi][k] = -1;
      const bool act = in && K > 0;  // group-uniform (the state has candidates)
      if (act) lds_ok = lds_ok && K <= 32;
      double emis = 0.0;
      if (act && lane < K) emis = a.cand_sqd[s * OTR_KMAX + lane] * inv2s2;
      double cost = __builtin_huge_val();
      int bi = -1;
      bool brk = prev_s < 0;
      if (act && !brk) {
        double best = __builtin_huge_val();
        const bool split = SPLIT && K <= 32;  // (group-uniform)
        if (split) {
          const uint32_t* tr = a.trans + a.trans_off[s];
          const uint32_t* tcr = a.trans_tc + a.trans_off[s];
          const double gcd = a.g[s];
          const int j = lane & 31;
          if (j < K) {
            if (wturns) vit_scan_half<true>(tr, tcr, cst, Kp, K, j, lane >> 5, gcd, inv_beta, turns, &best, &bi);
            else vit_scan_half<false>(tr, tcr, cst, Kp, K, j, lane >> 5, gcd, inv_beta, false, &best, &bi);
          }
          vit_pair(&best, &bi);
          if (lane >= 32) {
            best = __builtin_huge_val();
            bi = -1;
          }
        } else if (lane < K) {
          // the array holds route lengths (u32 mm); the transition cost (turn_cost +
          // |route - gc|) / beta (K4) is evaluated here.  Without turn costs (group-
          // uniform) the 0 + x term is left out (0 + x == x exactly)
          const uint32_t* tr = a.trans + a.trans_off[s];
          const uint32_t* tcr = a.trans_tc + a.trans_off[s];
          const double gcd = a.g[s];
          // (G = 2: 8 loads in flight per chunk, so the kernel fits five waves per SIMD)
          if (wturns) vit_scan<true, G == 1 ? 16 : 8>(tr, tcr, cst, Kp, Kw, K, lane, gcd, inv_beta, turns, &best, &bi);
          else vit_scan<false, G == 1 ? 16 : 8>(tr, tcr, cst, Kp, Kw, K, lane, gcd, inv_beta, false, &best, &bi);
        }
        const unsigned long long am = __ballot(lane < K && bi >= 0);
        const bool any = (G == 1 ? am : (am >> (GL * gi)) & ((1ull << GL) - 1ull)) != 0ull;
        if (!any) {
          brk = true;
          bi = -1;
        } else {
          cost = bi >= 0 ? best + emis : __builtin_huge_val();
        }
      }
      // a break ends the previous sub-path at prev_s: its winner = lowest-index argmin
      double mc;
      int mj;
      argmin_lane<G>(lane < Kp ? cst[lane] : __builtin_huge_val(), lane < Kp ? lane : OTR_KMAX, &mc, &mj);
      if (act && brk) {
        if (prev_s >= 0) {
          if (lane == 0) a.end_win[prev_s] = mj;
          if (lds_ok && lane == 0) s_win[gi][prev_s - so] = (int8_t)mj;
        }
        cost = emis;
        bi = -1;
      }
      if (act) {
        if (lane < K) a.bp[s * OTR_KMAX + lane] = (int8_t)bi;
        if (lane == 0) a.brk[s] = brk ? 1 : 0;
        if (lds_ok) {
          if (lane < K) s_bp[gi][k][lane] = (int8_t)bi;
          if (lane == 0) s_brk[gi][k] = brk ? 1 : 0;
        }
      }
      __syncthreads();
      if (act && lane < K) cst[lane] = cost;
      __syncthreads();
      if (act) {
        prev_s = s;
        Kp = K;
      }
    }
    {
      double mc;
      int mj;
      argmin_lane<G>(lane < Kp ? cst[lane] : __builtin_huge_val(), lane < Kp ? lane : OTR_KMAX, &mc, &mj);
      if (prev_s >= 0) {
        if (lane == 0) a.end_win[prev_s] = mj;
        if (lds_ok && lane == 0) s_win[gi][prev_s - so] = (int8_t)mj;
      }
    }
    __syncthreads();
    // backtrack (lane 0 of each group), then sub-path ordinals
    if (have && lds_ok && lane == 0) {
      int cur = -1;
      bool next_brk = true;  // "state after this one starts a sub-path" (true past the end)
      for (int64_t s = eo - 1; s >= so; --s) {
        const int k = (int)(s - so);
        const int b = s_brk[gi][k];
        if (b < 0) {
          a.winner[s] = -1;
          continue;
        }
        if (next_brk) cur = s_win[gi][k];
        a.winner[s] = cur;
        if (!b) cur = s_bp[gi][k][cur];
        next_brk = b != 0;
      }
      int sp = -1;
      for (int64_t s = so; s < eo; ++s) {
        const int b = s_brk[gi][s - so];
        sp += b > 0 ? 1 : 0;
        a.subpath[s] = b < 0 ? -1 : sp;
      }
    } else if (have && lane == 0) {
      int cur = -1;
      bool next_brk = true;  // "state after this one starts a sub-path" (true past the end)
      for (int64_t s = eo - 1; s >= so; --s) {
        if (a.cand_count[s] <= 0) {
          a.winner[s] = -1;
          a.subpath[s] = -1;
          continue;
        }
        if (next_brk) cur = a.end_win[s];
        a.winner[s] = cur;
        const bool b = a.brk[s] != 0;
        if (!b) cur = a.bp[s * OTR_KMAX + cur];
        next_brk = b;
      }
      int sp = -1;
      for (int64_t s = so; s < eo; ++s) {
        if (a.cand_count[s] <= 0) continue;
        if (a.brk[s]) ++sp;
        a.subpath[s] = sp;
      }
    }
    __syncthreads();
  }
  (void)counters;
}

// ------------------------------------------------------------------------------
// K6: winner path reconstruction, one wave per step (state s with prev >= 0,
// not a sub-path start).  Single-target search from the root dst(e_i) whose label
// words carry the smallest-id predecessor edge; the walk from T back to the root
// follows them (one edge_src load per path edge).
// ------------------------------------------------------------------------------
struct PathArgs {
  const int64_t* steps;        // state ids to reconstruct
  int64_t n_steps;
  const int64_t* prev;
  const double* bound;
  const uint8_t* brk;
  const int32_t* winner;
  const uint32_t* cand_edge;
  const double* cand_p;
  const int32_t* state_trace;
  const uint8_t* mode;
  const uint4* cprep;          // per state candidate (k_prep)
  const uint2* cprep_t;        // per state candidate: route-time parts (k_prep)
  const int32_t* bt;           // per state: the step's time bound (0.1 s), -1 none
  uint32_t turn_modes;         // bit m: mode m has turn costs (its paths run in k_general)
  const unsigned long long* n_steps_dev;  // number of steps, on the device
  int64_t* path_off;           // per state
  int32_t* path_len;           // per state; -1 = same-edge step
  uint32_t* path;              // bump-allocated edge list
  unsigned long long* cursor;
  int64_t capacity;
  int32_t* overflow_flag;      // per step index: 1 table overflow, 3 global-memory search
  int32_t* cap_flag;           // global: path buffer too small
  const int32_t* cand_count;
  const int64_t* trans_off;    // the route lengths k_route found (u32 mm per transition)
  const uint32_t* trans;
  int force_edge;              // test build only (OTR_FORCE_RETRY): RouteArgs::force_edge bits 3-4
  unsigned long long* queue;   // list tiers: this launch's per-XCD step counters (XcdQueue), zeroed
  bool from_back;              // first tier: its steps are the last *n_steps_dev of steps[0, n_steps)
                               // (k_step_lists: the small-search tier's at the front)
};

// winner-path steps for the small-search path tier (k_paths<OTR_CAP4, 4>): the search is
// bounded by the winning route r (k_paths), so its keys grow with r^2; a node-mode step
// whose estimate est4 * min(B, r)^2 is at most small_keys goes to the front of the step
// list, the rest to the back (k_step_lists)
struct PathClass {
  const int32_t* winner;
  const int64_t* trans_off;
  const uint32_t* trans;
  const double* bound;
  const int32_t* state_trace;
  const uint8_t* mode;
  uint32_t turn_modes;
  float est4;                 // keys per m^2 of route length
  float small_keys;
};

// G searches per wave (G = 2 for the first tier, lanes split 32/32; G = 4 the small-search
// tier, 16 lanes each), each a single-target search from the winner's root with
// predecessor labels.  First tiers: step_list == null, the step count is read on the
// device (n_steps_dev), one unit per block; retry tiers: a fixed grid strides over
// step_list[0 .. *list_count).
template <int CAP, int G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(G >= 2 ? 6 : 8, 8))) void k_paths(DevGraph gr, PathArgs a, const int64_t* step_list, const unsigned long long* list_count) {
  using Gr = Grp<G>;
  __shared__ SearchLds<CAP, true> Ls[G];
  const int gl = Gr::gl();
  const int64_t n_list = (int64_t)(step_list ? *list_count : *a.n_steps_dev);
  const int64_t n_units = (n_list + G - 1) / G;
  // first tier: grid = 8 x (upper bound of units / 8), XCD-mapped, one unit per block;
  // retry tiers: waves claim units from per-XCD queues
  XcdQueue q(a.queue, step_list ? n_units : 0);
  const int64_t wend = step_list ? q.hi : n_units;
  for (int64_t w = step_list ? q.next() : xcd_remap(blockIdx.x, gridDim.x / 8); w < wend;
       w = step_list ? q.next() : wend) {
  const int64_t iw = w * G + Gr::g();
  const bool have = iw < n_list;
  const int64_t k = have ? (step_list ? step_list[iw] : (a.from_back ? a.n_steps - n_list + iw : iw)) : 0;
  const int64_t s = have ? a.steps[k] : 0;
  const int64_t sp = have ? a.prev[s] : 0;
  bool active = false;
  uint32_t S = 0, T = kEmpty, bmm = 0, tpart = 0, gapT = 1, d0 = 0, mode_bit = 1, pd = 0, pt = 0xFFFFFFFFu;
  int mode = 0;
  Pack K;
  K.sh = 0;
  if (have) {
    const int wi = a.winner[sp], wj = a.winner[s];
    const uint32_t ei = a.cand_edge[sp * OTR_KMAX + wi], ej = a.cand_edge[s * OTR_KMAX + wj];
    const double pi = a.cand_p[sp * OTR_KMAX + wi], pj = a.cand_p[s * OTR_KMAX + wj];
    mode = a.mode[a.state_trace[s]] < OTR_MODES ? a.mode[a.state_trace[s]] : 0;
    bmm = (uint32_t)bound_mm_of(a.bound[s]);
    // the winning transition's route (mm, k_route) bounds the search instead of the step's
    // bound: every node of the route and every in-edge achieving a node's label lies within
    // it, so labels, predecessor edges and tie bits along the route are unchanged, while
    // nothing beyond the route's length is relaxed
    {
      const uint32_t r = a.trans[a.trans_off[s] + (int64_t)wi * a.cand_count[s] + wj];
      if (r < bmm) bmm = r;
    }
    const int32_t bt = a.bt[s];
    K.sh = pack_shift(bt);
    if (ej == ei && pj >= pi) {
      if (gl == 0) a.path_len[s] = -1;
    } else if (((a.turn_modes >> mode) & 1u)
#ifdef OTR_FORCE_GENERAL
               && false  // test build: every winner path in k_general
#endif
    ) {
      if (gl == 0) a.overflow_flag[k] = 5;  // turn costs: the edge-state search (otr_edge.h)
    } else if (!pack_fits(bmm, K.sh)
#ifdef OTR_FORCE_GENERAL
               || true
#endif
    ) {
      if (gl == 0) a.overflow_flag[k] = 3;  // 64-bit labels: k_general
    } else {
      active = true;
      mode_bit = 1u << mode;
      const uint4 cs = a.cprep[sp * OTR_KMAX + wi], ct = a.cprep[s * OTR_KMAX + wj];
      d0 = cs.w;
      // the search from the winner's root, pruned at the bounds relative to it (the
      // route's length bounds the length: pruning is monotone in length, so every label
      // on the route is the full step's, route_unit)
      pd = bmm >= d0 ? bmm - d0 : 0u;
      if (bt >= 0) {
        const uint32_t t0 = a.cprep_t[sp * OTR_KMAX + wi].y;
        pt = t0 <= (uint32_t)bt ? (uint32_t)bt - t0 : 0u;
      }
      S = gr.edge_dst[ei];
      T = ct.y;
      gapT = ct.z ? ct.z : 1u;
      tpart = ct.x;
    }
  }
  search_init<CAP, true, G>(Ls);
  const bool ok = search_run<CAP, true, G>(Ls, gr, K, mode_bit, active, S, pd, pt, gl == 0 ? T : kEmpty, tpart, gapT,
                                           1, nullptr, nullptr, nullptr);
  SearchLds<CAP, true>& L = Ls[Gr::g()];
  if (active && !ok) {
    if (gl == 0) a.overflow_flag[k] = 1;  // the next (larger) table
    active = false;
  }
  // walk predecessor edges T → S (the group's lane 0).  The predecessor node of every
  // labelled slot, src(pred edge), is loaded first by all lanes in parallel (one memory
  // latency instead of one per path edge), into the pend + work area (>= CAP u32); the
  // walks then stay in LDS: one to count the edges, one to store them in path order.
  static_assert(sizeof(L.pend) + sizeof(L.work) >= 4 * CAP, "predecessor nodes reuse pend + work");
  using PL = SearchLds<CAP, true>;
  static_assert(offsetof(PL, work) == offsetof(PL, pend) + sizeof(L.pend), "pend and work are contiguous");
  uint32_t* pn = reinterpret_cast<uint32_t*>(L.pend);  // pend+work are contiguous: >= CAP u32
  constexpr int kPer = (CAP + Gr::GL - 1) / Gr::GL;
  if (active) {
    for (int r0 = 0; r0 < kPer; r0 += 8) {  // 8 loads in flight per lane
      uint32_t u[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int q = gl + (r0 + r) * Gr::GL;
        u[r] = kEmpty;
        if (q < CAP && L.key[q] != kEmpty) {
          const uint32_t e = (uint32_t)(L.lab[q] & 0xFFFFFFFFull);
          if (e != kEmpty) u[r] = gr.edge_src[e];
        }
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (gl + (r0 + r) * Gr::GL < CAP) pn[gl + (r0 + r) * Gr::GL] = u[r];
    }
  }
  __syncthreads();
  int n = 0;
  if (active && gl == 0) {
    uint32_t v = T;
    while (v != S) {
      const int sv = lds_find(L, v);
      const uint32_t e = sv >= 0 ? (uint32_t)(L.lab[sv] & 0xFFFFFFFFull) : kEmpty;
      if (e == kEmpty || n >= CAP) {
        n = -1;
        break;
      }
      ++n;
      v = pn[sv];
    }
  }
  n = __shfl(n, Gr::g() * Gr::GL);
  if (active && n < 0) {
    if (gl == 0) a.overflow_flag[k] = 1;
    active = false;
  }
  // bump allocation in one of 64 regions (a single cursor serialises ~1M returning
  // atomics on one address)
  const int shard = (int)((blockIdx.x * G + Gr::g()) & (kShards - 1));
  const int64_t region = a.capacity / kShards;
  int64_t off = 0;
  if (active && gl == 0) off = (int64_t)atomicAdd(&a.cursor[shard], (unsigned long long)n);
  off = __shfl(off, Gr::g() * Gr::GL);
  if (active && off + n > region) {
    if (gl == 0) *a.cap_flag = 1;
    active = false;
  }
  if (active && gl == 0) {
    off += (int64_t)shard * region;
    uint32_t v = T;
    for (int q = n - 1; q >= 0; --q) {  // the same walk, storing S → T order
      const int sv = lds_find(L, v);
      a.path[off + q] = (uint32_t)(L.lab[sv] & 0xFFFFFFFFull);
      v = pn[sv];
    }
    a.path_off[s] = off;
    a.path_len[s] = n;
  }
  __syncthreads();
  }
}

// ------------------------------------------------------------------------------
// K7: route stitching, OSMLR traffic segments and report(), one wave per trace.
//
// Route positions are integer millimetres, so the oracle's sequential stitching is an
// exact segmented prefix sum: the wave scans states 64 at a time (positions, the entry
// position of the current edge, sub-path starts), emits edge portions and route edges
// at scanned offsets, finds segment groups by comparing each portion with its
// predecessor, fills every segment lane-parallel (binary searches for times and shape
// indices), and runs the short report() state machine on lane 0.  Outputs sit at the
// trace's capacity offset cap_off[t]; counts in *_n.
// ------------------------------------------------------------------------------
struct SegArgs {
  BatchDev b;
  const int64_t* trace_state_off;
  const int64_t* state_probe;
  const int32_t* cand_count;
  const uint32_t* cand_edge;
  const double* cand_p;
  const int64_t* prev;
  const uint8_t* brk;
  const int32_t* winner;
  const int64_t* path_off;
  const int32_t* path_len;
  const uint32_t* path;
  // scratch per state (indexed by active ordinal from trace_state_off[t])
  int64_t* pos;                // route position of the state, mm
  int64_t* ent;                // position where the state's current edge was entered, mm
  int64_t* act;                // compact active state list
  int32_t* suba;               // first active ordinal of the state's sub-path
  int32_t* subb;               // at a sub-path's first ordinal: its last ordinal
  // scratch at capacity offsets
  uint32_t* por_e;  int64_t* por_s0;  int64_t* por_s1;  int32_t* por_sa;  int32_t* gstart;
  const int64_t* cap_off;      // per trace capacity offset (route/segments/ways/reports)
  int64_t n_traces_pad;
  uint32_t* route;  int64_t* route_n;
  unsigned long long* seg_id;  double* seg_start;  double* seg_end;  int32_t* seg_length;
  int32_t* seg_queue;  uint8_t* seg_internal;  int32_t* seg_bshape;  int32_t* seg_eshape;
  uint32_t* seg_index;  int64_t* seg_n;
  int64_t* seg_way_n;  uint32_t* seg_way;  int64_t* way_n;
  unsigned long long* rep_id;  unsigned long long* rep_next;  double* rep_t0;  double* rep_t1;
  int32_t* rep_length;  int32_t* rep_queue;  uint32_t* rep_seg;  int64_t* rep_n;
  int32_t* shape_used;  int32_t* stats;  double* stats_len;
  double threshold;
  uint32_t report_levels, transition_levels;
  double queue_kph[OTR_MODES];  // queue_length speed threshold per mode
};

template <class T>
__device__ inline T wave_excl_sum(T v, T* total) {
  const int lane = threadIdx.x;
  T x = v;
  for (int off = 1; off < OTR_WAVE; off <<= 1) {
    const T u = __shfl_up(x, off);
    if (lane >= off) x += u;
  }
  *total = __shfl(x, OTR_WAVE - 1);
  return x - v;
}

// does portion edge e continue the segment group whose last edge is ep?
__device__ inline bool group_continues(const DevGraph& g, uint32_t ep, uint32_t e) {
  const uint32_t key = g.edge_seg[ep];
  if (key != OTR_NO_SEGMENT)
    return g.edge_seg[e] == key && !(g.edge_attr[ep] & OTR_ATTR_SEG_END) && !(g.edge_attr[e] & OTR_ATTR_SEG_BEGIN);
  return g.edge_seg[e] == OTR_NO_SEGMENT &&
         ((g.edge_attr[e] & OTR_ATTR_INTERNAL) != 0) == ((g.edge_attr[ep] & OTR_ATTR_INTERNAL) != 0);
}

__global__ __launch_bounds__(64) void k_segments(DevGraph g, SegArgs a, unsigned long long* counters) {
  const int lane = threadIdx.x;
  const int64_t t = xcd_remap(blockIdx.x, (a.b.n_traces + 7) / 8);
  if (t >= a.b.n_traces) return;
  const int64_t so = a.trace_state_off[t], eo = a.trace_state_off[t + 1];
  const int64_t lo_probe = a.b.trace_off[t], n_probe = a.b.trace_off[t + 1] - lo_probe;
  const int64_t co = a.cap_off[t];
  const double qkph = a.queue_kph[a.b.mode[t] < OTR_MODES ? a.b.mode[t] : 0];
  int64_t* act = a.act + so;
  int64_t* pos = a.pos + so;
  int64_t* ent = a.ent + so;
  int32_t* suba = a.suba + so;
  int32_t* subb = a.subb + so;
  // ---- A1: compact the active states
  int na = 0;
  for (int64_t base = so; base < eo; base += OTR_WAVE) {
    const int64_t s = base + lane;
    const bool on = s < eo && a.cand_count[s] > 0;
    const unsigned long long m = __ballot(on);
    if (on) act[na + prefix_count(m)] = s;
    na += __popcll(m);
  }
  __syncthreads();
  // ---- A2: positions, portions and route edges, 64 states at a time
  int64_t c_pos = 0, c_ent = 0, n_por = 0, n_route = 0;
  int c_sa = 0;
  bool emitted_any = false;
  for (int kb = 0; kb < na; kb += OTR_WAVE) {
    const int k = kb + lane;
    const bool valid = k < na;
    int64_t s = 0;
    bool brk_k = false, last_k = false, same = false, change = false;
    uint32_t ek = 0, ep = 0;
    double pk = 0, pp = 0;
    int pl = 0;
    int64_t inc = 0;
    if (valid) {
      s = act[k];
      brk_k = a.brk[s] != 0;
      last_k = (k == na - 1) || a.brk[act[k + 1]] != 0;
      ek = a.cand_edge[s * OTR_KMAX + a.winner[s]];
      pk = a.cand_p[s * OTR_KMAX + a.winner[s]];
      if (!brk_k) {
        const int64_t sp = act[k - 1];
        ep = a.cand_edge[sp * OTR_KMAX + a.winner[sp]];
        pp = a.cand_p[sp * OTR_KMAX + a.winner[sp]];
        same = ek == ep && pk >= pp;
        change = !same;
      }
      if (same) inc = part_mm(pk - pp, g.len_mm[ep]);
      if (change) {
        pl = a.path_len[s];
        inc = part_mm(1.0 - pp, g.len_mm[ep]);
        for (int z = 0; z < pl; ++z) inc += (int64_t)g.len_mm[a.path[a.path_off[s] + z]];
        inc += part_mm(pk, g.len_mm[ek]);
      }
    }
    // segmented inclusive scan of the position increments (segments start at brk)
    int64_t v = inc;
    bool f = brk_k;
    for (int off = 1; off < OTR_WAVE; off <<= 1) {
      const int64_t vu = __shfl_up(v, off);
      const bool fu = __shfl_up((int)f, off) != 0;
      if (lane >= off) {
        if (!f) v += vu;
        f = f || fu;
      }
    }
    if (!f) v += c_pos;
    const int64_t pos_k = v;
    // entry position of the current edge: defined at sub-path starts and edge changes
    int64_t ev = brk_k ? 0 : (change ? pos_k - part_mm(pk, g.len_mm[ek]) : 0);
    bool eh = brk_k || change;
    int sv = brk_k ? k : 0;
    bool sh = brk_k;
    for (int off = 1; off < OTR_WAVE; off <<= 1) {
      const int64_t vu = __shfl_up(ev, off);
      const bool hu = __shfl_up((int)eh, off) != 0;
      const int su = __shfl_up(sv, off);
      const bool shu = __shfl_up((int)sh, off) != 0;
      if (lane >= off) {
        if (!eh) {
          ev = vu;
          eh = hu;
        }
        if (!sh) {
          sv = su;
          sh = shu;
        }
      }
    }
    if (!eh) ev = c_ent;
    if (!sh) sv = c_sa;
    int64_t ent_prev = __shfl_up(ev, 1), pos_prev = __shfl_up(pos_k, 1);
    if (lane == 0) {
      ent_prev = c_ent;
      pos_prev = c_pos;
    }
    if (valid) {
      pos[k] = pos_k;
      ent[k] = ev;
      suba[k] = sv;
      if (last_k) subb[sv] = k;
    }
    // portion and route-edge counts, offsets by wave scans
    const bool start_emit = valid && brk_k && !last_k;
    const unsigned long long m_se = __ballot(start_emit);
    const bool sep = start_emit && (emitted_any || prefix_count(m_se) > 0);
    const int64_t cnt_por = (change ? 1 + pl : 0) + (valid && last_k && !brk_k ? 1 : 0);
    const int64_t cnt_route = (sep ? 1 : 0) + (start_emit ? 1 : 0) + (change ? pl + 1 : 0);
    int64_t tot_por, tot_route;
    const int64_t por_off = n_por + wave_excl_sum(cnt_por, &tot_por);
    const int64_t route_off = n_route + wave_excl_sum(cnt_route, &tot_route);
    if (valid) {
      int64_t r = co + route_off;
      if (sep) a.route[r++] = 0xFFFFFFFFu;
      if (start_emit) a.route[r++] = ek;
      int64_t q = co + por_off;
      if (change) {
        const int64_t s1 = pos_prev + part_mm(1.0 - pp, g.len_mm[ep]);
        a.por_e[q] = ep;
        a.por_s0[q] = ent_prev;
        a.por_s1[q] = s1;
        a.por_sa[q] = sv;
        ++q;
        int64_t x = s1;
        for (int z = 0; z < pl; ++z) {
          const uint32_t ed = a.path[a.path_off[s] + z];
          const int64_t x1 = x + (int64_t)g.len_mm[ed];
          a.por_e[q] = ed;
          a.por_s0[q] = x;
          a.por_s1[q] = x1;
          a.por_sa[q] = sv;
          ++q;
          x = x1;
          a.route[r++] = ed;
        }
        a.route[r++] = ek;
      }
      if (last_k && !brk_k) {
        a.por_e[q] = ek;
        a.por_s0[q] = ev;
        a.por_s1[q] = pos_k;
        a.por_sa[q] = sv;
      }
    }
    n_por += tot_por;
    n_route += tot_route;
    emitted_any = emitted_any || m_se != 0ull;
    c_pos = __shfl(pos_k, OTR_WAVE - 1);
    c_ent = __shfl(ev, OTR_WAVE - 1);
    c_sa = __shfl(sv, OTR_WAVE - 1);
  }
  __syncthreads();
  // ---- B1: segment-group starts
  int ng = 0;
  for (int64_t qb = 0; qb < n_por; qb += OTR_WAVE) {
    const int64_t q = qb + lane;
    bool st = false;
    if (q < n_por) {
      const uint32_t e = a.por_e[co + q];
      st = q == 0 || a.por_sa[co + q - 1] != a.por_sa[co + q] || !group_continues(g, a.por_e[co + q - 1], e);
    }
    const unsigned long long m = __ballot(st);
    if (st) a.gstart[co + ng + prefix_count(m)] = (int32_t)q;
    ng += __popcll(m);
  }
  __syncthreads();
  // ---- B2: one lane per segment group
  int64_t n_way = 0;
  for (int gb = 0; gb < ng; gb += OTR_WAVE) {
    const int gi = gb + lane;
    const bool valid = gi < ng;
    int64_t cnt_w = 0;
    int32_t first = 0, last = 0;
    if (valid) {
      first = a.gstart[co + gi];
      last = (gi + 1 < ng) ? a.gstart[co + gi + 1] - 1 : (int32_t)n_por - 1;
      uint32_t lw = 0;
      for (int32_t z = first; z <= last; ++z) {
        const uint32_t w = g.edge_way[a.por_e[co + z]];
        if (z == first || w != lw) ++cnt_w;
        lw = w;
      }
    }
    int64_t tot_w;
    const int64_t woff = n_way + wave_excl_sum(cnt_w, &tot_w);
    if (valid) {
      const int64_t o = co + gi;
      const uint32_t e0 = a.por_e[co + first], eL = a.por_e[co + last];
      const int64_t s0 = a.por_s0[co + first], s1 = a.por_s1[co + last];
      const int32_t sa = a.por_sa[co + first];
      const int32_t sb = subb[sa];
      const bool route_first = first == 0 || a.por_sa[co + first - 1] != sa;
      const bool is_last = last == (int32_t)n_por - 1 || a.por_sa[co + last + 1] != sa;
      const uint32_t key = g.edge_seg[e0];
      const bool internal = (g.edge_attr[e0] & OTR_ATTR_INTERNAL) != 0;
      // time at route position x: linear between the states around it (oracle time_at)
      auto time_at = [&](int64_t x) -> double {
        int32_t lo_i = sa + 1, hi_i = sb + 1;  // first ordinal m in [sa+1, sb] with pos[m] >= x
        while (lo_i < hi_i) {
          const int32_t mid = (lo_i + hi_i) >> 1;
          if (pos[mid] >= x) hi_i = mid;
          else lo_i = mid + 1;
        }
        const int32_t kk = (lo_i > sb ? sb : lo_i) - 1;
        const double t0 = (double)a.b.time[a.state_probe[act[kk]]];
        const double t1 = (double)a.b.time[a.state_probe[act[kk + 1]]];
        const int64_t p0 = pos[kk], p1 = pos[kk + 1];
        if (p1 > p0) return t0 + (t1 - t0) * ((double)(x - p0) / (double)(p1 - p0));
        return t0;
      };
      const int64_t lo = sa == 0 ? 0 : a.state_probe[act[sa]] - lo_probe;
      const int64_t hi = (sb + 1 < na) ? a.state_probe[act[sb + 1]] - lo_probe - 1 : n_probe - 1;
      auto shape_at = [&](int64_t x) -> int32_t {
        int32_t lo_i = sa, hi_i = sb + 1;  // last ordinal m in [sa, sb] with pos[m] <= x
        while (lo_i < hi_i) {
          const int32_t mid = (lo_i + hi_i) >> 1;
          if (pos[mid] <= x) lo_i = mid + 1;
          else hi_i = mid;
        }
        const int32_t m = lo_i - 1;
        const int64_t r = (m < sb) ? a.state_probe[act[m + 1]] - lo_probe - 1 : hi;
        return (int32_t)(r < lo ? lo : r);
      };
      double st = -1.0, et = -1.0;
      int32_t length = -1;
      if (key != OTR_NO_SEGMENT) {
        if (!route_first && (g.edge_attr[e0] & OTR_ATTR_SEG_BEGIN)) st = time_at(s0);
        if (!is_last && (g.edge_attr[eL] & OTR_ATTR_SEG_END)) et = time_at(s1);
        if (st != -1.0 && et != -1.0) length = (int32_t)g.seg_len[key];
        a.seg_id[o] = g.seg_id[key];
      } else {
        if (!route_first) st = time_at(s0);
        if (!is_last) et = time_at(s1);
        a.seg_id[o] = OTR_NO_ID_U64;
      }
      // queue_length (README.md:283,295; oracle queue_at): the piece between the states
      // around the exit s1 and the slow pieces right before it, clipped to [s0, s1]
      int32_t queue = 0;
      if (et != -1.0) {
        auto tm_of = [&](int32_t m) { return (double)a.b.time[a.state_probe[act[m]]]; };
        auto slow = [&](int32_t m) { return (double)(pos[m + 1] - pos[m]) * 0.0036 < qkph * (tm_of(m + 1) - tm_of(m)); };
        int32_t lo_i = sa + 1, hi_i = sb + 1;  // first ordinal m in [sa+1, sb] with pos[m] >= s1
        while (lo_i < hi_i) {
          const int32_t mid = (lo_i + hi_i) >> 1;
          if (pos[mid] >= s1) hi_i = mid;
          else lo_i = mid + 1;
        }
        int32_t kq = (lo_i > sb ? sb : lo_i) - 1;
        if (slow(kq)) {
          while (kq > sa && pos[kq] > s0 && slow(kq - 1)) --kq;
          const int64_t q0 = pos[kq] > s0 ? pos[kq] : s0;
          queue = (int32_t)((s1 - q0 + 500) / 1000);
        }
      }
      a.seg_start[o] = st;
      a.seg_end[o] = et;
      a.seg_length[o] = length;
      a.seg_queue[o] = queue;
      a.seg_internal[o] = (key == OTR_NO_SEGMENT && internal) ? 1 : 0;
      a.seg_index[o] = key;
      a.seg_bshape[o] = shape_at(s0);
      a.seg_eshape[o] = shape_at(s1);
      a.seg_way_n[o] = cnt_w;
      int64_t wq = co + woff;
      uint32_t lw = 0;
      for (int32_t z = first; z <= last; ++z) {
        const uint32_t w = g.edge_way[a.por_e[co + z]];
        if (z == first || w != lw) a.seg_way[wq++] = w;
        lw = w;
      }
    }
    n_way += tot_w;
  }
  __syncthreads();
  if (lane == 0) {
    a.route_n[t] = n_route;
    a.seg_n[t] = ng;
    a.way_n[t] = n_way;
    // report() over this trace's segments (reporter_service.py:79-179)
    ReportStats rs;
    const int64_t end_t = n_probe > 0 ? a.b.time[lo_probe + n_probe - 1] : 0;
    report_segments((int32_t)ng, a.seg_id + co, a.seg_start + co, a.seg_end + co, a.seg_internal + co,
                    a.seg_queue + co, nullptr, a.seg_length + co, a.seg_bshape + co, a.seg_index + co, end_t,
                    a.threshold, a.report_levels, a.transition_levels, a.rep_id + co, a.rep_next + co,
                    a.rep_t0 + co, a.rep_t1 + co, a.rep_length + co, a.rep_queue + co, a.rep_seg + co, &rs);
    a.rep_n[t] = rs.n_rep;
    a.shape_used[t] = rs.shape_used;
    for (int q = 0; q < 6; ++q) a.stats[7 * t + q] = rs.counts[q];
    a.stats[7 * t + 6] = 0;
    a.stats_len[2 * t] = rs.lengths[0];
    a.stats_len[2 * t + 1] = rs.lengths[1];
    if (counters) atomicAdd(&counters[7 * kCShards + cshard()], (unsigned long long)ng);
  }
}

// ------------------------------------------------------------------------------
// Copy-out compaction: K7 writes each trace's route / segments / ways / reports at its
// capacity offset; one wave per trace moves them to dense arrays (offsets = scans of
// the per-trace counts) so only used entries cross PCIe.
// ------------------------------------------------------------------------------
struct CompactArgs {
  int32_t n_traces;
  const int64_t* cap_off;
  const int64_t* route_off;  // null: skip the route edges
  const int64_t* seg_off;
  const int64_t* way_off;
  const int64_t* rep_off;
  const SegArgs* s;          // capacity-layout arrays (device copy of the K7 arguments)
  uint32_t* route;
  unsigned long long* seg_id;  double* seg_start;  double* seg_end;  int32_t* seg_length;
  int32_t* seg_queue;  uint8_t* seg_internal;  int32_t* seg_bshape;  int32_t* seg_eshape;
  int64_t* seg_way_n;  uint32_t* seg_way;
  unsigned long long* rep_id;  unsigned long long* rep_next;  double* rep_t0;  double* rep_t1;
  int32_t* rep_length;  int32_t* rep_queue;
};

__global__ __launch_bounds__(64) void k_compact(CompactArgs a) {
  const int t = blockIdx.x;
  if (t >= a.n_traces) return;
  const SegArgs& s = *a.s;
  const int64_t co = a.cap_off[t];
  const int lane = threadIdx.x;
  if (a.route_off) {
    const int64_t o = a.route_off[t], n = a.route_off[t + 1] - o;
    for (int64_t k = lane; k < n; k += 64) a.route[o + k] = s.route[co + k];
  }
  {
    const int64_t o = a.seg_off[t], n = a.seg_off[t + 1] - o;
    for (int64_t k = lane; k < n; k += 64) {
      a.seg_id[o + k] = s.seg_id[co + k];
      a.seg_start[o + k] = s.seg_start[co + k];
      a.seg_end[o + k] = s.seg_end[co + k];
      a.seg_length[o + k] = s.seg_length[co + k];
      a.seg_queue[o + k] = s.seg_queue[co + k];
      a.seg_internal[o + k] = s.seg_internal[co + k];
      a.seg_bshape[o + k] = s.seg_bshape[co + k];
      a.seg_eshape[o + k] = s.seg_eshape[co + k];
      a.seg_way_n[o + k] = s.seg_way_n[co + k];
    }
  }
  {
    const int64_t o = a.way_off[t], n = a.way_off[t + 1] - o;
    for (int64_t k = lane; k < n; k += 64) a.seg_way[o + k] = s.seg_way[co + k];
  }
  {
    const int64_t o = a.rep_off[t], n = a.rep_off[t + 1] - o;
    for (int64_t k = lane; k < n; k += 64) {
      a.rep_id[o + k] = s.rep_id[co + k];
      a.rep_next[o + k] = s.rep_next[co + k];
      a.rep_t0[o + k] = s.rep_t0[co + k];
      a.rep_t1[o + k] = s.rep_t1[co + k];
      a.rep_length[o + k] = s.rep_length[co + k];
      a.rep_queue[o + k] = s.rep_queue[co + k];
    }
  }
}

// inclusive prefix sum over the wave (lane order)
__device__ inline unsigned long long wave_incl_scan_u64(unsigned long long v) {
  const int l = lane_id();
  for (int o = 1; o < OTR_WAVE; o <<= 1) {
    const unsigned long long u = __shfl_up(v, o);
    if (l >= o) v += u;
  }
  return v;
}

// ------------------------------------------------------------------------------
// K8: simple_reporter filter + hour bucketing (simple_reporter.py:176-196) into a
// dense [hour][segment][speed bin] count histogram; one wave per trace, a lane per
// report (one thread per trace left ~40 CUs busy on a 10K-trace batch: 105 us).
// ------------------------------------------------------------------------------
struct HistArgs {
  BatchDev b;
  const int64_t* cap_off;
  const int64_t* rep_n;
  const unsigned long long* rep_id;
  const double* rep_t0;
  const double* rep_t1;
  const int32_t* rep_length;
  const int32_t* rep_queue;
  const uint32_t* rep_seg;
  int64_t quantisation;
  int64_t base_time;
  int32_t hours;
  uint32_t n_segments;
  uint32_t* hist;
  unsigned long long* n_rows;
};

constexpr int kTraceWaves = 4;  // K8 / K9: waves (traces) per 256-thread block
__global__ __launch_bounds__(256) void k_histogram(HistArgs a) {
  const int t = blockIdx.x * kTraceWaves + threadIdx.x / OTR_WAVE;
  if (t >= a.b.n_traces) return;  // wave-uniform
  const int64_t lo = a.b.trace_off[t], hi = a.b.trace_off[t + 1];
  if (hi <= lo) return;
  const int64_t first = a.b.time[lo], last = a.b.time[hi - 1];
  const int64_t co = a.cap_off[t], nrep = a.rep_n[t];
  unsigned long long rows = 0;
  for (int64_t r = lane_id(); r < nrep; r += OTR_WAVE) {
    const double t0 = a.rep_t0[co + r], t1 = a.rep_t1[co + r];
    const int32_t len = a.rep_length[co + r];
    if (!bucket_keep(t0, t1, len, a.rep_queue[co + r])) continue;
    const BucketSpan sp = bucket_span(t0, t1, first, last, a.quantisation);
    if (!sp.ok) continue;
    const double kmh = ((double)len / (t1 - t0)) * 3.6;
    int bin = (int)(kmh / 20.0);
    bin = bin < 0 ? 0 : (bin > OTR_HIST_BINS - 1 ? OTR_HIST_BINS - 1 : bin);
    const uint32_t seg = a.rep_seg[co + r];
    for (int64_t bk = sp.min_bucket; bk <= sp.max_bucket; ++bk) {
      ++rows;
      const int64_t h = (bk * a.quantisation - a.base_time) / a.quantisation;
      if (h >= 0 && h < a.hours && seg < a.n_segments && a.hist)
        atomicAdd(&a.hist[((size_t)h * a.n_segments + seg) * OTR_HIST_BINS + bin], 1u);
    }
  }
  for (int o = OTR_WAVE / 2; o > 0; o >>= 1) rows += __shfl_xor(rows, o);
  if (rows && lane_id() == 0) atomicAdd(&a.n_rows[cshard()], rows);
}

// ------------------------------------------------------------------------------
// K9: simple_reporter tile rows (simple_reporter.py:176-196), one thread per trace:
// pass 1 (rows == nullptr) counts each trace's rows, pass 2 writes them at row_off.
// ------------------------------------------------------------------------------
struct TileArgs {
  BatchDev b;
  const int64_t* cap_off;
  const int64_t* rep_n;
  const unsigned long long* rep_id;
  const unsigned long long* rep_next;
  const double* rep_t0;
  const double* rep_t1;
  const int32_t* rep_length;
  const int32_t* rep_queue;
  int64_t quantisation;
  int32_t rules;           // OTR_TILE_RULES_*: simple_reporter.py or the Java streaming path
  int64_t* row_cnt;        // pass 1 output
  const int64_t* row_off;  // pass 2 input (exclusive offsets)
  otr_tile_row* rows;      // pass 2 output
};

// one wave per trace, a lane per report; a report's rows are contiguous, reports in order
// (wave prefix sums place them), so the rows come out trace by trace in report order
__global__ __launch_bounds__(256) void k_tile_rows(TileArgs a) {
  const int t = blockIdx.x * kTraceWaves + threadIdx.x / OTR_WAVE;
  if (t >= a.b.n_traces) return;  // wave-uniform
  const int64_t lo = a.b.trace_off[t], hi = a.b.trace_off[t + 1];
  int64_t base = a.rows ? a.row_off[t] : 0;
  const int64_t base0 = base;
  if (hi > lo) {
    const int64_t first = a.b.time[lo], last = a.b.time[hi - 1];
    const int64_t co = a.cap_off[t], nrep = a.rep_n[t];
    for (int64_t r0 = 0; r0 < nrep; r0 += OTR_WAVE) {
      const int64_t r = r0 + lane_id();
      BucketSpan sp;
      bool keep = false;
      double t0 = 0, t1 = 0;
      int32_t len = 0, qu = 0;
      if (r < nrep) {
        t0 = a.rep_t0[co + r];
        t1 = a.rep_t1[co + r];
        len = a.rep_length[co + r];
        qu = a.rep_queue[co + r];
        if (a.rules == OTR_TILE_RULES_STREAM) {
          // BatchingProcessor.java:119-126 (Segment.valid, Segment.java:38-40) and
          // TimeQuantisedTile.getTiles (TimeQuantisedTile.java:26-35): buckets from the
          // truncated times, no span limit; duration Math.round (ties up), Segment.java:65-71
          if (t0 > 0 && t1 > 0 && t1 > t0 && len > 0 && qu >= 0) {
            sp.duration = py2_round_int(t1 - t0);
            sp.start = (int64_t)floor(t0);
            sp.end = (int64_t)ceil(t1);
            sp.min_bucket = (int64_t)t0 / a.quantisation;
            sp.max_bucket = (int64_t)t1 / a.quantisation;
            keep = true;
          }
        } else if (bucket_keep(t0, t1, len, qu)) {
          sp = bucket_span(t0, t1, first, last, a.quantisation);
          keep = sp.ok;
        }
      }
      const unsigned long long nb = keep ? (unsigned long long)(sp.max_bucket - sp.min_bucket + 1) : 0ull;
      const unsigned long long incl = wave_incl_scan_u64(nb);
      if (a.rows && keep) {
        const unsigned long long id = a.rep_id[co + r], nx = a.rep_next[co + r];
        // the report's 20 km/h speed bin, as K8 bins it (oracle/tiles.py speed_bin)
        const double bq = (((double)len / (t1 - t0)) * 3.6) / 20.0;
        const int speed_bin = bq >= (double)(OTR_HIST_BINS - 1) ? OTR_HIST_BINS - 1 : (bq < 0.0 ? 0 : (int)bq);
        int64_t k = base + (int64_t)(incl - nb);
        for (int64_t bk = sp.min_bucket; bk <= sp.max_bucket; ++bk, ++k) {
          otr_tile_row row;
          row.file = ((unsigned long long)bk << 25) | ((id & 7ull) << 22) | ((id >> 3) & 0x3FFFFFull);
          row.id = id;
          row.next_id = nx == OTR_NO_ID ? OTR_INVALID_SEGMENT_ID : nx;
          row.start = sp.start;
          row.end = sp.end;
          row.duration = (int32_t)sp.duration;
          row.length = len;
          row.queue_length = qu;
          row.speed_bin = speed_bin;
          a.rows[k] = row;
        }
      }
      base += (int64_t)__shfl(incl, OTR_WAVE - 1);
    }
  }
  if (!a.rows && lane_id() == 0) a.row_cnt[t] = base - base0;
}

// Line order of simple_reporter.py:218 (segments.sort() over whole text lines).  Every
// field before the constant tail is a non-negative decimal integer followed by ',',
// and ',' sorts below every digit, so the string order is the field-by-field
// lexicographic order of the digit strings (a proper prefix sorts first).
__host__ __device__ inline int dec_digits(unsigned long long v) {
  int n = 1;
  while (v >= 10ull) {
    v /= 10ull;
    ++n;
  }
  return n;
}
__host__ __device__ inline int dec_cmp(unsigned long long a, unsigned long long b) {
  if (a == b) return 0;
  const int na = dec_digits(a), nb = dec_digits(b);
  unsigned long long pa = a, pb = b;
  for (int k = nb; k < na; ++k) pa /= 10ull;  // leading min(na, nb) digits
  for (int k = na; k < nb; ++k) pb /= 10ull;
  if (pa != pb) return pa < pb ? -1 : 1;
  return na < nb ? -1 : 1;
}
struct TileLineLess {
  __host__ __device__ bool operator()(const otr_tile_row& x, const otr_tile_row& y) const {
    if (x.file != y.file) return x.file < y.file;  // files are independent: any fixed order
    int c = dec_cmp(x.id, y.id);
    if (!c) c = dec_cmp(x.next_id, y.next_id);
    if (!c) c = dec_cmp((unsigned long long)x.duration, (unsigned long long)y.duration);
    if (!c) c = dec_cmp((unsigned long long)x.length, (unsigned long long)y.length);
    if (!c) c = dec_cmp((unsigned long long)x.queue_length, (unsigned long long)y.queue_length);
    if (!c) c = dec_cmp((unsigned long long)x.start, (unsigned long long)y.start);
    if (!c) c = dec_cmp((unsigned long long)x.end, (unsigned long long)y.end);
    return c < 0;
  }
};

// Radix keys for the line order: a non-negative integer's decimal string, left-aligned
// in 18 base-11 digits (digit d → d + 1, padding → 0), is an integer whose numeric
// order is the string order of the decimal strings (a proper prefix sorts first).
// 11^18 < 2^63.  Fields are stable-sorted least significant first (LSD over fields).
// Digits are taken least significant first by constant divisions (multiply-high), the
// weight of the last digit being 11^(18 - n); a number of more than 18 digits keys on its
// leading 18.
__host__ __device__ inline unsigned long long dec_key(unsigned long long v) {
  int n = dec_digits(v);
  for (; n > 18; --n) v /= 10ull;
  unsigned long long m = 1, key = 0;
  for (int k = n; k < 18; ++k) m *= 11ull;
  for (int k = 0; k < n; ++k) {
    key += (v % 10ull + 1ull) * m;
    v /= 10ull;
    m *= 11ull;
  }
  return key;
}
enum TileField { TF_FILE = 0, TF_ID, TF_NEXT, TF_DURATION, TF_LENGTH, TF_QUEUE, TF_START, TF_END, TF_COUNT };
// Segment.compareTo (Segment.java:50-53): numeric (id, next_id), stable
// (Collections.sort keeps arrival order within equal keys)
__global__ void k_pair_key(const otr_tile_row* rows, const int32_t* perm, int64_t n, int field,
                           unsigned long long* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const otr_tile_row& r = rows[perm[i]];
  key[i] = field == TF_FILE ? r.file : (field == TF_ID ? r.id : r.next_id);
}
__global__ void k_line_key(const otr_tile_row* rows, const int32_t* perm, int64_t n, int field,
                           unsigned long long* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const otr_tile_row& r = rows[perm[i]];
  unsigned long long v;
  switch (field) {
    case TF_FILE: key[i] = r.file; return;
    case TF_ID: v = r.id; break;
    case TF_NEXT: v = r.next_id; break;
    case TF_DURATION: v = (unsigned long long)(uint32_t)r.duration; break;
    case TF_LENGTH: v = (unsigned long long)(uint32_t)r.length; break;
    case TF_QUEUE: v = (unsigned long long)(uint32_t)r.queue_length; break;
    case TF_START: v = (unsigned long long)r.start; break;
    default: v = (unsigned long long)r.end; break;
  }
  key[i] = dec_key(v);
}
__global__ void k_iota_i32(int32_t* v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}
__global__ void k_gather_rows(const otr_tile_row* in, const int32_t* idx, int64_t n, otr_tile_row* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}
// stream compaction by an inclusive scan of 0/1 flags: out[pos[i] - 1] = in[i]
template <class T>
__global__ void k_scatter_flagged(const T* in, const int64_t* flag, const int64_t* pos, int64_t n, T* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) out[pos[i] - 1] = in[i];
}
__global__ void k_scatter_index(const int64_t* flag, const int64_t* pos, int64_t n, int64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) out[pos[i] - 1] = i;
}

// K10: privacy cull (simple_reporter.py:221-239), one thread per file over its sorted
// rows.  Runs of equal (id, next_id) are kept iff at least `privacy` long — except that
// a trailing run of length 1 is judged together with the run before it (the loop
// reaches the last line while its range still starts at the previous run).
// Run-parallel form: rows → runs of equal (file, id, next_id) (head flags, scan,
// scatter of run starts); one thread per run decides from its own length and its
// neighbours' whether it is kept; rows inherit their run's decision.
__global__ void k_run_heads(const otr_tile_row* r, int64_t n, int64_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    head[i] = (i == 0 || r[i].file != r[i - 1].file || r[i].id != r[i - 1].id || r[i].next_id != r[i - 1].next_id)
                  ? 1 : 0;
}

__global__ void k_cull_runs(const otr_tile_row* r, int64_t n, const int64_t* run_start, int64_t n_runs,
                            int32_t privacy, uint8_t* run_keep) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_runs) return;
  auto len = [&](int64_t q) { return (q + 1 < n_runs ? run_start[q + 1] : n) - run_start[q]; };
  auto same_file = [&](int64_t p, int64_t q) { return r[run_start[p]].file == r[run_start[q]].file; };
  const bool last = k + 1 == n_runs || !same_file(k, k + 1);
  const int64_t L = len(k);
  bool keep;
  if (last) {
    // the final run of a file: a singleton after another run is judged with it
    keep = (L == 1 && k > 0 && same_file(k - 1, k)) ? len(k - 1) + 1 >= privacy : L >= privacy;
  } else {
    const bool next_last = k + 2 == n_runs || !same_file(k + 1, k + 2);
    keep = (next_last && len(k + 1) == 1) ? L + 1 >= privacy : L >= privacy;
  }
  run_keep[k] = keep ? 1 : 0;
}

// row keep flag from its run (run index = inclusive scan of run heads - 1)
__global__ void k_row_keep(const int64_t* run_pos, const uint8_t* run_keep, int64_t n, int64_t* keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keep[i] = run_keep[run_pos[i] - 1];
}

}  // namespace otr
