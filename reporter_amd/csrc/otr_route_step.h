// otr_route_step.h — K3 + K4 as one multi-root search per step (gfx950, wave64).
//
// A step's search tasks (one per distinct root node dst(e_i) of the previous state's
// candidates, k_tasks) start within a few tens of metres of each other and aim at the
// same target disk, so their per-root searches cover nearly the same nodes.  Here one
// wave runs up to RMAX of them together over ONE LDS hash table: a node's slot holds a
// label per root (the same packed (length << sh | time) words as k_route), the adjacency
// record of a settled node is loaded and its heads are hashed once for all roots, and the
// lanes of the relaxation are (edge, root) pairs.  Every root's labels are exact integer
// shortest-path lengths from that root, reached as a fixed point whatever the order, so
// the transition rows are bit-identical to the per-root kernels' (DESIGN.md §3.4, §4).
//
// Order and stopping (work only, never labels): a node is pending while some root's label
// improved since it was last settled (`dirty` bit per root, the dirty word doubles as the
// pending flag: the lane that turns it non-zero appends the node); its key is the smallest
// f = length + h among those improvements (`fkey`).  Rounds settle the pending nodes with
// f < fmin + delta.  Every later improvement of any root's label at a target T comes
// through a pending node, so L_r(T) + h(T) < fmin makes T final for root r and
// d0min_r + min(L_r(T), fmin - h(T)) + tpart > B makes it unreachable (as in
// target_resolved, with fmin the minimum over all roots — smaller, so conservative).
// A root whose targets are all resolved stops propagating (its later labels are never
// read).  A unit that outgrows the table hands its tasks to the per-root retry tiers
// (overflow flag 1), exactly as a first-tier overflow does.
#pragma once

#include "otr_kernels.h"

namespace otr {

#ifndef OTR_STEP_WCAP
#define OTR_STEP_WCAP 16
#endif

// deployed table: 128 slots x 8 roots (8.6 KB of LDS per wave); route_tier_code of the
// launch = 1,000,000 + CAP * 100 + RMAX
constexpr int kStepCap = 128;
constexpr int kStepCode = 1000000 + kStepCap * 100 + 8;

struct StepArgs {
  const int64_t* unit;      // units: state * 8 + root group (RMAX roots of the state's tasks each)
  int64_t n_units;
  const int64_t* task_off;  // per state: first task
  const int64_t* ntask;     // per state: tasks
};

template <int CAP, int RMAX>
struct StepLds {
  static constexpr int WCAP = OTR_STEP_WCAP;  // nodes settled per round (at most)
  static constexpr int ECAP = 4 * WCAP + 32;  // edges relaxed per round: adjacency slots + CSR tails
  static constexpr int RS = RMAX + 1;         // label row stride (words): rows 9 words apart spread one root over all banks
  uint32_t lab[CAP * RS];                     // [slot][root] packed label words, kNoLabel
  uint32_t key[CAP];                          // node id, kEmpty
  uint32_t dirty[CAP];                        // roots improved since the node was last settled
  uint32_t fkey[CAP];                         // smallest f = length + h of those improvements
  uint32_t dk[CAP];                           // smallest length of those improvements (bound test of the settle)
  uint4 edge[ECAP];                           // this round's edges: {head slot | tail slot << 8 | roots << 16, len mm, time, h(head)}
  uint4 work[WCAP];                           // this round's settled nodes: {node, slot | roots << 8, min length, edge offset | count << 16}
  uint32_t pair[WCAP * RMAX];                 // this round's (settled node, dirty root) pairs: root | tail slot << 3 | first edge << 11 | edges << 18
  static constexpr int PCAP = 256;            // pending-list entries (duplicates until the next partition)
  uint8_t pend[PCAP];                         // pending slots; an entry is live iff pmark[slot] names its position
  uint8_t pmark[CAP];                         // position of the slot's live pending entry
  int n_edge, overflow;
};

template <int CAP>
__device__ inline int step_insert(uint32_t* key, uint32_t node, bool* isnew) {
  uint32_t h = hslot<CAP>(node);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = atomicCAS(&key[h], kEmpty, node);
    if (k == kEmpty) {
      *isnew = true;
      return (int)h;
    }
    if (k == node) {
      *isnew = false;
      return (int)h;
    }
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  *isnew = false;
  return -1;
}

template <int CAP>
__device__ inline int step_find(const uint32_t* key, uint32_t node) {
  uint32_t h = hslot<CAP>(node);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = key[h];
    if (k == kEmpty) return -1;
    if (k == node) return (int)h;
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  return -1;
}

// inclusive prefix sum over the wave (DPP row scans + row broadcasts)
__device__ inline uint32_t wave_incl_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ inline uint32_t wave_or_u32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

#ifndef OTR_STEP_WAVES
#define OTR_STEP_WAVES 4
#endif

// One unit (a step's roots q = 0..R-1, tasks task_off[s] + 8 * grp + q) per block of one
// wave; grid = units, XCD-mapped (neighbouring units: same trace, same neighbourhood).
template <int CAP, int RMAX>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OTR_STEP_WAVES, 8))) void k_route_step(
    DevGraph gr, RouteArgs a, StepArgs sa, unsigned long long* counters) {
  static_assert(RMAX == 8, "roots index 3 bits of a pair");
  constexpr int RS = StepLds<CAP, RMAX>::RS;
  static_assert(CAP <= 256, "slots are bytes");
  __shared__ StepLds<CAP, RMAX> L;
  constexpr int WCAP = StepLds<CAP, RMAX>::WCAP;
  constexpr int ECAP = StepLds<CAP, RMAX>::ECAP;
  constexpr int PCAP = StepLds<CAP, RMAX>::PCAP;
  constexpr int kMaxKeys = (CAP * 7) / 8;
  const int64_t NU = sa.n_units;
  const int64_t u = xcd_remap(blockIdx.x, (NU + 7) / 8);
  if (u >= NU) return;
  const int lane = (int)threadIdx.x;
  const int64_t code = sa.unit[u];
  const int64_t s = code >> 3;
  const int grp = (int)(code & 7);
  const int64_t t0 = sa.task_off[s] + (int64_t)grp * RMAX;
  const int64_t nt = sa.ntask[s] - (int64_t)grp * RMAX;
  const int R = nt < RMAX ? (int)nt : RMAX;
  // ---- per root (lane q < R): its task record; step-uniform fields from root 0
  uint4 q0 = make_uint4(0u, 0u, 0u, 0u), q1 = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
  uint32_t hroot = 0xFFFFFFFFu;
  if (lane < R) {
    q0 = a.rec[3 * (t0 + lane)];
    q1 = a.rec[3 * (t0 + lane) + 1];
    hroot = a.rec[3 * (t0 + lane) + 2].x;
  }
  const uint4 r2 = a.rec[3 * t0 + 2];
  const int64_t sp = (int64_t)__builtin_amdgcn_readfirstlane((int)q0.y);
  const uint32_t bmm = (uint32_t)__builtin_amdgcn_readfirstlane((int)q0.w);
  const uint32_t meta = (uint32_t)__builtin_amdgcn_readfirstlane((int)q1.y);
  const int32_t bt = (int32_t)__builtin_amdgcn_readfirstlane((int)r2.y);
  const int64_t toff = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)r2.w) << 32) |
                                 (uint32_t)__builtin_amdgcn_readfirstlane((int)r2.z));
  const int Kb = (int)(meta & 0xFFu);
  const int md = (int)((meta >> 8) & 3u);
  const bool forced = (meta >> 10) & 1u;
  Pack K;
  K.sh = (meta >> 11) & 31u;
  const bool general = (meta >> 16) & 1u;
  const uint32_t mode_bit = 1u << md;
  const unsigned long long mask_q = ((unsigned long long)q1.w << 32) | q1.z;
  // sources of the unit (the union of its roots' masks) and each source's root index
  unsigned long long umask = 0;
  const uint32_t d0v = lane < R ? q1.x : 0xFFFFFFFFu;  // lane q: d0min of root q
#pragma unroll
  for (int q = 0; q < RMAX; ++q) {
    const unsigned long long mq = q < R ? ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)q1.w, q) << 32) |
                                              (uint32_t)__builtin_amdgcn_readlane((int)q1.z, q)
                                        : 0ull;
    umask |= mq;
  }
  uint32_t* trow = a.trans + toff;
  // overflow flag of every task of the unit (retry tiers / global search take them)
  auto hand_over = [&](int flag) {
    if (lane < R) a.overflow_flag[t0 + lane] = flag;
  };
#ifdef OTR_FORCE_RETRY
  if (!forced) {  // test build: every search takes the retry tiers
    hand_over(general ? 3 : (bmm > a.direct_bmm ? 2 : 1));
    return;
  }
#endif
  if (!forced && general) {
    hand_over(3);
    return;
  }
  if (!forced && bmm > a.direct_bmm) {  // long bounds: straight to the large-table tiers
    hand_over(2);
    return;
  }
  // source lane i (< Ka): edge, fraction, exit part (mm, time), root index
  uint32_t e_i = 0, w_i = 0, t_i = 0;
  double p_i = 0;
  int qi = 0;
  if ((umask >> lane) & 1ull) {
    e_i = a.cand_edge[sp * OTR_KMAX + lane];
    p_i = a.cand_p[sp * OTR_KMAX + lane];
    const uint4 cp = a.cprep[sp * OTR_KMAX + lane];
    w_i = cp.w;
    if (bt >= 0) t_i = a.cprep_t[sp * OTR_KMAX + lane].y;
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const unsigned long long mq = q < R ? ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)q1.w, q) << 32) |
                                                (uint32_t)__builtin_amdgcn_readlane((int)q1.z, q)
                                          : 0ull;
      if ((mq >> lane) & 1ull) qi = q;
    }
  }
  // target lane j (< Kb): edge, fraction, entry part, node src(e_j), h, and the roots
  // whose labels it needs (a source of the root that is not a same-edge forward move)
  uint32_t ej = 0, tpart = 0, tnode = kEmpty, hT = 0, tpt = 0;
  double pj = 0;
  uint32_t unres = 0;
  if (lane < Kb) {
    ej = a.cand_edge[s * OTR_KMAX + lane];
    pj = a.cand_p[s * OTR_KMAX + lane];
    const uint4 cq = a.cprep[s * OTR_KMAX + lane];
    tpart = cq.x;
    tnode = cq.y;
    hT = cq.z;
    if (bt >= 0) tpt = a.cprep_t[s * OTR_KMAX + lane].x;
  }
  for (unsigned long long m = umask; m; m &= m - 1) {  // wave-uniform
    const int i = __ffsll((long long)m) - 1;
    const uint32_t ei = (uint32_t)__shfl((int)e_i, i);
    const double pi = __shfl(p_i, i);
    const int q = __shfl(qi, i);
    if (lane < Kb && !(ej == ei && pj >= pi)) unres |= 1u << q;
  }
  if (forced) unres = 0;
  const bool search = !forced && __ballot(unres != 0u) != 0ull;
  // ---- search
  uint32_t n_settle = 0, n_edges = 0, n_lab = 0, n_rounds = 0;
  int nkeys = 0;
  int tslot = -1;
  bool ok = true;
  if (search) {
    {
      uint4* lab4 = reinterpret_cast<uint4*>(L.lab);
      const uint4 inf4 = make_uint4(kNoLabel, kNoLabel, kNoLabel, kNoLabel);
      static_assert((CAP * RS) % 4 == 0, "label rows clear as 16-B words");
      for (int k = lane; k < CAP * RS / 4; k += OTR_WAVE) lab4[k] = inf4;
      for (int k = lane; k < CAP; k += OTR_WAVE) {
        L.key[k] = kEmpty;
        L.dirty[k] = 0u;
        L.fkey[k] = 0xFFFFFFFFu;
        L.dk[k] = 0xFFFFFFFFu;
      }
      if (lane == 0) L.overflow = 0;
    }
    __syncthreads();
    // roots (distinct nodes): label 0, dirty, pending in lane order; targets pre-inserted
    bool isnew = false;
    if (lane < R) {
      const int sl = step_insert<CAP>(L.key, q0.z, &isnew);  // an empty table: always a slot
      L.lab[sl * RS + lane] = 0u;
      L.dirty[sl] = 1u << lane;
      L.fkey[sl] = hroot;
      L.dk[sl] = 0u;
      L.pend[lane] = (uint8_t)sl;
      L.pmark[sl] = (uint8_t)lane;
    }
    nkeys += __popcll(__ballot(isnew));
    __syncthreads();
    isnew = false;
    if (lane < Kb && tnode != kEmpty) tslot = step_insert<CAP>(L.key, tnode, &isnew);
    nkeys += __popcll(__ballot(isnew));
    __syncthreads();
    const uint32_t hTm = hT + a.heur[s].margin;
    const Heur H = a.heur[s];
    const uint32_t* adjt = gr.adj_t + (size_t)md * gr.adj_t_stride;
    const uint32_t delta_mm = a.delta * 1000.0 >= 1.0 ? (uint32_t)(a.delta * 1000.0) : 1u;  // > 0: every round settles
    uint32_t fmin = wave_min_u32(hroot);
    int npend = R;
    for (;;) {
      // targets: resolve (root, target) pairs, one pass per root some target still needs
      const uint32_t live = wave_or_u32(unres);
      for (uint32_t mq = live; mq; mq &= mq - 1) {  // wave-uniform
        const int q = __ffs(mq) - 1;
        const uint32_t d0q = (uint32_t)__builtin_amdgcn_readlane((int)d0v, q);
        if ((unres >> q) & 1u) {
          const uint32_t lw = L.lab[tslot * RS + q];
          // lengths < 2^31 (<= the bound), h < 2^31: 32-bit sums cannot wrap
          bool res = npend == 0 || (lw != kNoLabel && K.d(lw) + hTm < fmin);
          if (!res) {
            const int64_t rest = (int64_t)fmin - (int64_t)hTm;
            const int64_t lab = lw == kNoLabel ? rest : ((int64_t)K.d(lw) < rest ? (int64_t)K.d(lw) : rest);
            res = (int64_t)d0q + lab + (int64_t)tpart > (int64_t)bmm;
          }
          if (res) unres &= ~(1u << q);
        }
      }
      if (__ballot(unres != 0u) == 0ull || npend == 0) break;
      ++n_rounds;
      const uint32_t theta = fmin + delta_mm < fmin ? 0xFFFFFFFFu : fmin + delta_mm;
      uint32_t fnext = 0xFFFFFFFFu;
      // partition the pending list: settle (f < theta), drop (only finished roots dirty),
      // keep the rest in place; a settled node's dirty live roots become (node, root) pairs
      int kept = 0, nw = 0, np = 0;
      for (int base = 0; base < npend; base += OTR_WAVE) {
        const int k = base + lane;
        const bool in = k < npend;
        int sl = 0;
        uint32_t f = 0, m = 0;
        bool live_e = false;
        if (in) {
          sl = L.pend[k];
          live_e = L.pmark[sl] == (uint8_t)k;  // a later push of the same slot superseded this entry
          f = L.fkey[sl];
          m = L.dirty[sl] & live;
        }
        const uint32_t dmin = in ? L.dk[sl] : 0u;
        const bool drop = in && live_e && m == 0u;
        bool take = in && live_e && !drop && f < theta;
        take = take && nw + prefix_count(__ballot(take)) < WCAP;
        const unsigned long long mt = __ballot(take), mk = __ballot(live_e && !take && !drop);
        const uint32_t c = take ? (uint32_t)__popc(m) : 0u;
        const uint32_t cin = wave_incl_scan_u32(c);
        const uint32_t ctot = (uint32_t)__builtin_amdgcn_readlane((int)cin, 63);
        if (take) L.work[nw + prefix_count(mt)] = make_uint4(L.key[sl], (uint32_t)sl | (m << 8), dmin, np + cin - c);
        if (take || drop) {
          L.dirty[sl] = 0u;
          L.fkey[sl] = 0xFFFFFFFFu;
          L.dk[sl] = 0xFFFFFFFFu;
        } else if (live_e) {
          const int p = kept + prefix_count(mk);
          L.pend[p] = (uint8_t)sl;
          L.pmark[sl] = (uint8_t)p;
          fnext = f < fnext ? f : fnext;
        }
        nw += __popcll(mt);
        kept += __popcll(mk);
        np += (int)ctot;
        __syncthreads();
      }
      npend = kept;
      n_settle += (uint32_t)nw;
      // phase A: lane = (settled node, adjacency slot): load, bound, hash the head once;
      // a node's edges land contiguously, its range goes to work[].w
      int ne = 0;
      bool tail = false;
      for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
        const int k = base + lane;
        bool valid = false, nn = false;
        uint4 e = make_uint4(0u, 0u, 0u, 0u);
        uint4 wk = make_uint4(0u, 0u, 0u, 0u);
        if (k < 4 * nw) {
          wk = L.work[k >> 2];
          const int slot = k & 3;
          const uint32_t tq = adjt[4 * (size_t)wk.x + slot];
          const uint4 r = ld16(gr.adj + 4 * (size_t)wk.x + slot);
          tail = tail || (slot == 3 && (r.x & kAdjMore));
          if ((((r.x >> 28) & 7u) & mode_bit) && wk.z + r.y <= bmm) {
            const int sv = step_insert<CAP>(L.key, r.x & kAdjDstMask, &nn);
            if (sv < 0) {
              L.overflow = 1;
            } else {
              valid = true;
              e = make_uint4((uint32_t)sv | ((wk.y & 0xFFu) << 8) | ((wk.y >> 8) << 16), r.y, tq, H((int32_t)r.z, (int32_t)r.w));
            }
          }
        }
        nkeys += __popcll(__ballot(nn));
        const unsigned long long mv = __ballot(valid);
        const int pv = prefix_count(mv);
        if (valid && ne + pv < ECAP) L.edge[ne + pv] = e;
        if (k < 4 * nw && (k & 3) == 0) {  // the node's (root, edge range) pairs for phase B
          const uint32_t ed = ((uint32_t)(ne + pv) << 11) | ((uint32_t)__popcll((mv >> lane) & 0xFull) << 18) |
                              ((wk.y & 0xFFu) << 3);
          uint32_t pp = wk.w;
          for (uint32_t mm = wk.y >> 8; mm; mm &= mm - 1) L.pair[pp++] = ed | (uint32_t)(__ffs(mm) - 1);
        }
        ne += __popcll(mv);
      }
      const int ne_main = ne;
      if (__ballot(tail) != 0ull) {
        // rare: nodes with more than 4 out-edges walk their CSR tails (appends by counter)
        if (lane == 0) L.n_edge = ne;
        __syncthreads();
        for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
          const int k = base + lane;
          if (k < 4 * nw && (k & 3) == 3) {
            const uint4 wk = L.work[k >> 2];
            if (gr.adj[4 * (size_t)wk.x + 3].x & kAdjMore)
              for (uint32_t ee = gr.node_row[wk.x] + 4; ee < gr.node_row[wk.x + 1]; ++ee) {
                const uint4 pk = ld16(gr.edge_pack + ee);
                if (!((pk.z & 7u) & mode_bit) || wk.z + pk.y > bmm) continue;
                const int2 vll = gr.node_ll[pk.x];
                const uint32_t tq = gr.et(md)[ee];
                bool nn;
                const int sv = step_insert<CAP>(L.key, pk.x, &nn);
                if (nn) atomicAdd(&L.overflow, 2);  // new-key count rides on the overflow word (bit 0 kept)
                if (sv < 0) {
                  atomicOr(&L.overflow, 1);
                  continue;
                }
                const int p = atomicAdd(&L.n_edge, 1);
                if (p < ECAP)
                  L.edge[p] = make_uint4((uint32_t)sv | ((wk.y & 0xFFu) << 8) | ((wk.y >> 8) << 16), pk.y, tq,
                                         H(vll.x, vll.y));
              }
          }
        }
        __syncthreads();
        ne = L.n_edge;
        const int ov = L.overflow;
        nkeys += ov >> 1;
        __syncthreads();
        if (lane == 0) L.overflow = ov & 1;
      }
      if (ne > ECAP) {
        ok = false;
        break;
      }
      n_edges += (uint32_t)ne;
      __syncthreads();
      // one relaxation of root q's label over edge e (head slot e.x & 0xFF) from word pu
      auto relax = [&](const uint4& e, uint32_t pu, int q) -> int {
        ++n_lab;
        const uint32_t nd = K.d(pu) + e.y;
        if (nd > bmm) return -1;
        const uint32_t tt = K.t(pu) + e.z;
        const uint32_t nwd = (nd << K.sh) | (tt < K.tcap() ? tt : K.tcap());
        const uint32_t sv = e.x & 0xFFu;
        const uint32_t old = atomicMin(&L.lab[sv * RS + q], nwd);
        if (nwd >= old) return -1;
        const uint32_t f = nd + e.w;
        fnext = f < fnext ? f : fnext;
        atomicMin(&L.fkey[sv], f);      // no return value waited on:
        atomicMin(&L.dk[sv], nd);
        atomicOr(&L.dirty[sv], 1u << q);  // every improvement appends a fresh entry
        return (int)sv;
      };
      auto append = [&](int push) {
        const unsigned long long mp = __ballot(push >= 0);
        if (push >= 0) {
          const int p = npend + prefix_count(mp);
          if (p < PCAP) {
            L.pend[p] = (uint8_t)push;
            L.pmark[push] = (uint8_t)p;
          } else {
            L.overflow = 1;
          }
        }
        npend += __popcll(mp);
      };
      // phase B: lane = (settled node, dirty root, adjacency edge): the root's label over the edge
      for (int base = 0; base < 4 * np; base += OTR_WAVE) {
        const int idx = base + lane;
        int push = -1;
        if (idx < 4 * np) {
          const uint32_t pr = L.pair[idx >> 2];
          const int q = (int)(pr & 7u);
          const uint32_t d = (uint32_t)(idx & 3);
          if (d < (pr >> 18)) push = relax(L.edge[((pr >> 11) & 0x7Fu) + d], L.lab[((pr >> 3) & 0xFFu) * RS + q], q);
        }
        append(push);
      }
      // CSR tails: lane = (tail edge, root), the root mask carried by the edge
      const int ntl = (ne - ne_main) * RMAX;
      for (int base = 0; base < ntl; base += OTR_WAVE) {
        const int idx = base + lane;
        const int k = ne_main + (idx >> 3), q = idx & 7;
        int push = -1;
        if (idx < ntl) {
          const uint4 e = L.edge[k];
          if ((e.x >> (16 + q)) & 1u) push = relax(e, L.lab[((e.x >> 8) & 0xFFu) * RS + q], q);
        }
        append(push);
      }
      __syncthreads();
      fmin = wave_min_u32(fnext);
      if (L.overflow || nkeys > kMaxKeys || npend > PCAP) {
        ok = false;
        break;
      }
    }
    if (ok && tslot < 0 && lane < Kb && tnode != kEmpty) ok = false;  // (never: the table had room)
    ok = __ballot(!ok) == 0ull;
  }
  if (!ok) {
    hand_over(1);
  } else {
    // ---- transition rows: lane j = target, one pass per source of the unit
    for (unsigned long long m = umask; m; m &= m - 1) {  // wave-uniform
      const int i = __ffsll((long long)m) - 1;
      const uint32_t ei = (uint32_t)__shfl((int)e_i, i);
      const double pi = __shfl(p_i, i);
      const uint32_t wi = (uint32_t)__shfl((int)w_i, i);
      const uint32_t ti = (uint32_t)__shfl((int)t_i, i);
      const int q = __shfl(qi, i);
      if (lane < Kb) {
        int64_t r = -1, rt = 0;
        if (forced) {
          r = -1;
        } else if (ej == ei && pj >= pi) {
          r = part_mm(pj - pi, gr.len_mm[ei]);
          if (bt >= 0) rt = part_mm(pj - pi, gr.et(md)[ei]);
        } else if (tslot >= 0) {
          const uint32_t lw = L.lab[tslot * RS + q];
          if (lw != kNoLabel) {
            r = (int64_t)wi + K.d(lw) + tpart;
            if (bt >= 0) rt = (int64_t)ti + K.t(lw) + tpt;
          }
        }
        const bool valid = r >= 0 && r <= (int64_t)bmm && (bt < 0 || rt <= (int64_t)bt);
        trow[(int64_t)i * Kb + lane] = valid ? (uint32_t)r : kNoRoute;
      }
    }
  }
  if (counters) {
    const uint32_t ntr = ok ? (uint32_t)Kb * (uint32_t)__popcll(umask) : 0u;
    const uint32_t lab_sum = wave_sum_u32(n_lab);
    if (lane == 0) {
      const int sh = cshard();
      atomicAdd(&counters[3 * kCShards + sh], (unsigned long long)n_settle);
      atomicAdd(&counters[4 * kCShards + sh], (unsigned long long)n_edges);
      atomicAdd(&counters[5 * kCShards + sh], (unsigned long long)ntr);
      atomicAdd(&counters[6 * kCShards + sh], (unsigned long long)((search && ok) ? 1 : 0));
      atomicAdd(&counters[13 * kCShards + sh], (unsigned long long)n_rounds);
      atomicAdd(&counters[14 * kCShards + sh], (unsigned long long)(search ? nkeys : 0));
      atomicAdd(&counters[15 * kCShards + sh], (unsigned long long)lab_sum);
    }
  }
}

// one unit per (state with tasks, group of RMAX of its tasks): entries state * 8 + group
__global__ void k_step_units(int64_t n_states, const int64_t* ntask, const int64_t* unit_off, int rmax,
                             int64_t* unit) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_states) return;
  const int64_t nt = ntask[s];
  const int64_t o = unit_off[s];
  for (int64_t g = 0; g * rmax < nt; ++g) unit[o + g] = s * 8 + g;
}

__global__ void k_step_nunit(int64_t n_states, const int64_t* ntask, int rmax, int64_t* nunit) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_states) return;
  nunit[s] = (ntask[s] + rmax - 1) / rmax;
}

}  // namespace otr
