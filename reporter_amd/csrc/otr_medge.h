// otr_medge.h — K3m: the multi-source edge-state route search, the first tier of the
// turn-cost modes (the deployed configuration: a Batch.java request carries only its mode,
// and every mode's default turn_penalty_factor is > 0, Batch.java:56-65).
//
// The edge-state search of otr_edge.h runs one source candidate per wave.  Its table is
// sized for the wide spread of single searches (162 keys on average, 380 at the 98th
// percentile at C2) and each of its ~13 exact rounds is one partition pass and one relax
// pass over a few dozen lanes, so the wave's instruction stream — not the lanes — is the
// cost.  Here one wave runs the searches of up to S source candidates of ONE step
// together, over one hash table of edge states:
//   * a state (edge) is inserted once for all sources (the sources lie within twice the
//     search radius of each other, so their regions overlap: 4 sources' searches touch 250
//     distinct states against 608 apart, tools/edge_stats.py);
//   * labels are per (state, source) pair, lab[slot * S + source]; the pending list, the
//     settled list and the IN criterion work on pairs; every source keeps its own smallest
//     pending key / length (kmin, dmin), bounds (pd, pt) and targets, and stops when its
//     targets resolve, exactly as the single-source search does;
//   * one round serves every source: the partition, relax and reductions of a round are
//     shared, and relax lanes = (settled pair, adjacency slot) fill the wave;
//   * the adjacency of a state is ONE 16-B per-mode record (DevGraph::erec: head, length,
//     edge id, route time, begin and end headings), not four loads.
// The IN criterion adds the mode's smallest turn cost: every later offer to state b for
// source i comes from a pending or later state of i at src(b) (key >= kmin_i) through a
// turn (>= tmin, the table's minimum) and b itself (>= len(b)), so lab_i(b) < kmin_i +
// len(b) + tmin is final (likewise a target: tlab < kmin_i + tpart + tmin).  Only final
// labels are relaxed, so every label equals the oracle's label-setting one whatever the
// grouping (oracle.c search).  A group whose union outgrows the table (or a step with more
// than 32 targets) flags its tasks 5: they run in the single-source tiers (otr_edge.h).
#pragma once
#include "otr_edge.h"
#include <type_traits>

namespace otr {

#ifndef OTR_MS
#define OTR_MS 4  // sources per multi-source search
#endif
#ifndef OTR_MCAP
#define OTR_MCAP 448  // edge states per multi-source table
#endif
#ifndef OTR_MPCAP
#define OTR_MPCAP 640  // pending (state, source) pairs per table
#endif
#ifndef OTR_MWCAP
#define OTR_MWCAP 96  // pairs settled per round
#endif

// the per-mode edge-state adjacency record, one per (node, slot) like DevGraph::adj:
// {dst | access << 28 | more << 31, len_mm, edge | end heading bits 0-3 << 28,
//  route time (0.1 s, saturated at 2^17 - 1) | begin heading << 17 | end heading bits 4-8 << 26}
__host__ __device__ inline uint4 erec_make(uint32_t dw, uint32_t len, uint32_t e, uint32_t t, uint32_t hb,
                                           uint32_t he) {
  return make_uint4(dw, len, (e & kAdjDstMask) | ((he & 15u) << 28),
                    (t < 0x1FFFFu ? t : 0x1FFFFu) | ((hb & 0x1FFu) << 17) | ((he >> 4) << 26));
}
__device__ inline uint32_t er_edge(const uint4& r) { return r.z & kAdjDstMask; }
__device__ inline uint32_t er_he(const uint4& r) { return (r.z >> 28) | ((r.w >> 26) << 4); }
__device__ inline uint32_t er_hb(const uint4& r) { return (r.w >> 17) & 0x1FFu; }
__device__ inline uint32_t er_t(const uint4& r) { return r.w & 0x1FFFFu; }

template <int CAP, int S>
struct MEdgeLds {
  static constexpr int TG = 32;                       // targets (steps with more go to otr_edge.h)
  static constexpr int PCAP = OTR_MPCAP;             // pending pairs (more: the group fails)
  static constexpr int WCAP = OTR_MWCAP;             // pairs settled per round (the rest wait)
  unsigned long long lab[CAP * S];  // [slot][source] gpack labels, kGInf: none
  uint32_t key[CAP];                // edge id, kEmpty
  uint32_t node[CAP];               // dst(edge): where the state stands
  uint16_t hback[CAP];              // the edge's end heading reversed: the turn out of the state
  uint8_t mi[CAP];                  // mi8_of(len(edge)): the IN gap of the state
  uint32_t pm[(CAP * S + 31) / 32]; // pair bit: on the pending list (or settled)
  uint16_t pend[PCAP];              // pending pairs, slot * S + source
  uint16_t wpair[WCAP];             // this round's settled pairs
  unsigned long long wlab[WCAP];    //   and their labels
  uint4 src[S];                     // per source {pd, pt, kmin, dmin}
  uint32_t kn[S], dn[S];            // the next round's kmin / dmin (LDS atomicMin)
  uint32_t need[S];                 // per source: target lanes it must resolve
  unsigned long long tlab[S * TG];  // [source][target] the best feasible offer
  uint32_t tpart[TG], tpt[TG];      // target entry parts (mm, 0.1 s)
  uint16_t thb[TG];                 // begin heading of the target edge
  uint32_t tmap_node[TG], tmap_mask[TG];  // target node src(ej) -> target lanes
  int32_t turn[181];
  int turn_md;
  uint32_t tmin;
  int n_pend, n_keys, overflow;
};

template <int CAP, int S>
__device__ inline int m_insert(MEdgeLds<CAP, S>& L, uint32_t e, bool* isnew) {
  uint32_t h = hslot<CAP>(e);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = atomicCAS(&L.key[h], kEmpty, e);
    if (k == kEmpty) {
      *isnew = true;
      return (int)h;
    }
    if (k == e) {
      *isnew = false;
      return (int)h;
    }
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  L.overflow = 1;
  *isnew = false;
  return -1;
}

template <int CAP, int S>
__device__ inline uint32_t m_tmap_get(const MEdgeLds<CAP, S>& L, uint32_t v) {
  constexpr int TG = MEdgeLds<CAP, S>::TG;
  uint32_t h = tmap_home<TG>(v);
  for (int probe = 0; probe < TG; ++probe) {
    const uint32_t k = L.tmap_node[h];
    if (k == kEmpty) return 0u;
    if (k == v) return L.tmap_mask[h];
    h = (h + 1) & (TG - 1);
  }
  return 0u;
}

// A new state: its node, heading and IN gap, and no label for any source yet (the
// inserting lane writes these before any lane's atomicMin on the slot: one wave, LDS
// operations in program order).
template <int CAP, int S>
__device__ inline void m_new_state(MEdgeLds<CAP, S>& L, int sl, uint32_t w, uint32_t he, uint32_t len) {
  L.node[sl] = w;
  L.hback[sl] = (uint16_t)heading_back((int)he);
  L.mi[sl] = mi8_of(len);
#pragma unroll
  for (int j = 0; j < S; ++j) L.lab[sl * S + j] = kGInf;
}

// Relax the final pair (label lb, source i) through edge b (head w, length len, time tt,
// begin / end headings hb / hend; access in dw's high bits); hb_: the state's reversed end heading.
// Returns the pair id when the pair (b, i) became newly pending.
template <int CAP, int S>
__device__ inline int m_relax(MEdgeLds<CAP, S>& L, unsigned long long lb, int i, uint32_t hb_, uint32_t dw,
                              uint32_t len, uint32_t tt, uint32_t b, uint32_t hb, uint32_t hend, uint32_t pd,
                              uint32_t pt, uint32_t mode_bit, uint32_t& relaxed, bool& isnew) {
  isnew = false;
  if (!(((dw >> 28) & 7u) & mode_bit)) return -1;
  ++relaxed;
  const uint32_t tc = (uint32_t)L.turn[turn_from_back((int)hb_, (int)hb)];
  const EOffer o = e_step(lb, tc, len, tt);
  if (!e_feasible(o, pd, pt)) return -1;  // pruned (label-setting semantics)
  const int sl = m_insert(L, b, &isnew);
  if (sl < 0) return -1;
  if (isnew) m_new_state(L, sl, dw & kAdjDstMask, hend, len);
  const int pid = sl * S + i;
  const unsigned long long nw = gpack(o.k, o.c, o.t);
  const unsigned long long old = atomicMin(&L.lab[pid], nw);
  if (nw < old) {
    atomicMin(&L.kn[i], o.k);
    atomicMin(&L.dn[i], o.d);
    const uint32_t bit = 1u << (pid & 31);
    if (!(atomicOr(&L.pm[pid >> 5], bit) & bit)) return pid;
  }
  return -1;
}

// the final pair's offers to the targets at its node v (the turn into ej + the entry
// part), each target keeping the lexicographic minimum per source
template <int CAP, int S>
__device__ inline void m_target_offers(MEdgeLds<CAP, S>& L, unsigned long long lb, int i, uint32_t hb_, uint32_t v,
                                       uint32_t pd, uint32_t pt) {
  constexpr int TG = MEdgeLds<CAP, S>::TG;
  uint32_t m = m_tmap_get(L, v);
  while (m) {
    const int q = __ffs((int)m) - 1;
    m &= m - 1;
    const uint32_t tc = (uint32_t)L.turn[turn_from_back((int)hb_, (int)L.thb[q])];
    const EOffer o = e_step(lb, tc, L.tpart[q], L.tpt[q]);
    if (e_feasible(o, pd, pt)) atomicMin(&L.tlab[i * TG + q], gpack(o.k, o.c, o.t));
  }
}

// the mode's turn table into LDS (when the group's mode differs from the last one's) and
// its smallest entry (the IN criterion's turn margin)
template <int CAP, int S>
__device__ inline void m_turn_table(MEdgeLds<CAP, S>& L, const int32_t* turn_tab, int md) {
  if (L.turn_md != md) {  // (uniform)
    __syncthreads();
    uint32_t m = 0xFFFFFFFFu;
    for (int k = threadIdx.x; k < 181; k += OTR_WAVE) {
      const int32_t t = turn_tab[181 * md + k];
      L.turn[k] = t;
      m = (uint32_t)t < m ? (uint32_t)t : m;
    }
    m = wave_min_u32(m);
    if (threadIdx.x == 0) {
      L.turn_md = md;
      L.tmin = m;
    }
  }
  __syncthreads();
}

// group record: first task | task count << 56 (the tasks of one step, in candidate order)
constexpr uint64_t kGroupTaskMask = (1ull << 56) - 1ull;

// ------------------------------------------------------------------------------
// K3m kernel: a persistent grid over the device-side group list (k_mgroups), the 8 XCDs
// taking contiguous eighths of it (neighbouring groups = consecutive steps of a trace).
// force_fail (test build only): every group fails, its tasks go to the single-source tiers.
// ------------------------------------------------------------------------------
template <int CAP, int S>
__global__ __launch_bounds__(64) void k_route_medge(DevGraph gr, RouteArgs a, const uint64_t* groups,
                                                    const unsigned long long* n_groups,
                                                    unsigned long long* counters) {
  using LT = MEdgeLds<CAP, S>;
  constexpr int TG = LT::TG;
  constexpr int kMaxKeys = (CAP * 7) / 8;
  constexpr int PCAP = LT::PCAP;
  constexpr int WCAP = LT::WCAP;
  static_assert((S & (S - 1)) == 0 && S <= 32, "S: a power of two");
  static_assert(CAP * S <= 65536, "pair ids fit 16 bits");
  __shared__ LT L;
  if (threadIdx.x == 0) L.turn_md = -1;
  const int64_t n = (int64_t)*n_groups;
  const int lane = (int)threadIdx.x;
  const int64_t per = (n + 7) / 8;
  const int64_t lo = (int64_t)(blockIdx.x & 7) * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  const int64_t stride = (int64_t)(gridDim.x >> 3);
  for (int64_t w = lo + (int64_t)(blockIdx.x >> 3); w < hi; w += stride) {
    const uint64_t gw = groups[w];
    const int64_t t0 = (int64_t)(gw & kGroupTaskMask);
    const int ns = (int)(gw >> 56);
    // ---- the step (every task of the group shares it) and my source (lane < ns)
    const uint4 r0 = a.rec[3 * t0], r1 = a.rec[3 * t0 + 1], r2 = a.rec[3 * t0 + 2];
    const int64_t s = r0.x, sp = r0.y;
    const int Kb = (int)(r1.y & 0xFFu);
    const int md = (int)((r1.y >> 8) & 3u);
    const bool forced = (r1.y >> 10) & 1u;
    const uint32_t bmm = r0.w;
    const int32_t bt = (int32_t)r2.y;
    const bool timed = bt >= 0;
    int ci = 0;
    uint32_t ei = 0, d0 = 0, ts0 = 0;
    double pi = 0;
    if (lane < ns) {
      const uint4 q1 = a.rec[3 * (t0 + lane) + 1];
      const unsigned long long mk = ((unsigned long long)q1.w << 32) | q1.z;
      ci = __ffsll((long long)mk) - 1;
      ei = a.cand_edge[sp * OTR_KMAX + ci];
      pi = a.cand_p[sp * OTR_KMAX + ci];
      d0 = a.cprep[sp * OTR_KMAX + ci].w;
      ts0 = timed ? a.cprep_t[sp * OTR_KMAX + ci].y : 0u;
    }
    // ---- targets (lane < Kb)
    uint32_t ej = 0, tv = kEmpty, tpart = 0, tpt = 0;
    double pj = 0;
    if (lane < Kb && Kb <= TG) {
      ej = a.cand_edge[s * OTR_KMAX + lane];
      pj = a.cand_p[s * OTR_KMAX + lane];
      const uint4 cq = a.cprep[s * OTR_KMAX + lane];
      tpart = cq.x;
      tv = cq.y;
      tpt = timed ? a.cprep_t[s * OTR_KMAX + lane].x : 0u;
    }
    // ---- table reset (keys and pending bits; labels are set when a state is inserted)
    for (int k = lane; k < CAP; k += OTR_WAVE) L.key[k] = kEmpty;
    for (int k = lane; k < (CAP * S + 31) / 32; k += OTR_WAVE) L.pm[k] = 0u;
    for (int k = lane; k < S * TG; k += OTR_WAVE) L.tlab[k] = kGInf;
    if (lane < TG) {
      L.tmap_node[lane] = kEmpty;
      L.tmap_mask[lane] = 0u;
    }
    if (lane == 0) {
      L.n_keys = 0;
      L.overflow = 0;
    }
    m_turn_table(L, a.turn, md);
    // ---- which sources search: the targets each must resolve (not the same-edge forward
    // ones), a feasible root, no forced break, at most TG targets
    uint32_t smask = 0;  // (uniform) sources that search
    uint32_t my_need = 0;
    for (int i = 0; i < ns; ++i) {
      const uint32_t e_i = (uint32_t)__shfl((int)ei, i);
      const double p_i = __shfl(pi, i);
      const unsigned long long nb = __ballot(lane < Kb && !(ej == e_i && pj >= p_i));
      if (lane == i) my_need = (uint32_t)nb;
      const uint32_t d0i = (uint32_t)__shfl((int)d0, i), t0i = (uint32_t)__shfl((int)ts0, i);
      const bool root_ok = d0i <= bmm && (!timed || t0i <= (uint32_t)bt);
      if (!forced && Kb <= TG && root_ok && nb != 0ull) smask |= 1u << i;
    }
#ifdef OTR_FORCE_RETRY
    if (a.force_edge & 1) smask = 0xFFFFFFFFu;  // test build: every group fails below
#endif
    if (lane < S) {
      const uint32_t pd = lane < ns && bmm >= d0 ? bmm - d0 : 0u;
      const uint32_t pt = !timed ? 0xFFFFFFFFu : (lane < ns && ts0 <= (uint32_t)bt ? (uint32_t)bt - ts0 : 0u);
      L.src[lane] = make_uint4(pd, pt, 0u, 0u);
      L.need[lane] = lane < ns ? my_need : 0u;
      L.kn[lane] = 0xFFFFFFFFu;
      L.dn[lane] = 0xFFFFFFFFu;
    }
    __syncthreads();
    const bool tgt = lane < Kb && Kb <= TG && tv != kEmpty;
    if (tgt) {
      L.tpart[lane] = tpart;
      L.tpt[lane] = tpt;
      L.thb[lane] = (uint16_t)gr.edge_head[ej].x;
      uint32_t h = tmap_home<TG>(tv);
      for (int probe = 0; probe < TG; ++probe) {
        const uint32_t k = atomicCAS(&L.tmap_node[h], kEmpty, tv);
        if (k == kEmpty || k == tv) {
          atomicOr(&L.tmap_mask[h], 1u << lane);
          break;
        }
        h = (h + 1) & (TG - 1);
      }
    }
    // ---- roots: source i's state ei with label 0
    const bool root = lane < ns && ((smask >> lane) & 1u) && smask != 0xFFFFFFFFu;
    int rsl = -1;
    bool rnew = false;
    if (root) {
      rsl = m_insert(L, ei, &rnew);
      if (rsl >= 0) {
        if (rnew) m_new_state(L, rsl, gr.edge_dst[ei], (uint32_t)(uint16_t)gr.edge_head[ei].y, gr.len_mm[ei]);
        const int pid = rsl * S + lane;
        L.lab[pid] = gpack(0u, 0u, 0u);
        atomicOr(&L.pm[pid >> 5], 1u << (pid & 31));
      }
    }
    __syncthreads();
    const unsigned long long mr = __ballot(root && rsl >= 0);
    if (root && rsl >= 0) L.pend[prefix_count(mr)] = (uint16_t)(rsl * S + lane);
    int npend = __popcll(mr);
    int nkeys = __popcll(__ballot(rnew));
    __syncthreads();
    uint32_t active = smask == 0xFFFFFFFFu ? 0u : smask;  // (uniform) sources still searching
    const uint32_t mode_bit = 1u << md;
    const uint4* er = gr.erec + (size_t)md * gr.erec_stride;
    const uint32_t* et = gr.et(md);
    const uint32_t tmin = L.tmin;
    uint32_t my_settled = 0, my_relaxed = 0;
    bool fail = smask == 0xFFFFFFFFu;
    while (active != 0u && !fail) {
      // ---- target resolution (lane = (source, target), 64 / TG sources per pass): source i is
      // done once every target it needs is final (tlab < kmin_i + tpart + tmin) or
      // unreachable (dmin_i + tpart > pd_i), or it has nothing pending (kmin_i = none)
      {
        constexpr int SP = OTR_WAVE / TG;  // sources per pass
        const int q = lane & (TG - 1);
        const uint32_t tp = (uint32_t)__shfl((int)tpart, q);
        uint32_t unres = 0;
#pragma unroll
        for (int i0 = 0; i0 < S; i0 += SP) {
          const int i = i0 + lane / TG;
          bool res = true;
          if (i < S && ((active >> i) & 1u)) {
            const uint4 sv = L.src[i];
            if (sv.z == 0xFFFFFFFFu) res = false;  // (reported below as done)
            else if ((L.need[i] >> q) & 1u) {
              const unsigned long long tl = L.tlab[i * TG + q];
              res = (tl != kGInf && (uint64_t)g_k(tl) < (uint64_t)sv.z + tp + tmin) ||
                    (uint64_t)sv.w + tp > (uint64_t)sv.x;
            }
          }
          const unsigned long long mb = __ballot(!res);
#pragma unroll
          for (int j = 0; j < SP; ++j)
            if (i0 + j < S && ((mb >> (j * TG)) & ((TG == 64 ? 0ull : (1ull << TG)) - 1ull)) != 0ull) unres |= 1u << (i0 + j);
        }
        // sources with a pending pair and an open target go on; kmin = none means no pending pair
        uint32_t nopend = 0;
        if (lane < S && ((active >> lane) & 1u) && L.src[lane].z == 0xFFFFFFFFu) nopend = 1u;
        const uint32_t np_mask = (uint32_t)__ballot(nopend != 0u);
        active &= unres & ~np_mask;
      }
      if (active == 0u) break;
      // ---- partition the pending pairs: final (IN criterion) → settled list; pairs of a
      // finished source are dropped; the rest stay, giving the next kmin / dmin
      int kept = 0, nw = 0;
      for (int base = 0; base < npend; base += OTR_WAVE) {
        const int k = base + lane;
        const bool in = k < npend;
        int pid = 0, i = 0;
        unsigned long long lb = 0;
        bool take = false, keep = false;
        if (in) {
          pid = L.pend[k];
          i = pid & (S - 1);
          if ((active >> i) & 1u) {
            lb = L.lab[pid];
            const uint32_t kk = g_k(lb);
            take = (uint64_t)kk < (uint64_t)L.src[i].z + in_gap8(L.mi[pid / S]) + tmin;
            keep = !take;
          }
        }
        const bool tk = take && nw + prefix_count(__ballot(take)) < WCAP;
        keep = keep || (take && !tk);
        const unsigned long long mt = __ballot(tk), mk = __ballot(keep);
        __syncthreads();
        if (tk) {
          const int wq = nw + prefix_count(mt);
          L.wpair[wq] = (uint16_t)pid;
          L.wlab[wq] = lb;
        } else if (keep) {
          L.pend[kept + prefix_count(mk)] = (uint16_t)pid;
          atomicMin(&L.kn[i], g_k(lb));
          atomicMin(&L.dn[i], g_d(lb));
        }
        nw += __popcll(mt);
        kept += __popcll(mk);
        __syncthreads();
      }
      npend = kept;
      // ---- relax: lane = (settled pair, adjacency slot); slot-0 lanes make the pair's
      // target offers; slot 3 of a node with more than 4 out-edges walks the CSR tail
      bool tail = false;
      for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
        const int k = base + lane;
        int ppid = -1;
        bool isnew = false;
        if (k < 4 * nw) {
          const int pid = L.wpair[k >> 2];
          const unsigned long long lb = L.wlab[k >> 2];
          const int sl = pid / S, i = pid & (S - 1);
          const uint32_t v = L.node[sl], ha = L.hback[sl];
          const uint4 sv = L.src[i];
          const int slot = k & 3;
          const uint4 r = ld16(er + 4 * (size_t)v + slot);
          if (slot == 0) {
            ++my_settled;
            m_target_offers(L, lb, i, ha, v, sv.x, sv.y);
          }
          ppid = m_relax(L, lb, i, ha, r.x & ~kAdjMore, r.y, timed ? er_t(r) : 0u, er_edge(r), er_hb(r), er_he(r),
                           sv.x, sv.y, mode_bit, my_relaxed, isnew);
          tail = tail || (slot == 3 && (r.x & kAdjMore));
        }
        nkeys += __popcll(__ballot(isnew));
        const unsigned long long mp = __ballot(ppid >= 0);
        if (ppid >= 0) {
          const int p = npend + prefix_count(mp);
          if (p < PCAP) L.pend[p] = (uint16_t)ppid;
          else L.overflow = 1;
        }
        npend += __popcll(mp);
      }
      if (__ballot(tail) != 0ull) {
        if (lane == 0) {
          L.n_pend = npend;
          L.n_keys = 0;
        }
        __syncthreads();
        for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
          const int k = base + lane;
          if (k < 4 * nw && (k & 3) == 3) {
            const int pid = L.wpair[k >> 2];
            const unsigned long long lb = L.wlab[k >> 2];
            const int sl = pid / S, i = pid & (S - 1);
            const uint32_t v = L.node[sl], ha = L.hback[sl];
            const uint4 sv = L.src[i];
            if (er[4 * (size_t)v + 3].x & kAdjMore)
              for (uint32_t e = gr.node_row[v] + 4; e < gr.node_row[v + 1]; ++e) {
                const uint4 pk = ld16(gr.edge_pack + e);
                const short2 hh = gr.edge_head[e];
                bool nw2;
                const int p2 = m_relax(L, lb, i, ha, pk.x | ((pk.z & 7u) << 28), pk.y, timed ? et[e] : 0u, e,
                                       (uint32_t)(uint16_t)hh.x, (uint32_t)(uint16_t)hh.y, sv.x, sv.y, mode_bit,
                                       my_relaxed, nw2);
                if (nw2) atomicAdd(&L.n_keys, 1);
                if (p2 >= 0) {
                  const int p = atomicAdd(&L.n_pend, 1);
                  if (p < PCAP) L.pend[p] = (uint16_t)p2;
                  else L.overflow = 1;
                }
              }
          }
        }
        __syncthreads();
        npend = L.n_pend;
        nkeys += L.n_keys;
        if (npend > PCAP) npend = PCAP;
      }
      __syncthreads();
      // ---- the next round's per-source minima
      if (lane < S) {
        L.src[lane].z = L.kn[lane];
        L.src[lane].w = L.dn[lane];
        L.kn[lane] = 0xFFFFFFFFu;
        L.dn[lane] = 0xFFFFFFFFu;
      }
      fail = L.overflow != 0 || nkeys > kMaxKeys;
      __syncthreads();
    }
#ifdef OTR_FORCE_RETRY
    if (a.force_edge & 1) fail = true;
#endif
    // ---- transition rows of every source (or the group's tasks to the single-source tiers)
    if (fail) {
      if (lane < ns) a.overflow_flag[t0 + lane] = 5;
    } else {
      const int64_t toff = (int64_t)(((uint64_t)r2.w << 32) | r2.z);
      uint32_t ntr = 0;
      for (int i = 0; i < ns; ++i) {
        const int cii = __shfl(ci, i);
        const uint32_t e_i = (uint32_t)__shfl((int)ei, i);
        const double p_i = __shfl(pi, i);
        const uint32_t d0i = (uint32_t)__shfl((int)d0, i), t0i = (uint32_t)__shfl((int)ts0, i);
        const bool searched = (smask >> i) & 1u;
        if (searched) ntr += (uint32_t)Kb;
        if (lane < Kb) {
          int64_t rr = -1, rt = 0;
          uint32_t rc = 0;
          if (forced) {
            rr = -1;
          } else if (ej == e_i && pj >= p_i) {
            const uint2 li = a.clen[sp * OTR_KMAX + cii];
            rr = part_mm(pj - p_i, li.x);
            if (timed) rt = part_mm(pj - p_i, li.y);
          } else if (searched) {
            const unsigned long long tl = L.tlab[i * TG + lane];
            if (tl != kGInf) {
              rr = (int64_t)d0i + g_d(tl);
              rt = (int64_t)t0i + g_t(tl);
              rc = g_c(tl);
            }
          }
          const bool valid = rr >= 0 && rr <= (int64_t)bmm && (!timed || rt <= (int64_t)bt);
          const int64_t o = toff + (int64_t)cii * Kb + lane;
          a.trans[o] = valid ? (uint32_t)rr : kNoRoute;
          a.trans_tc[o] = valid ? rc : 0u;
        }
      }
      if (counters) {
        const uint32_t st = wave_sum_u32(my_settled), rl = wave_sum_u32(my_relaxed);
        if (lane == 0) {
          const int sh = cshard();
          atomicAdd(&counters[3 * kCShards + sh], (unsigned long long)st);
          atomicAdd(&counters[4 * kCShards + sh], (unsigned long long)rl);
          atomicAdd(&counters[5 * kCShards + sh], (unsigned long long)ntr);
          atomicAdd(&counters[6 * kCShards + sh], (unsigned long long)__popc(smask));
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------
// K3m group list: the tasks of every turn-mode step (one per source candidate, in
// candidate order, k_tasks) cut into ceil(n / S) balanced groups of consecutive
// candidates (the nearest candidates share the most states), appended per wave.
// ------------------------------------------------------------------------------
template <int S>
__global__ __launch_bounds__(256) void k_mgroups(int64_t n_states, const int64_t* prev, const int32_t* cand_count,
                                                 const int64_t* task_off, const int32_t* state_trace,
                                                 const uint8_t* mode, uint32_t turn_modes, uint64_t* groups,
                                                 unsigned long long* count) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int ng = 0;
  int64_t t0 = 0, nt = 0;
  if (s < n_states && prev[s] >= 0 && cand_count[s] > 0) {
    const int md = mode[state_trace[s]] < OTR_MODES ? mode[state_trace[s]] : 0;
    if ((turn_modes >> md) & 1u) {
      t0 = task_off[s];
      nt = task_off[s + 1] - t0;
      ng = (int)((nt + S - 1) / S);
    }
  }
  // wave-aggregated append: inclusive scan of ng by shuffles, one atomic per wave
  int incl = ng;
  for (int d = 1; d < OTR_WAVE; d <<= 1) {
    const int y = __shfl_up(incl, d);
    if ((int)__lane_id() >= d) incl += y;
  }
  const int total = __shfl(incl, OTR_WAVE - 1);
  unsigned long long base = 0;
  if (__lane_id() == 0 && total > 0) base = atomicAdd(count, (unsigned long long)total);
  base = __shfl(base, 0);
  const int64_t first = (int64_t)base + incl - ng;
  for (int g = 0; g < ng; ++g) {
    const int64_t a = t0 + nt * g / ng, b = t0 + nt * (g + 1) / ng;
    groups[first + g] = (uint64_t)a | ((uint64_t)(b - a) << 56);
  }
}

}  // namespace otr
