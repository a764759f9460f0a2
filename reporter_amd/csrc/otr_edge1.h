// otr_edge1.h — K3e1: the lean single-source edge-state route search, the first tier of
// the turn-cost modes (the deployed configuration, Batch.java:56-65: every mode's default
// turn_penalty_factor is > 0).
//
// The semantics are otr_edge.h's (one source candidate per wave, states = edges, 64-bit
// labels key << 38 | (cap - turn) << 17 | time, exact IN-criterion rounds, the bounds
// pruning during the search, targets offered by every settled state at src(ej)); what
// changes is the cost of a round, which is what bounds this search (otr_edge.h's kernel,
// measured: ~13 rounds of ~600 wave instructions each, a third of the SIMD's VALU issue
// used at 4.25 waves per SIMD; this one: 4 waves per SIMD):
//   * one 16-B record per relaxation, indexed by the settled state (edge) and the out-edge
//     slot (DevGraph::erec: the out-edge's id, access and length, the turn degree from the
//     state into it, resolved at graph load), beside one 4-B per-mode route time;
//   * the IN criterion adds the mode's smallest turn cost (every later offer to a state
//     crosses a turn >= tmin and the state's own edge): lab(b) < kmin + len(b) + tmin is
//     final, and a target is final once tlab < kmin + tpart + tmin — fewer rounds, the
//     same final labels;
//   * a target is also resolved once the smallest pending route time plus its entry time
//     breaks the time bound (no later offer can be feasible): ~7 % fewer rounds at C2
//     (tools/edge_stats.py);
//   * settled states keep their pending bit (a final label can never improve, so it is
//     never pushed again): no write per settled state;
//   * probe loops are not unrolled, the target map is consulted only when a 64-bit bloom
//     of the target nodes (a wave-uniform register) admits the settled node, and the
//     wave's scalar state is kept small (no SGPR spills);
//   * small tables: the first tier holds 360 states (table + lists + targets + the turn
//     table in 10.1 KB: 16 waves per CU, ~96 % of the C2 searches); a search that outgrows
//     it goes on to 512 and 1024 states (this kernel again), then k_general: same results;
//   * a state is its label, its key (edge id) and its IN-gap code in LDS (15 B with the
//     pending index: 21 waves per CU), a settled state's label, edge and code one 16-B list
//     entry;
//   * the relax step is branch-free on its common path (e1_relax_sink);
//   * waves claim tasks from per-XCD queues (XcdQueue, otr_device.h).
#pragma once
#include <type_traits>

#include "otr_edge.h"

namespace otr {

// the edge-state record of slot k of state b (DevGraph::erec[4 b + k]):
// {e | access << 28 | more << 31, len_mm(e), turn degree b -> e | end heading of b << 8, dst(b)}
__device__ inline uint32_t er_edge(const uint4& r) { return r.x & kAdjDstMask; }
__device__ inline uint32_t er_deg(const uint4& r) { return r.z & 0xFFu; }
__device__ inline uint32_t er_hbk(const uint4& r) { return (uint32_t)heading_back((int)((r.z >> 8) & 0x1FFu)); }


// the first tier's settled-list size (states settled per round at most), and the larger tiers'
#ifndef OTR_E1WCAP
#define OTR_E1WCAP 32
#endif
#ifndef OTR_E1WCAP2
#define OTR_E1WCAP2 64
#endif
// the main relax loop without branches on its common path (e1_relax_sink), with this
// many scratch words (0: the branching e1_relax)
#ifndef OTR_E1SINK
#define OTR_E1SINK 16
#endif
// pending-list entries of the first table (at most OTR_E1CAP)
// (96: 23 waves per CU, but the 512-state tier's restarts cost more, 7.3 -> 9.6 ms)
#ifndef OTR_E1PCAP
#define OTR_E1PCAP OTR_E1CAP
#endif
// waves per SIMD the compiler fits the kernel's registers for (8: 64 VGPRs)
#ifndef OTR_E1WAVES
#define OTR_E1WAVES 8
#endif

template <int CAP>
struct E1Lds {
  static constexpr int TG = 32;   // targets (steps with more go on to k_general)
  static constexpr int TM = 32;   // target-node map slots (a target node per target at most)
  // states settled per round (the rest wait; a round's relax passes cover 16 states each)
  static constexpr int WCAP = CAP == OTR_E1CAP ? OTR_E1WCAP : (CAP <= 256 ? 32 : OTR_E1WCAP2);
  using Idx = typename std::conditional<(CAP <= 256), uint8_t, uint16_t>::type;
  unsigned long long lab[CAP];  // gpack label, kGInf: none
  uint32_t key[CAP];            // edge id | kInq (on the pending list, or settled); kEmpty
  uint8_t mi[CAP];              // mi8_of(len(edge)): the IN criterion's gap (0 at the root)
  // pending list capacity: the first table's may be shorter (OTR_E1PCAP: LDS for more
  // resident waves; a search whose frontier outgrows it restarts in the next table)
  static constexpr int PCAP = CAP == OTR_E1CAP ? OTR_E1PCAP : CAP;
  Idx pend[PCAP];               // pending slots
  uint4 wst[WCAP];              // this round's settled states: {label lo, hi, edge, mi} (one 16-B access)
  unsigned long long tlab[TG];  // the targets' best feasible offers
  uint32_t tpart[TG], tpt[TG];  // entry parts (mm, 0.1 s)
  uint16_t thb[TG];             // begin heading of the target edge
  uint32_t tm_node[TM];         // target node -> target lanes
  uint32_t tm_mask[TM];
  unsigned long long bloom;     // bit tm_home(v) of every target node v
  int32_t turn[181];
  int turn_md;
  uint32_t tmin;
  int n_pend, n_keys, overflow;
#if OTR_E1SINK
  unsigned long long sink[OTR_E1SINK];  // e1_relax_sink: the lanes' scratch words (never read)
#endif
};

__device__ inline uint32_t tm_home(uint32_t v) { return (v * 0x9E3779B1u) >> 26; }  // 64 bloom bits
__device__ inline uint32_t tm_slot(uint32_t v) { return (v * 0x9E3779B1u) >> 27; }  // 32 map slots


template <int CAP>
__device__ inline int e1_insert(E1Lds<CAP>& L, uint32_t e, bool& isnew) {
  uint32_t h = hslot<CAP>(e);
#pragma unroll 1
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = atomicCAS(&L.key[h], kEmpty, e);
    if (k == kEmpty) {
      isnew = true;
      return (int)h;
    }
    if ((k & kNodeMask) == e) return (int)h;
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  L.overflow = 1;
  return -1;
}

template <int CAP>
__device__ inline void e1_target_offers(E1Lds<CAP>& L, unsigned long long lb, uint32_t hbk, uint32_t v, uint32_t pd,
                                        uint32_t pt) {
  uint32_t h = tm_slot(v), m = 0;
#pragma unroll 1
  for (int probe = 0; probe < E1Lds<CAP>::TM; ++probe) {
    const uint32_t k = L.tm_node[h];
    if (k == v) m = L.tm_mask[h];
    if (k == v || k == kEmpty) break;
    h = (h + 1) & (E1Lds<CAP>::TM - 1);
  }
#pragma unroll 1
  while (m) {
    const int q = __ffs((int)m) - 1;
    m &= m - 1;
    const uint32_t tc = (uint32_t)L.turn[turn_from_back((int)hbk, (int)L.thb[q])];
    const EOffer o = e_step(lb, tc, L.tpart[q], L.tpt[q]);
    if (e_feasible(o, pd, pt)) atomicMin(&L.tlab[q], gpack(o.k, o.c, o.t));
  }
}

// relax the final state (label lb) through one out-edge b: access bits in dw, length,
// time, the turn degree into b; returns the slot when b's state became newly pending
template <int CAP>
__device__ inline int e1_relax(E1Lds<CAP>& L, unsigned long long lb, uint32_t dw, uint32_t len, uint32_t tt,
                               uint32_t b, uint32_t deg, uint32_t pd, uint32_t pt, uint32_t mode_bit,
                               uint32_t& relaxed, uint32_t& knext, uint32_t& dnext, uint32_t& tnext, bool& isnew) {
  if (!(((dw >> 28) & 7u) & mode_bit)) return -1;
  ++relaxed;
  const uint32_t tc = (uint32_t)L.turn[deg];
  const EOffer o = e_step(lb, tc, len, tt);
  if (!e_feasible(o, pd, pt)) return -1;  // pruned (label-setting semantics)
  const int sl = e1_insert(L, b, isnew);
  if (sl < 0) return -1;
  if (isnew) {
    L.mi[sl] = mi8_of(len);
    L.lab[sl] = kGInf;
  }
  const unsigned long long nw = gpack(o.k, o.c, o.t);
  const unsigned long long old = atomicMin(&L.lab[sl], nw);
  if (nw >= old) return -1;
  knext = o.k < knext ? o.k : knext;
  dnext = o.d < dnext ? o.d : dnext;
  tnext = o.t < tnext ? o.t : tnext;
  return (atomicOr(&L.key[sl], kInq) & kInq) ? -1 : sl;
}

#if OTR_E1SINK
// e1_relax with its common path branch-free (as relax_sink, otr_kernels.h): every lane
// issues the insert, the new state's stores, the label and the pending-bit atomics, a lane
// with nothing to do aiming them at its own scratch word L.sink[lane], so the exec-mask
// bookkeeping of the nested ifs (scalar-unit work) is gone.  Only a probe chain past the
// home slot branches.  Same slots, labels and pending list as e1_relax.
template <int CAP>
__device__ inline int e1_relax_sink(E1Lds<CAP>& L, unsigned long long lb, uint32_t dw, uint32_t len, uint32_t tt,
                                    uint32_t b, uint32_t deg, uint32_t pd, uint32_t pt, uint32_t mode_bit,
                                    uint32_t& relaxed, uint32_t& knext, uint32_t& dnext, uint32_t& tnext,
                                    bool& isnew) {
  unsigned long long* mine = &L.sink[threadIdx.x % OTR_E1SINK];  // (lanes sharing a word: a few-way atomic)
  uint32_t* mine32 = reinterpret_cast<uint32_t*>(mine);
  const bool mode_ok = (((dw >> 28) & 7u) & mode_bit) != 0u;
  relaxed += mode_ok ? 1u : 0u;
  // the insert needs only the length and time bounds (neither depends on the turn), so
  // its CAS and the turn-table read are in flight together; an offer that then breaks the
  // turn-cost cap leaves a key without a label (never pending: same labels)
  bool go = mode_ok && g_d(lb) + len <= pd && g_t(lb) + tt <= pt;
  const uint32_t h0 = hslot<CAP>(b);
  const uint32_t k0 = atomicCAS(go ? &L.key[h0] : mine32, kEmpty, b);
  const uint32_t tc = (uint32_t)L.turn[deg];
  const EOffer o = e_step(lb, tc, len, tt);
  isnew = go && k0 == kEmpty;
  int sl = (go && (k0 == kEmpty || (k0 & kNodeMask) == b)) ? (int)h0 : -1;
  const bool coll = go && sl < 0;
  if (__ballot(coll) != 0ull) {  // the home slot holds another edge: linear probing
    if (coll) {
      uint32_t hh = h0;
#pragma unroll 1
      for (int probe = 1; probe < CAP; ++probe) {
        hh = hh + 1 == (uint32_t)CAP ? 0u : hh + 1;
        const uint32_t k = atomicCAS(&L.key[hh], kEmpty, b);
        if (k == kEmpty) {
          isnew = true;
          sl = (int)hh;
          break;
        }
        if ((k & kNodeMask) == b) {
          sl = (int)hh;
          break;
        }
      }
      if (sl < 0) L.overflow = 1;
    }
  }
  go = go && sl >= 0;
  const bool fresh = go && isnew;
  *(fresh ? &L.mi[sl] : reinterpret_cast<uint8_t*>(mine)) = mi8_of(len);
  *(fresh ? &L.lab[sl] : mine) = kGInf;
  const unsigned long long nw = gpack(o.k, o.c, o.t);
  const bool feas = go && o.c <= kTcCap;
  const unsigned long long old = atomicMin(feas ? &L.lab[sl] : mine, nw);
  const bool imp = feas && nw < old;
  knext = (imp && o.k < knext) ? o.k : knext;
  dnext = (imp && o.d < dnext) ? o.d : dnext;
  tnext = (imp && o.t < tnext) ? o.t : tnext;
  const uint32_t was = atomicOr(imp ? &L.key[sl] : mine32, kInq);
  return (imp && !(was & kInq)) ? sl : -1;
}
#endif

template <int CAP>
__device__ inline void e1_turn_table(E1Lds<CAP>& L, const int32_t* turn_tab, int md) {
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

// ------------------------------------------------------------------------------
// Resuming an outgrown search in the next table.  A search stops between two rounds when
// its keys pass the table's load limit (no relaxation lost: the table never filled), and
// its whole state goes to a dump slot in HBM: the round's frontier values (kmin, dmin,
// tmn), the targets' best offers, and every key of the table with its label — settled
// states too, whose final labels must keep rejecting later offers.  The next tier's wave
// re-inserts the keys into its larger table, rebuilds each state's static word from the
// graph (its IN-gap code), refills the pending list and goes
// on with the next round: the same rounds the search would have run in one big table, so
// the same labels, without redoing the part already searched.
// Slot layout (u64 words): [0..1] {entries, pending, kmin, dmin}, [2..3] {tmn, settled,
// relaxed, 0}, [8..39] the targets' offers, [40..40+CAP) labels, then CAP u32 keys
// (edge id | kInq | kDumpPend).
// ------------------------------------------------------------------------------
constexpr uint32_t kDumpPend = 0x40000000u;  // dump key bit: the state is on the pending list
__host__ __device__ constexpr uint32_t e1_dump_words(int cap) { return 40u + (uint32_t)cap + ((uint32_t)cap + 1u) / 2u; }

template <int CAP>
__device__ inline void e1_dump(E1Lds<CAP>& L, unsigned long long* D, int npend, uint32_t kmin, uint32_t dmin,
                               uint32_t tmn, uint32_t settled, uint32_t relaxed) {
  const int lane = (int)threadIdx.x;
  for (int k = lane; k < npend; k += OTR_WAVE) L.key[L.pend[k]] |= kDumpPend;  // (one list entry per state)
  __syncthreads();
  unsigned long long* dl = D + 40;
  uint32_t* dk = reinterpret_cast<uint32_t*>(dl + CAP);
  int n = 0;
#pragma unroll 1
  for (int base = 0; base < CAP; base += OTR_WAVE) {
    const int k = base + lane;
    const uint32_t kw = k < CAP ? L.key[k] : kEmpty;
    const bool has = kw != kEmpty;
    const unsigned long long m = __ballot(has);
    if (has) {
      const int pos = n + prefix_count(m);
      dl[pos] = L.lab[k];
      dk[pos] = kw;
    }
    n += __popcll(m);
  }
  if (lane < E1Lds<CAP>::TG) D[8 + lane] = L.tlab[lane];
  if (lane == 0) {
    reinterpret_cast<uint4*>(D)[0] = make_uint4((uint32_t)n, (uint32_t)npend, kmin, dmin);
    reinterpret_cast<uint4*>(D)[1] = make_uint4(tmn, settled, relaxed, 0u);
  }
}

// the dumped search back into this (empty, larger) table; returns its key count, the
// pending list in L.pend[0..npend)
template <int CAP>
__device__ inline int e1_restore(E1Lds<CAP>& L, const DevGraph& gr, const unsigned long long* D, uint32_t in_cap,
                                 uint32_t ei, int& npend, uint32_t& kmin, uint32_t& dmin, uint32_t& tmn,
                                 uint32_t& settled, uint32_t& relaxed) {
  const int lane = (int)threadIdx.x;
  const uint4 h0 = reinterpret_cast<const uint4*>(D)[0], h1 = reinterpret_cast<const uint4*>(D)[1];
  const int n = (int)h0.x;
  kmin = h0.z;
  dmin = h0.w;
  tmn = h1.x;
  if (lane == 0) {
    settled += h1.y;
    relaxed += h1.z;
  }
  if (lane < E1Lds<CAP>::TG) L.tlab[lane] = D[8 + lane];
  const unsigned long long* dl = D + 40;
  const uint32_t* dk = reinterpret_cast<const uint32_t*>(dl + in_cap);
  int np = 0;
#pragma unroll 1
  for (int base = 0; base < n; base += OTR_WAVE) {
    const int k = base + lane;
    bool pend = false;
    int sl = 0;
    if (k < n) {
      const uint32_t kw = dk[k];
      const unsigned long long lb = dl[k];
      const uint32_t e = kw & kNodeMask;
      uint32_t h = hslot<CAP>(e);
#pragma unroll 1
      for (int probe = 0; probe < CAP; ++probe) {  // (distinct keys, a larger table: an empty slot)
        if (atomicCAS(&L.key[h], kEmpty, e) == kEmpty) break;
        h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
      }
      sl = (int)h;
      L.key[sl] = kw & (kNodeMask | kInq);
      L.lab[sl] = lb;
      L.mi[sl] = e == ei ? (uint8_t)0 : mi8_of(gr.len_mm[e]);
      pend = (kw & kDumpPend) != 0u;
    }
    const unsigned long long mp = __ballot(pend);
    if (pend) L.pend[np + prefix_count(mp)] = (typename E1Lds<CAP>::Idx)sl;
    np += __popcll(mp);
  }
  npend = np;
  return n;
}

// ------------------------------------------------------------------------------
// K3e1 kernel: a persistent grid over the device-side list of the turn-mode tasks (one
// source candidate each), the 8 XCDs taking contiguous eighths of the list (consecutive
// tasks = the candidates of one step, then the next steps of the trace: one neighbourhood),
// each wave claiming its next task from its XCD's queue (XcdQueue).
// A search that outgrows the table flags its task for the next tier: 6 (512 states), 7
// (1024), 3 (k_general, global-memory labels).
// ------------------------------------------------------------------------------
template <int CAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(OTR_E1WAVES, 8))) void k_route_e1(
    DevGraph gr, RouteArgs a, unsigned long long* counters) {
  using LT = E1Lds<CAP>;
  constexpr int TG = LT::TG, TM = LT::TM, WCAP = LT::WCAP;
  constexpr int kMaxKeys = CAP == OTR_E1CAP ? (CAP * OTR_E1LOAD) / 16 : (CAP * 7) / 8;
  __shared__ LT L;
  if (threadIdx.x == 0) L.turn_md = -1;
  const int lane = (int)threadIdx.x;
  XcdQueue q(a.queue, (int64_t)*a.list_count);
  unsigned long long cyc_res = 0, cyc_part = 0, cyc_relax = 0, cyc_other = 0;  // (OTR_STAMPS)
  for (int64_t w = q.next(); w < q.hi; w = q.next()) {
    OTR_STAMP(ts0);
    const int64_t task = a.task_list[w];
    const uint4 r0 = a.rec[3 * task], r1 = a.rec[3 * task + 1], r2 = a.rec[3 * task + 2];
    const int64_t s = r0.x, sp = r0.y;
    const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
    const int i = __ffsll((long long)mask) - 1;  // the task's one source
    const int Kb = (int)(r1.y & 0xFFu);
    const int md = (int)((r1.y >> 8) & 3u);
    const bool forced = (r1.y >> 10) & 1u;
    const uint32_t bmm = r0.w;
    const int32_t bt = (int32_t)r2.y;
    const bool timed = bt >= 0;
    const uint32_t ei = a.cand_edge[sp * OTR_KMAX + i];
    const double pi = a.cand_p[sp * OTR_KMAX + i];
    const uint32_t d0 = a.cprep[sp * OTR_KMAX + i].w;
    const uint32_t t0 = timed ? a.cprep_t[sp * OTR_KMAX + i].y : 0u;
    uint32_t ej = 0, tv = kEmpty, tpart = 0, tpt = 0, thb = 0;
    double pj = 0;
    bool needed = false;
    if (lane < Kb) {
      ej = a.cand_edge[s * OTR_KMAX + lane];
      pj = a.cand_p[s * OTR_KMAX + lane];
      const uint4 cq = a.cprep[s * OTR_KMAX + lane];
      tpart = cq.x;
      thb = cq.z;  // (turn modes: the begin heading of ej, k_prep)
      tpt = timed ? a.cprep_t[s * OTR_KMAX + lane].x : 0u;
      needed = !(ej == ei && pj >= pi);
      if (needed) tv = cq.y;
    }
    const bool root_ok = d0 <= bmm && (!timed || t0 <= (uint32_t)bt);
    const bool search = Kb <= TG && !forced && root_ok && __ballot(needed) != 0ull;
    const uint32_t pd = bmm >= d0 ? bmm - d0 : 0u;
    const uint32_t pt = !timed ? 0xFFFFFFFFu : (t0 <= (uint32_t)bt ? (uint32_t)bt - t0 : 0u);
    // ---- reset: keys, targets, the target map and its bloom
    for (int k = lane; k < CAP; k += OTR_WAVE) L.key[k] = kEmpty;
    if (lane < TG) L.tlab[lane] = kGInf;
    if (lane < TM) {
      L.tm_node[lane] = kEmpty;
      L.tm_mask[lane] = 0u;
    }
    if (lane == 0) {
      L.overflow = 0;
      L.bloom = 0ull;
    }
    e1_turn_table(L, a.turn, md);
    const bool tgt = search && lane < Kb && tv != kEmpty;
    if (tgt) {
      L.tpart[lane] = tpart;
      L.tpt[lane] = tpt;
      L.thb[lane] = (uint16_t)thb;
      uint32_t h = tm_slot(tv);
#pragma unroll 1
      for (int probe = 0; probe < TM; ++probe) {
        const uint32_t k = atomicCAS(&L.tm_node[h], kEmpty, tv);
        if (k == kEmpty || k == tv) {
          atomicOr(&L.tm_mask[h], 1u << lane);
          break;
        }
        h = (h + 1) & (TM - 1);
      }
      atomicOr(&L.bloom, 1ull << tm_home(tv));
    }
    __syncthreads();
    // the bloom of the target nodes: a settled state consults the map only on a hit
    const unsigned long long bloom = L.bloom;
    bool ok = true, dump = false;
    uint32_t my_settled = 0, my_relaxed = 0;
    uint32_t kmin = 0, dmin = 0, tmn = 0;  // the smallest pending key / length / time
    int npend = 1, nkeys = 1;
    // a search the previous (smaller) table outgrew goes on from its dump (e1_restore)
    const int32_t rslot = (a.dump_in != nullptr && search) ? a.task_dump[task] : -1;
    if (search) {
      if (rslot >= 0) {
        nkeys = e1_restore(L, gr, a.dump_in + (size_t)rslot * a.dump_in_words, a.dump_in_cap, ei, npend, kmin, dmin, tmn,
                           my_settled, my_relaxed);
      } else if (lane == 0) {
        bool isnew = false;
        const int sl = e1_insert(L, ei, isnew);  // (an empty table: the home slot)
        // the root: label 0 is final at once (mi 0: gap 1 mm)
        L.mi[sl] = 0;
        L.lab[sl] = gpack(0u, 0u, 0u);
        L.key[sl] = ei | kInq;
        L.pend[0] = (typename LT::Idx)sl;
      }
      __syncthreads();
      const uint4* er = gr.erec;
      const uint32_t* ert = gr.erec_t + (size_t)md * gr.erec_stride;
      const uint32_t mode_bit = 1u << md;
      const uint32_t tmin = L.tmin;
#ifdef OTR_FORCE_RETRY
      int rounds = 0;
#endif
#pragma unroll 1
      for (;;) {
        OTR_STAMP(tr0);
        // ---- targets: every later offer to a target has key >= kmin + tpart + tmin,
        // length >= dmin + tpart and route time >= tmn + tpt (every later label descends
        // from a pending one); done when every needed target is final or unreachable
        // (branch-free: every lane reads a target word, lanes >= TG their lane - TG's)
        const unsigned long long tl = L.tlab[lane & (TG - 1)];
        const bool res = !tgt | ((tl != kGInf) & ((uint64_t)g_k(tl) < (uint64_t)kmin + tpart + tmin)) |
                         ((uint64_t)dmin + tpart > (uint64_t)pd) | ((uint64_t)tmn + tpt > (uint64_t)pt);
        if (__ballot(!res) == 0ull || npend == 0) break;
        OTR_STAMP(tr1);
        // ---- partition: final pending states (IN criterion) to the settled list; the
        // rest stay and give the next kmin / dmin
        uint32_t knext = 0xFFFFFFFFu, dnext = 0xFFFFFFFFu, tnext = 0xFFFFFFFFu;
        int kept = 0, nw = 0;
#pragma unroll 1
        for (int base = 0; base < npend; base += OTR_WAVE) {
          const int k = base + lane;
          const bool in = k < npend;
          // the reads are unconditional (a lane past the list reads entry 0: npend > 0 here),
          // so no exec-mask branch around them
          const int sl = L.pend[in ? k : 0];
          const unsigned long long lb = L.lab[sl];
          const uint32_t kw = L.key[sl];  // (read beside the label: the relax lanes then need no dependent read)
          const uint32_t mq = L.mi[sl];
          bool take = in && (uint64_t)g_k(lb) < (uint64_t)kmin + in_gap8((uint8_t)mq) + tmin;
          take = take && nw + prefix_count(__ballot(take)) < WCAP;
          const bool keep = in && !take;
          const unsigned long long mtk = __ballot(take), mk = __ballot(keep);
          __syncthreads();
          if (take) {
            const int wq = nw + prefix_count(mtk);
            L.wst[wq] = make_uint4((uint32_t)lb, (uint32_t)(lb >> 32), kw & kNodeMask, mq);
          } else if (keep) {
            L.pend[kept + prefix_count(mk)] = (typename LT::Idx)sl;
            knext = g_k(lb) < knext ? g_k(lb) : knext;
            dnext = g_d(lb) < dnext ? g_d(lb) : dnext;
            tnext = g_t(lb) < tnext ? g_t(lb) : tnext;
          }
          nw += __popcll(mtk);
          kept += __popcll(mk);
          __syncthreads();
        }
        npend = kept;
        OTR_STAMP(tr2);
        // ---- relax: lane = (settled state, adjacency slot)
        uint32_t tail = 0u;  // (a lane word, not a lane mask: VALU ors instead of scalar mask updates)
#pragma unroll 1
        for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
          const int k = base + lane;
          int psl = -1;
          bool isnew = false;
          if (k < 4 * nw) {
            const uint4 ws = L.wst[k >> 2];
            const unsigned long long lb = ((unsigned long long)ws.y << 32) | ws.x;
            const size_t ri = 4 * (size_t)ws.z + (k & 3);  // the settled state's slot record
            // the slot's route time, loaded beside the record and unconditionally
            const uint32_t tq = ert[ri];
            const uint4 r = ld16(er + ri);
            const uint32_t tt = timed ? tq : 0u;
            if ((k & 3) == 0) {  // the state's head node (r.w) may be a target's source
              ++my_settled;
              if ((bloom >> tm_home(r.w)) & 1ull) e1_target_offers(L, lb, er_hbk(r), r.w, pd, pt);
            }
#if OTR_E1SINK
            psl = e1_relax_sink(L, lb, r.x & ~kAdjMore, r.y, tt, er_edge(r), er_deg(r), pd, pt, mode_bit, my_relaxed,
                                knext, dnext, tnext, isnew);
#else
            psl = e1_relax(L, lb, r.x & ~kAdjMore, r.y, tt, er_edge(r), er_deg(r), pd, pt, mode_bit, my_relaxed, knext,
                           dnext, tnext, isnew);
#endif
            tail |= ((k & 3) == 3) ? (r.x & kAdjMore) : 0u;
          }
          nkeys += __popcll(__ballot(isnew));
          const unsigned long long mp = __ballot(psl >= 0);
          if (psl >= 0 && (LT::PCAP == CAP || npend + prefix_count(mp) < LT::PCAP))  // (< CAP: one entry per state)
            L.pend[npend + prefix_count(mp)] = (typename LT::Idx)psl;
          npend += __popcll(mp);
        }
        if (__ballot(tail != 0u) != 0ull) {  // nodes with more than four out-edges: the CSR tail
          if (lane == 0) {
            L.n_pend = npend;
            L.n_keys = 0;
          }
          __syncthreads();
#pragma unroll 1
          for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
            const int k = base + lane;
            if (k < 4 * nw && (k & 3) == 3) {
              const uint4 ws = L.wst[k >> 2];
              const unsigned long long lb = ((unsigned long long)ws.y << 32) | ws.x;
              const uint4 r3 = er[4 * (size_t)ws.z + 3];
              if (r3.x & kAdjMore) {
                const uint32_t* et = gr.et(md);
                const uint32_t v = r3.w, hbk = er_hbk(r3);
#pragma unroll 1
                for (uint32_t e = gr.node_row[v] + 4; e < gr.node_row[v + 1]; ++e) {
                  const uint4 pk = ld16(gr.edge_pack + e);
                  const uint32_t deg = (uint32_t)turn_from_back((int)hbk, (int)(uint16_t)gr.edge_head[e].x);
                  bool nw2 = false;
                  const int p2 = e1_relax(L, lb, pk.x | ((pk.z & 7u) << 28), pk.y, timed ? et[e] : 0u, e, deg, pd, pt,
                                          mode_bit, my_relaxed, knext, dnext, tnext, nw2);
                  if (nw2) atomicAdd(&L.n_keys, 1);
                  if (p2 >= 0) {
                    const int p = atomicAdd(&L.n_pend, 1);
                    if (LT::PCAP == CAP || p < LT::PCAP) L.pend[p] = (typename LT::Idx)p2;
                  }
                }
              }
            }
          }
          __syncthreads();
          npend = L.n_pend;
          nkeys += L.n_keys;
        }
        OTR_STAMP(tr3);
        __syncthreads();
        kmin = wave_min_u32(knext);
        dmin = wave_min_u32(dnext);
        tmn = wave_min_u32(tnext);
#ifdef OTR_STAMPS
        OTR_STAMP(tr4);
        cyc_res += (tr1 - tr0) + (tr4 - tr3);
        cyc_part += tr2 - tr1;
        cyc_relax += tr3 - tr2;
#endif
        // (a pending list past its capacity lost appends, as a full table loses a
        // relaxation: that search restarts)
        const bool pover = LT::PCAP < CAP && npend > LT::PCAP;
        if (L.overflow || pover || nkeys > kMaxKeys) {
          ok = false;
          dump = !L.overflow && !pover;  // (a full table lost a relaxation: that search restarts)
          break;
        }
#ifdef OTR_FORCE_RETRY  // test build: OTR_FORCE_EDGE bit 5 / 6 stops every OTR_E1CAP / 512-state search
                        // after 2 / 4 rounds, to be resumed in the next table
        ++rounds;
        if (((a.force_edge & 32) && CAP == OTR_E1CAP && rounds == 2) ||
            ((a.force_edge & 64) && CAP == 512 && rounds == 4)) {
          ok = false;
          dump = true;
          break;
        }
#endif
      }
    }
#ifdef OTR_FORCE_RETRY  // test build: OTR_FORCE_EDGE bit 0 / 1 / 2 fails every OTR_E1CAP (360) / 512 / 1024-state search
    if (a.force_edge & (CAP < 512 ? 1 : (CAP < 1024 ? 2 : 4))) {
      ok = false;
      dump = false;
    }
#endif
    ok = ok && Kb <= TG;
    if (ok) {
      uint32_t* trow = a.trans + (int64_t)(((uint64_t)r2.w << 32) | r2.z);
      if (lane < Kb) {
        // the target's edge and fraction re-read here (L2-warm) rather than held in
        // registers through the search
        const uint32_t ej2 = a.cand_edge[s * OTR_KMAX + lane];
        const double pj2 = a.cand_p[s * OTR_KMAX + lane];
        int64_t rr = -1, rt = 0;
        uint32_t rc = 0;
        if (forced) {
          rr = -1;
        } else if (ej2 == ei && pj2 >= pi) {
          const uint2 li = a.clen[sp * OTR_KMAX + i];
          rr = part_mm(pj2 - pi, li.x);
          if (timed) rt = part_mm(pj2 - pi, li.y);
        } else if (search) {
          const unsigned long long tl = L.tlab[lane];
          if (tl != kGInf) {
            rr = (int64_t)d0 + g_d(tl);
            rt = (int64_t)t0 + g_t(tl);
            rc = g_c(tl);
          }
        }
        const bool valid = rr >= 0 && rr <= (int64_t)bmm && (!timed || rt <= (int64_t)bt);
        trow[(int64_t)i * Kb + lane] = valid ? (uint32_t)rr : kNoRoute;
        a.trans_tc[trow - a.trans + (int64_t)i * Kb + lane] = valid ? rc : 0u;
      }
      if (counters) {
        const uint32_t st = wave_sum_u32(my_settled), rl = wave_sum_u32(my_relaxed);
        if (lane == 0) {
          const int sh = cshard();
          atomicAdd(&counters[3 * kCShards + sh], (unsigned long long)st);
          atomicAdd(&counters[4 * kCShards + sh], (unsigned long long)rl);
          atomicAdd(&counters[5 * kCShards + sh], search ? (unsigned long long)Kb : 0ull);
          atomicAdd(&counters[6 * kCShards + sh], search ? 1ull : 0ull);
          if (rslot >= 0) atomicAdd(&counters[22 * kCShards + sh], 1ull);  // (resumed from a dump)
        }
      }
    } else {
      // the next table (512, 1024 states, then k_general) resumes the search from its dump
      // when it stopped between two rounds and a dump slot is free, else starts it afresh
      int32_t slot = -1;
      if (dump && a.dump_out != nullptr) {
        unsigned long long v = 0;
        if (lane == 0) v = atomicAdd(a.dump_ctr, 1ull);
        v = (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        if (v < (unsigned long long)a.dump_out_slots) slot = (int32_t)v;
      }
      if (slot >= 0) e1_dump(L, a.dump_out + (size_t)slot * a.dump_out_words, npend, kmin, dmin, tmn, 0u, 0u);
      if (counters && slot >= 0 && lane == 0) atomicAdd(&counters[23 * kCShards + cshard()], 1ull);
      if (lane == 0) {
        a.overflow_flag[task] = CAP < 512 ? 6 : (CAP < 1024 ? 7 : 3);
        if (a.task_dump != nullptr) a.task_dump[task] = slot;
      }
    }
    __syncthreads();
#ifdef OTR_STAMPS
    OTR_STAMP(ts1);
    cyc_other += ts1 - ts0;
#endif
  }
#ifdef OTR_STAMPS  // phase cycles summed over waves: 16 resolution + round end, 17 partition, 18 relax, 19 all
  if (threadIdx.x == 0 && a.stamps) {
    const int sh = cshard();
    atomicAdd(&a.stamps[16 * kCShards + sh], cyc_res);
    atomicAdd(&a.stamps[17 * kCShards + sh], cyc_part);
    atomicAdd(&a.stamps[18 * kCShards + sh], cyc_relax);
    atomicAdd(&a.stamps[19 * kCShards + sh], cyc_other);
  }
#endif
}

}  // namespace otr
