// otr_edge.h — K3e/K6e: the edge-state route search in LDS, for modes with turn costs.
//
// With turn costs a route's key (length + turn cost) depends on the edge a
// node is entered by, so the states of the search are edges: state b = "at dst(b), having
// arrived through b".  The search is the node search of otr_kernels.h (search_run) over
// those states — exact rounds (the IN criterion: a state b is final once its key is below
// the smallest pending key + len(b), since every later offer to b crosses b itself), one
// lane per (settled state, adjacency slot), LDS hash insert + 64-bit atomicMin — with:
//   * 64-bit labels key << 38 | (kTcCap - turn) << 17 | time (otr_general.h gpack): the
//     atomicMin keeps the lexicographic minimum of (key, length, time), the oracle's order;
//   * the turn cost of every relaxation from the table of the mode, by the turn degree
//     between the state's end heading (kept in the table) and the out-edge's begin heading
//     (DevGraph::adj_e, loaded beside the adjacency record: no dependent load);
//   * targets are not states: the target edge ej is entered from any state at src(ej), so
//     every settled state at a target node offers to the target (with the turn into ej
//     and the entry part) and the target keeps the lexicographic minimum offer (tlab);
//   * two search frontiers: kmin over the key decides finality, dmin over the length
//     decides unreachability (the bounds are on the length);
//   * the same pruning as search_run (time, length and turn cost all prune); every offer
//     comes from a final label, so the labels are the oracle's label-setting ones.
// One search per wave (G = 1).  The route tiers of the turn modes are otr_edge1.h's
// k_route_e1; this header's edge_search is the winner-path search (k_paths_edge).
#pragma once
#include "otr_general.h"

namespace otr {

// TG: the targets a search holds (lanes < TG; 32 when every mode keeps <= 32 candidates).
// The state's end heading (the turn out of it) is read from DevGraph::edge_head by the
// relaxing lane, beside the adjacency loads, rather than kept per slot: 18 B per state, so
// more waves fit the LDS (the search waits on memory, not issue).
template <int CAP, int TG = OTR_WAVE>
struct EdgeLds {
  static constexpr int WCAP = CAP <= 512 ? 32 : 128;
  unsigned long long lab[CAP];   // gpack label, kGInf: none
  uint32_t key[CAP];             // edge id | kInq | kRel, kEmpty
  uint32_t node[CAP];            // dst(edge): where the state stands
  uint16_t pend[CAP];            // pending slots
  uint8_t mi[CAP];               // mi8_of(len(edge)): the IN criterion's gap of the state
  int32_t turn[181];             // the task's mode's turn cost table (mm), loaded per mode
  int turn_md;                   // the mode whose table is loaded (-1: none)
  uint16_t wslot[WCAP];          // this round's settled states' slots
  unsigned long long wlab[WCAP];  // ... and their labels
  // targets (lanes of the wave): the best offer, entry parts, begin heading of ej
  unsigned long long tlab[TG];
  uint32_t tpart[TG], tpt[TG];
  uint16_t thb[TG];
  // target nodes src(ej) → lane masks (open addressing)
  uint32_t tmap_node[TG];
  unsigned long long tmap_mask[TG];
  int n_pend, n_keys, overflow;
};

template <int CAP, int TG>
__device__ inline int e_find(const EdgeLds<CAP, TG>& L, uint32_t e) {
  uint32_t h = hslot<CAP>(e);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = L.key[h];
    if (k == kEmpty) return -1;
    if ((k & kNodeMask) == e) return (int)h;
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  return -1;
}

template <int CAP, int TG>
__device__ inline int e_insert(EdgeLds<CAP, TG>& L, uint32_t e, bool* isnew) {
  uint32_t h = hslot<CAP>(e);
  for (int probe = 0; probe < CAP; ++probe) {
    const uint32_t k = atomicCAS(&L.key[h], kEmpty, e);
    if (k == kEmpty) {
      *isnew = true;
      return (int)h;
    }
    if ((k & kNodeMask) == e) {
      *isnew = false;
      return (int)h;
    }
    h = h + 1 == (uint32_t)CAP ? 0u : h + 1;
  }
  L.overflow = 1;
  *isnew = false;
  return -1;
}

// a state's IN-criterion gap in 256-mm units rounded down (a lower bound of its edge's
// length, saturating at 65 m), 1 mm when below one unit
__device__ inline uint8_t mi8_of(uint32_t len) { return (uint8_t)((len >> 8) < 255u ? (len >> 8) : 255u); }
__device__ inline uint32_t in_gap8(uint8_t mq) { return mq ? (uint32_t)mq << 8 : 1u; }

// the mode's turn table into LDS (one global read per task whose mode differs from the
// last one's): every relaxation's turn cost is then an LDS read, not a dependent global load
template <int CAP, int TG>
__device__ inline void e_turn_table(EdgeLds<CAP, TG>& L, const int32_t* turn_tab, int md) {
  if (L.turn_md != md) {  // (uniform: the whole wave runs one task)
    __syncthreads();
    for (int k = threadIdx.x; k < 181; k += OTR_WAVE) L.turn[k] = turn_tab[181 * md + k];
    if (threadIdx.x == 0) L.turn_md = md;
    __syncthreads();
  }
}

template <int TG>
__device__ inline uint32_t tmap_home(uint32_t v) {  // TG slots (a power of two)
  return (v * 0x9E3779B1u) >> (32 - __builtin_ctz((unsigned)TG));
}

template <int CAP, int TG>
__device__ inline unsigned long long tmap_get(const EdgeLds<CAP, TG>& L, uint32_t v) {
  uint32_t h = tmap_home<TG>(v);
  for (int probe = 0; probe < TG; ++probe) {
    const uint32_t k = L.tmap_node[h];
    if (k == kEmpty) return 0ull;
    if (k == v) return L.tmap_mask[h];
    h = (h + 1) & (TG - 1);
  }
  return 0ull;
}

// an offer (relative key, length, time, turn) and its feasibility under the task's bounds
struct EOffer {
  uint32_t k, d, t, c;
};
__device__ inline bool e_feasible(const EOffer& o, uint32_t pd, uint32_t pt) {
  return o.d <= pd && o.t <= pt && o.c <= kTcCap;
}

// the offer of label lb through a step (turn tc, length len, time tt)
__device__ inline EOffer e_step(unsigned long long lb, uint32_t tc, uint32_t len, uint32_t tt) {
  EOffer o;
  o.c = g_c(lb) + tc;
  o.d = g_d(lb) + len;
  o.k = o.d + o.c;
  o.t = g_t(lb) + tt;
  return o;
}

// Relax the FINAL state (label lb, at node v, end heading ha) through the edge b (head w,
// length len, time tt, begin / end headings hb / he, access in dw's high bits).  Returns
// the slot when b became newly pending.
template <int CAP, int TG>
__device__ inline int e_relax(EdgeLds<CAP, TG>& L, unsigned long long lb, uint32_t ha, uint32_t dw,
                              uint32_t len, uint32_t tt, uint32_t b, uint32_t hb, uint32_t pd, uint32_t pt,
                              uint32_t mode_bit, uint32_t& relaxed, uint32_t& knext, uint32_t& dnext, bool& isnew) {
  isnew = false;
  if (!(((dw >> 28) & 7u) & mode_bit)) return -1;
  ++relaxed;
  const uint32_t tc = (uint32_t)L.turn[turn_degree((int)ha, (int)hb)];
  const EOffer o = e_step(lb, tc, len, tt);
  if (!e_feasible(o, pd, pt)) return -1;  // pruned (label-setting semantics)
  const uint32_t w = dw & kAdjDstMask;
  const int sl = e_insert(L, b, &isnew);
  if (sl < 0) return -1;
  if (isnew) {
    L.node[sl] = w;
    L.mi[sl] = mi8_of(len);
  }
  const unsigned long long nw = gpack(o.k, o.c, o.t);
  const unsigned long long old = atomicMin(&L.lab[sl], nw);
  if (nw < old) {
    knext = o.k < knext ? o.k : knext;
    dnext = o.d < dnext ? o.d : dnext;
    const uint32_t was = atomicOr(&L.key[sl], kInq);
    if (!(was & kInq)) return sl;
  }
  return -1;
}

// The settled (final) state's offers to the targets at its node v (the turn into ej + the
// entry part), kept as each target's lexicographic minimum.
template <int CAP, int TG>
__device__ inline void e_target_offers(EdgeLds<CAP, TG>& L, unsigned long long lb, uint32_t ha,
                                       uint32_t v, uint32_t pd, uint32_t pt) {
  unsigned long long m = tmap_get(L, v);
  while (m) {
    const int q = __ffsll((long long)m) - 1;
    m &= m - 1;
    const uint32_t tc = (uint32_t)L.turn[turn_degree((int)ha, (int)L.thb[q])];
    const EOffer o = e_step(lb, tc, L.tpart[q], L.tpt[q]);
    if (e_feasible(o, pd, pt)) atomicMin(&L.tlab[q], gpack(o.k, o.c, o.t));
  }
}

template <int CAP, int TG>
__device__ inline void e_init(EdgeLds<CAP, TG>& L) {
  for (int k = threadIdx.x; k < CAP; k += OTR_WAVE) {
    L.key[k] = kEmpty;
    L.lab[k] = kGInf;
  }
  if (threadIdx.x < TG) {
    L.tlab[threadIdx.x] = kGInf;
    L.tmap_node[threadIdx.x] = kEmpty;
    L.tmap_mask[threadIdx.x] = 0ull;
  }
  if (threadIdx.x == 0) {
    L.n_pend = 0;
    L.n_keys = 0;
    L.overflow = 0;
  }
  __syncthreads();
}

// One search (one wave) from root edge `root` (label 0 at dst(root) = rnode).  Lanes <
// n_tgt (<= TG) hold a target: node tv = src(ej), entry parts tpart / tpt, begin
// heading thb.  pd / pt: the relative bounds.  Returns false on overflow.  timed = false:
// route times are not tracked (pt unused).
template <int CAP, int TG>
__device__ bool edge_search(EdgeLds<CAP, TG>& L, const DevGraph& g, int md, bool active,
                            uint32_t root, uint32_t rnode, uint32_t pd, uint32_t pt, bool timed,
                            int n_tgt, uint32_t tv, uint32_t tpart, uint32_t tpt, uint32_t thb,
                            unsigned long long* settled, unsigned long long* relaxed) {
  constexpr int kMaxKeys = (CAP * 7) / 8;
  constexpr int WCAP = EdgeLds<CAP, TG>::WCAP;
  const int gl = (int)threadIdx.x;
  const uint32_t mode_bit = 1u << md;
  const uint32_t* adjt = g.adj_t + (size_t)md * g.adj_t_stride;
  const uint32_t* et = g.et(md);
  if (!timed) pt = 0xFFFFFFFFu;
  // targets
  const bool tgt = active && gl < n_tgt && gl < TG && tv != kEmpty;
  if (tgt) {
    L.tpart[gl] = tpart;
    L.tpt[gl] = timed ? tpt : 0u;
    L.thb[gl] = (uint16_t)thb;
    uint32_t h = tmap_home<TG>(tv);
    for (int probe = 0; probe < TG; ++probe) {
      const uint32_t k = atomicCAS(&L.tmap_node[h], kEmpty, tv);
      if (k == kEmpty || k == tv) {
        atomicOr(&L.tmap_mask[h], 1ull << gl);
        break;
      }
      h = (h + 1) & (TG - 1);
    }
  }
  if (active && gl == 0) {
    bool isnew;
    const int sl = e_insert(L, root, &isnew);
    L.node[sl] = rnode;
    L.mi[sl] = 0;
    L.lab[sl] = gpack(0u, 0u, 0u);
    L.key[sl] |= kInq;
    L.pend[0] = (uint16_t)sl;
  }
  __syncthreads();
  uint32_t my_settled = 0, my_relaxed = 0;
  uint32_t kmin = 0, dmin = 0;  // the smallest pending key / length
  bool done = !active;
  int npend = active ? 1 : 0;
  int nkeys = active ? 1 : 0;
  for (;;) {
    const int np = done ? 0 : npend;
    bool res = true;
    if (!done && tgt && np > 0) {
      // every later offer to the target has key >= kmin + tpart and length >= dmin + tpart
      const unsigned long long tl = L.tlab[gl];
      res = (tl != kGInf && (int64_t)g_k(tl) < (int64_t)kmin + (int64_t)tpart) ||
            (int64_t)dmin + (int64_t)tpart > (int64_t)pd;
    }
    done = done || __ballot(!res) == 0ull || np == 0;
    if (__builtin_amdgcn_readfirstlane((int)done)) break;
    uint32_t knext = 0xFFFFFFFFu, dnext = 0xFFFFFFFFu;
    int kept = 0, nw = 0;
    for (int base = 0; base < np; base += OTR_WAVE) {
      const int k = base + gl;
      const bool in = k < np;
      int sl = 0;
      uint32_t kk = 0, dd = 0, key = 0;
      unsigned long long lb = 0;
      bool take = false;
      if (in) {
        sl = L.pend[k];
        lb = L.lab[sl];
        key = L.key[sl];
        kk = g_k(lb);
        dd = g_d(lb);
        take = (uint64_t)kk < (uint64_t)kmin + in_gap8(L.mi[sl]);  // final (IN criterion)
      }
      take = take && nw + prefix_count(__ballot(take)) < WCAP;
      const unsigned long long mt = __ballot(take), mk = __ballot(in && !take);
      __syncthreads();
      if (take) {
        const int w = nw + prefix_count(mt);
        L.wslot[w] = (uint16_t)sl;
        L.wlab[w] = lb;
        L.key[sl] = (key & kNodeMask) | kRel;
      } else if (in) {
        L.pend[kept + prefix_count(mk)] = (uint16_t)sl;
        knext = kk < knext ? kk : knext;
        dnext = dd < dnext ? dd : dnext;
      }
      nw += __popcll(mt);
      kept += __popcll(mk);
      __syncthreads();
    }
    npend = kept;
    // relax: lane = (settled state, adjacency slot); slot-0 lanes also make the state's
    // target offers; slot 3 of a node with more than 4 out-edges walks the CSR tail
    bool tail = false;
    for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
      const int k = base + gl;
      int psl = -1;
      bool isnew = false;
      if (k < 4 * nw) {
        const int sl = L.wslot[k >> 2];
        const unsigned long long lb = L.wlab[k >> 2];
        const uint32_t v = L.node[sl], a = L.key[sl] & kNodeMask;
        const int slot = k & 3;
        if (slot == 0) ++my_settled;
        const uint32_t ha = (uint32_t)(uint16_t)g.edge_head[a].y;  // beside the adjacency loads
        const uint32_t tq = adjt[4 * (size_t)v + slot];
        const uint2 xe = g.adj_e[4 * (size_t)v + slot];
        const uint4 r = ld16(g.adj + 4 * (size_t)v + slot);
        if (slot == 0) e_target_offers(L, lb, ha, v, pd, pt);
        psl = e_relax(L, lb, ha, r.x & ~kAdjMore, r.y, timed ? tq : 0u, xe.x, xe.y & 0xFFFFu, pd, pt, mode_bit,
                      my_relaxed, knext, dnext, isnew);
        tail = tail || (slot == 3 && (r.x & kAdjMore));
      }
      nkeys += __popcll(__ballot(isnew));
      const unsigned long long mp = __ballot(psl >= 0);
      if (psl >= 0) {
        const int p = npend + prefix_count(mp);
        if (p < CAP) L.pend[p] = (uint16_t)psl;
        else L.overflow = 1;
      }
      npend += __popcll(mp);
    }
    if (__ballot(tail) != 0ull) {
      if (gl == 0) L.n_pend = npend;
      __syncthreads();
      for (int base = 0; base < 4 * nw; base += OTR_WAVE) {
        const int k = base + gl;
        if (k < 4 * nw && (k & 3) == 3) {
          const int sl = L.wslot[k >> 2];
          const unsigned long long lb = L.wlab[k >> 2];
          const uint32_t v = L.node[sl];
          const uint32_t ha = (uint32_t)(uint16_t)g.edge_head[L.key[sl] & kNodeMask].y;
          if (g.adj[4 * (size_t)v + 3].x & kAdjMore)
            for (uint32_t e = g.node_row[v] + 4; e < g.node_row[v + 1]; ++e) {
              const uint4 pk = ld16(g.edge_pack + e);
              const short2 hh = g.edge_head[e];
              bool isnew;
              const int psl = e_relax(L, lb, ha, pk.x | ((pk.z & 7u) << 28), pk.y, timed ? et[e] : 0u, e,
                                      (uint32_t)hh.x, pd, pt, mode_bit, my_relaxed, knext, dnext, isnew);
              if (isnew) atomicAdd(&L.n_keys, 1);
              if (psl >= 0) {
                const int p = atomicAdd(&L.n_pend, 1);
                if (p < CAP) L.pend[p] = (uint16_t)psl;
                else L.overflow = 1;
              }
            }
        }
      }
      __syncthreads();
      npend = L.n_pend;
      if (npend > CAP) npend = CAP;
    }
    __syncthreads();
    kmin = wave_min_u32(knext);
    dmin = wave_min_u32(dnext);
    const int keys = L.n_keys + nkeys;
    if (!done && (L.overflow || keys > kMaxKeys)) done = true;
    __syncthreads();
    if (done && active && gl == 0 && keys > kMaxKeys) L.overflow = 1;
  }
  if (settled) *settled += my_settled;
  if (relaxed) *relaxed += my_relaxed;
  __syncthreads();
  return !L.overflow;
}

// ------------------------------------------------------------------------------
// K6e: winner paths of turn-mode steps: the winner's edge-state search with the winner's
// target only, then a walk back: at each state a, the smallest-id in-edge p of src(a)
// whose label extended by (turn(p, a), a) is exactly a's label (oracle walk_path); the
// first hop from the target takes the smallest a whose offer is the target's label.  The
// lanes test the in-edges of one node in parallel.
// ------------------------------------------------------------------------------
// overflow_flag: the step's flag when the table overflows (the next tier)
template <int CAP>
__global__ __launch_bounds__(64) void k_paths_edge(DevGraph gr, PathArgs a, const int32_t* turn_tab,
                                                   const int64_t* step_list, const unsigned long long* list_count,
                                                   int32_t overflow_flag) {
  __shared__ EdgeLds<CAP, 32> L;
  __shared__ uint32_t s_rev[CAP];
  if (threadIdx.x == 0) L.turn_md = -1;
  const int lane = (int)threadIdx.x;
  XcdQueue q(a.queue, (int64_t)*list_count);  // (waves claim steps: no fixed-stride generations)
  for (int64_t w = q.next(); w < q.hi; w = q.next()) {
    const int64_t k = step_list[w];
    const int64_t s = a.steps[k];
    const int64_t sp = a.prev[s];
    const int wi = a.winner[sp], wj = a.winner[s];
    const uint32_t ei = a.cand_edge[sp * OTR_KMAX + wi], ej = a.cand_edge[s * OTR_KMAX + wj];
    const int md = a.mode[a.state_trace[s]] < OTR_MODES ? a.mode[a.state_trace[s]] : 0;
    const int32_t* turn = turn_tab + 181 * md;
    const uint32_t bmm = (uint32_t)bound_mm_of(a.bound[s]);
    const int32_t bt = a.bt[s];
    const uint4 cs = a.cprep[sp * OTR_KMAX + wi], ct = a.cprep[s * OTR_KMAX + wj];
    const uint32_t d0 = cs.w, t0 = bt >= 0 ? a.cprep_t[sp * OTR_KMAX + wi].y : 0u;
    const uint32_t tpt = bt >= 0 ? a.cprep_t[s * OTR_KMAX + wj].x : 0u;
    const uint32_t pd = bmm >= d0 ? bmm - d0 : 0u;
    const uint32_t pt = bt >= 0 && t0 <= (uint32_t)bt ? (uint32_t)bt - t0 : 0u;
    const uint32_t thb = (uint32_t)gr.edge_head[ej].x;
    e_init(L);
    e_turn_table(L, turn_tab, md);
    bool ok = edge_search<CAP, 32>(L, gr, md, true, ei, gr.edge_dst[ei], pd, pt, bt >= 0, 1, ct.y, ct.x,
                                   tpt, thb, nullptr, nullptr);
#ifdef OTR_FORCE_RETRY  // test build: OTR_FORCE_EDGE bit 3 / 4 fails every 384 / 2048-state winner path
    if (a.force_edge & (CAP < 2048 ? 8 : 16)) ok = false;
#endif
    const unsigned long long tl = L.tlab[0];
    int n = -1;
    if (ok && tl != kGInf) {
      // first hop: the smallest in-edge a of src(ej) whose offer is the target's label
      uint32_t cur = kEmpty;
      {
        const uint32_t v = ct.y;
        const uint32_t r0 = gr.rev_row[v], r1 = gr.rev_row[v + 1];
        uint32_t best = kEmpty;
        for (uint32_t r = r0 + lane; r < r1; r += OTR_WAVE) {
          const uint32_t x = gr.rev_edge[r];
          const int sx = e_find(L, x);
          if (sx < 0 || L.lab[sx] == kGInf) continue;
          const unsigned long long lx = L.lab[sx];
          EOffer o;
          o.c = g_c(lx) + (uint32_t)turn[turn_degree((int)gr.edge_head[x].y, (int)thb)];
          o.d = g_d(lx) + ct.x;
          o.k = o.d + o.c;
          o.t = (bt >= 0 ? g_t(lx) + tpt : 0u);
          if (e_feasible(o, pd, bt >= 0 ? pt : 0xFFFFFFFFu) && gpack(o.k, o.c, o.t) == tl && x < best) best = x;
        }
        cur = wave_min_u32(best);
      }
      // no in-edge offers the target's label: the next tier (never a zero-edge success;
      // cur == ei is the legitimate empty path, ej entered straight from ei)
      n = cur == kEmpty ? -1 : 0;
      while (n >= 0 && cur != kEmpty && cur != ei) {
        if (n >= CAP) {
          n = -1;
          break;
        }
        if (lane == 0) s_rev[n] = cur;
        ++n;
        const int sa = e_find(L, cur);
        const unsigned long long la = sa >= 0 ? L.lab[sa] : kGInf;
        const uint32_t v = gr.edge_src[cur];
        const uint32_t len = gr.len_mm[cur], tt = bt >= 0 ? gr.et(md)[cur] : 0u;
        const uint32_t hb = (uint32_t)gr.edge_head[cur].x;
        const uint32_t r0 = gr.rev_row[v], r1 = gr.rev_row[v + 1];
        uint32_t best = kEmpty;
        for (uint32_t r = r0 + lane; r < r1; r += OTR_WAVE) {
          const uint32_t p = gr.rev_edge[r];
          const int sx = e_find(L, p);
          if (sx < 0 || L.lab[sx] == kGInf) continue;
          const unsigned long long lp = L.lab[sx];
          EOffer o;
          o.c = g_c(lp) + (uint32_t)turn[turn_degree((int)gr.edge_head[p].y, (int)hb)];
          o.d = g_d(lp) + len;
          o.k = o.d + o.c;
          o.t = g_t(lp) + tt;
          if (la != kGInf && e_feasible(o, pd, bt >= 0 ? pt : 0xFFFFFFFFu) && gpack(o.k, o.c, o.t) == la && p < best)
            best = p;
        }
        cur = wave_min_u32(best);
        if (cur == kEmpty) n = -1;
      }
    }
    if (n < 0) {
      if (lane == 0) a.overflow_flag[k] = overflow_flag;  // the next tier
    } else {
      const int shard = (int)(blockIdx.x & (kShards - 1));
      const int64_t region = a.capacity / kShards;
      int64_t off = 0;
      if (lane == 0) off = (int64_t)atomicAdd(&a.cursor[shard], (unsigned long long)n);
      off = __shfl(off, 0);
      if (off + n > region) {
        if (lane == 0) *a.cap_flag = 1;
      } else {
        __syncthreads();
        off += (int64_t)shard * region;
        for (int q = lane; q < n; q += OTR_WAVE) a.path[off + q] = s_rev[n - 1 - q];
        if (lane == 0) {
          a.path_off[s] = off;
          a.path_len[s] = n;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace otr
