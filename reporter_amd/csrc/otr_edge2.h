// otr_edge2.h — K3e2: two edge-state route searches per wave (32 lanes each), the same
// search as otr_edge1.h's k_route_e1 (same semantics, same table layout per search, same
// helpers), for the many small searches of the turn-cost modes (tools/edge_stats.py on the
// C2 traces: 152 settled states and ~12 rounds per search, ~12 settled and ~25 pending
// examined per round — a 64-lane pass is mostly idle lanes).  Two searches share every
// wave instruction of the control path, the target resolution and the partition; the
// relax passes cover 8 settled states of each search per pass.
//
// Search g (0, 1) of a wave owns lanes [32 g, 32 g + 32) and table Ls[g]; every value that
// was wave-uniform in k_route_e1 is group-uniform here (Grp<2>: ballots masked to the
// group, prefix counts within it, DPP minima per 32 lanes, loop bounds as the maximum over
// both groups).  A group whose search is done idles through the other's remaining rounds.
#pragma once
#include "otr_edge1.h"

namespace otr {

template <int CAP>
__global__ __launch_bounds__(64) void k_route_e2(DevGraph gr, RouteArgs a, unsigned long long* counters) {
  using LT = E1Lds<CAP>;
  using GP = Grp<2>;
  constexpr int GL = GP::GL;  // 32 lanes per search
  constexpr int TG = LT::TG, TM = LT::TM, WCAP = LT::WCAP;
  static_assert(TG <= GL && TM <= GL, "targets and target-map slots are one lane each");
  constexpr int kMaxKeys = (CAP * 7) / 8;
  __shared__ LT Ls[2];
  const int g = GP::g(), gl = GP::gl();
  LT& L = Ls[g];
  if (gl == 0) L.turn_md = -1;
  const int64_t n = (int64_t)*a.list_count;
  const int64_t per = (n + 7) / 8;
  const int64_t lo = (int64_t)(blockIdx.x & 7) * per;
  const int64_t hi = lo + per < n ? lo + per : n;
  const int64_t stride = 2 * (int64_t)(gridDim.x >> 3);
  for (int64_t w0 = lo + 2 * (int64_t)(blockIdx.x >> 3); w0 < hi; w0 += stride) {
    const int64_t w = w0 + g;
    const bool valid = w < hi;
    const int64_t task = valid ? a.task_list[w] : a.task_list[w0];
    const uint4 r0 = a.rec[3 * task], r1 = a.rec[3 * task + 1], r2 = a.rec[3 * task + 2];
    const int64_t s = r0.x, sp = r0.y;
    const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
    const int i = __ffsll((long long)mask) - 1;
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
    uint32_t ej = 0, tv = kEmpty, tpart = 0, tpt = 0;
    double pj = 0;
    bool needed = false;
    if (valid && gl < Kb) {
      ej = a.cand_edge[s * OTR_KMAX + gl];
      pj = a.cand_p[s * OTR_KMAX + gl];
      const uint4 cq = a.cprep[s * OTR_KMAX + gl];
      tpart = cq.x;
      tpt = timed ? a.cprep_t[s * OTR_KMAX + gl].x : 0u;
      needed = !(ej == ei && pj >= pi);
      if (needed) tv = cq.y;
    }
    const bool root_ok = d0 <= bmm && (!timed || t0 <= (uint32_t)bt);
    const bool search = valid && Kb <= TG && !forced && root_ok && GP::mine(__ballot(needed)) != 0ull;
    const uint32_t pd = bmm >= d0 ? bmm - d0 : 0u;
    const uint32_t pt = !timed ? 0xFFFFFFFFu : (t0 <= (uint32_t)bt ? (uint32_t)bt - t0 : 0u);
    // ---- reset: keys, targets, the target map and its bloom (each group its own table)
    for (int k = gl; k < CAP; k += GL) L.key[k] = kEmpty;
    if (gl < TG) L.tlab[gl] = kGInf;
    if (gl < TM) {
      L.tm_node[gl] = kEmpty;
      L.tm_mask[gl] = 0u;
    }
    if (gl == 0) {
      L.overflow = 0;
      L.bloom = 0ull;
    }
    // the group's turn table (both groups usually hold the same mode: consecutive tasks)
    {
      const bool load = L.turn_md != md;
      __syncthreads();
      uint32_t m = 0xFFFFFFFFu;
      if (load) {
        for (int k = gl; k < 181; k += GL) {
          const int32_t t = a.turn[181 * md + k];
          L.turn[k] = t;
          m = (uint32_t)t < m ? (uint32_t)t : m;
        }
      }
      m = GP::min_u32(m);
      if (load && gl == 0) {
        L.turn_md = md;
        L.tmin = m;
      }
      __syncthreads();
    }
    const bool tgt = search && gl < Kb && tv != kEmpty;
    if (tgt) {
      L.tpart[gl] = tpart;
      L.tpt[gl] = tpt;
      L.thb[gl] = (uint16_t)gr.edge_head[ej].x;
      uint32_t h = tm_slot(tv);
#pragma unroll 1
      for (int probe = 0; probe < TM; ++probe) {
        const uint32_t k = atomicCAS(&L.tm_node[h], kEmpty, tv);
        if (k == kEmpty || k == tv) {
          atomicOr(&L.tm_mask[h], 1u << gl);
          break;
        }
        h = (h + 1) & (TM - 1);
      }
      atomicOr(&L.bloom, 1ull << tm_home(tv));
    }
    __syncthreads();
    const unsigned long long bloom = L.bloom;
    bool ok = true;
    uint32_t my_settled = 0, my_relaxed = 0;
    if (search && gl == 0) {
      bool isnew = false;
      const int sl = e1_insert(L, ei, isnew);
      L.node[sl] = gr.edge_dst[ei];
      L.hbk[sl] = (uint16_t)heading_back((int)(uint16_t)gr.edge_head[ei].y);
      L.mi[sl] = 0;
      L.lab[sl] = gpack(0u, 0u, 0u);
      L.key[sl] = ei | kInq;
      L.pend[0] = (typename LT::Idx)sl;
    }
    __syncthreads();
    const uint4* er = gr.erec + (size_t)md * gr.erec_stride;
    const uint32_t mode_bit = 1u << md;
    const uint32_t tmin = L.tmin;
    uint32_t kmin = 0, dmin = 0;
    int npend = search ? 1 : 0, nkeys = 1;
    bool active = search;
#pragma unroll 1
    for (;;) {
      // ---- targets (per group): done when every needed target is final or unreachable
      bool res = true;
      if (tgt) {
        const unsigned long long tl = L.tlab[gl];
        res = (tl != kGInf && (uint64_t)g_k(tl) < (uint64_t)kmin + tpart + tmin) || (uint64_t)dmin + tpart > (uint64_t)pd;
      }
      active = active && GP::mine(__ballot(!res)) != 0ull && npend > 0;
      if (__ballot(active) == 0ull) break;
      if (!active) npend = 0;  // (an idle group takes no part in the passes below)
      // ---- partition
      uint32_t knext = 0xFFFFFFFFu, dnext = 0xFFFFFFFFu;
      int kept = 0, nw = 0;
      const int pend_max = GP::umax(npend);
#pragma unroll 1
      for (int base = 0; base < pend_max; base += GL) {
        const int k = base + gl;
        const bool in = k < npend;
        int sl = 0;
        unsigned long long lb = 0;
        uint32_t nd = 0, hk = 0;
        bool take = false;
        if (in) {
          sl = L.pend[k];
          lb = L.lab[sl];
          nd = L.node[sl];
          hk = L.hbk[sl];
          take = (uint64_t)g_k(lb) < (uint64_t)kmin + in_gap8(L.mi[sl]) + tmin;
        }
        take = take && nw + GP::prefix(__ballot(take)) < WCAP;
        const bool keep = in && !take;
        const unsigned long long mt = __ballot(take), mk = __ballot(keep);
        __syncthreads();
        if (take) {
          const int wq = nw + GP::prefix(mt);
          L.wlab[wq] = lb;
          L.wnode[wq] = nd;
          L.whbk[wq] = (uint16_t)hk;
        } else if (keep) {
          L.pend[kept + GP::prefix(mk)] = (typename LT::Idx)sl;
          knext = g_k(lb) < knext ? g_k(lb) : knext;
          dnext = g_d(lb) < dnext ? g_d(lb) : dnext;
        }
        nw += GP::count(mt);
        kept += GP::count(mk);
        __syncthreads();
      }
      npend = kept;
      // ---- relax: lane = (settled state, adjacency slot), 8 states of each group per pass
      bool tail = false;
      const int relax_max = GP::umax(4 * nw);
#pragma unroll 1
      for (int base = 0; base < relax_max; base += GL) {
        const int k = base + gl;
        int psl = -1;
        bool isnew = false;
        if (k < 4 * nw) {
          const unsigned long long lb = L.wlab[k >> 2];
          const uint32_t v = L.wnode[k >> 2], hbk = L.whbk[k >> 2];
          const int slot = k & 3;
          uint4 r = er[4 * (size_t)v + slot];
          if (slot == 0) {
            ++my_settled;
            if ((bloom >> tm_home(v)) & 1ull) e1_target_offers(L, lb, hbk, v, pd, pt);
          }
          asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w));  // (one 16-B load, not split)
          psl = e1_relax(L, lb, hbk, r.x & ~kAdjMore, r.y, timed ? er_t(r) : 0u, er_edge(r), er_hb(r), er_he(r), pd,
                         pt, mode_bit, my_relaxed, knext, dnext, isnew);
          tail = tail || (slot == 3 && (r.x & kAdjMore));
        }
        nkeys += GP::count(__ballot(isnew));
        const unsigned long long mp = __ballot(psl >= 0);
        if (psl >= 0) L.pend[npend + GP::prefix(mp)] = (typename LT::Idx)psl;
        npend += GP::count(mp);
      }
      if (__ballot(tail) != 0ull) {  // nodes with more than four out-edges: the CSR tail
        if (gl == 0) {
          L.n_pend = npend;
          L.n_keys = 0;
        }
        __syncthreads();
#pragma unroll 1
        for (int base = 0; base < relax_max; base += GL) {
          const int k = base + gl;
          if (k < 4 * nw && (k & 3) == 3) {
            const unsigned long long lb = L.wlab[k >> 2];
            const uint32_t v = L.wnode[k >> 2], hbk = L.whbk[k >> 2];
            if (er[4 * (size_t)v + 3].x & kAdjMore) {
              const uint32_t* et = gr.et(md);
#pragma unroll 1
              for (uint32_t e = gr.node_row[v] + 4; e < gr.node_row[v + 1]; ++e) {
                const uint4 pk = ld16(gr.edge_pack + e);
                const short2 hh = gr.edge_head[e];
                bool nw2 = false;
                const int p2 = e1_relax(L, lb, hbk, pk.x | ((pk.z & 7u) << 28), pk.y, timed ? et[e] : 0u, e,
                                        (uint32_t)(uint16_t)hh.x, (uint32_t)(uint16_t)hh.y, pd, pt, mode_bit,
                                        my_relaxed, knext, dnext, nw2);
                if (nw2) atomicAdd(&L.n_keys, 1);
                if (p2 >= 0) L.pend[atomicAdd(&L.n_pend, 1)] = (typename LT::Idx)p2;
              }
            }
          }
        }
        __syncthreads();
        npend = L.n_pend;
        nkeys += L.n_keys;
      }
      __syncthreads();
      kmin = GP::min_u32(knext);
      dmin = GP::min_u32(dnext);
      if (active && (L.overflow || nkeys > kMaxKeys)) {
        ok = false;
        active = false;
        npend = 0;
      }
    }
#ifdef OTR_FORCE_RETRY  // test build: OTR_FORCE_EDGE bit 0 fails every first-tier search
    if (a.force_edge & 1) ok = false;
#endif
    ok = ok && Kb <= TG;
    if (valid && ok) {
      uint32_t* trow = a.trans + (int64_t)(((uint64_t)r2.w << 32) | r2.z);
      if (gl < Kb) {
        int64_t rr = -1, rt = 0;
        uint32_t rc = 0;
        if (forced) {
          rr = -1;
        } else if (ej == ei && pj >= pi) {
          const uint2 li = a.clen[sp * OTR_KMAX + i];
          rr = part_mm(pj - pi, li.x);
          if (timed) rt = part_mm(pj - pi, li.y);
        } else if (search) {
          const unsigned long long tl = L.tlab[gl];
          if (tl != kGInf) {
            rr = (int64_t)d0 + g_d(tl);
            rt = (int64_t)t0 + g_t(tl);
            rc = g_c(tl);
          }
        }
        const bool vld = rr >= 0 && rr <= (int64_t)bmm && (!timed || rt <= (int64_t)bt);
        trow[(int64_t)i * Kb + gl] = vld ? (uint32_t)rr : kNoRoute;
        a.trans_tc[trow - a.trans + (int64_t)i * Kb + gl] = vld ? rc : 0u;
      }
    } else if (valid && gl == 0) {
      a.overflow_flag[task] = 6;  // the next table: 512 states (k_route_e1)
    }
    if (counters) {
      const bool lead = valid && ok && gl == 0;
      const uint32_t st = wave_sum_u32(valid && ok ? my_settled : 0u), rl = wave_sum_u32(valid && ok ? my_relaxed : 0u);
      const uint32_t kb = wave_sum_u32(lead && search ? (uint32_t)Kb : 0u), ns = wave_sum_u32(lead && search ? 1u : 0u);
      if (threadIdx.x == 0) {
        const int sh = cshard();
        atomicAdd(&counters[3 * kCShards + sh], (unsigned long long)st);
        atomicAdd(&counters[4 * kCShards + sh], (unsigned long long)rl);
        atomicAdd(&counters[5 * kCShards + sh], (unsigned long long)kb);
        atomicAdd(&counters[6 * kCShards + sh], (unsigned long long)ns);
      }
    }
    __syncthreads();
  }
}

}  // namespace otr
