// otr_general.h — K3g/K6g: the bounded route search with its labels in HBM.
//
// The LDS search (otr_kernels.h, search_run) is the fast path: node labels packed in
// 32 bits (length mm << sh | time 0.1 s), at most 4096 slots per search.  Everything
// it cannot hold runs here, with no capacity limit below the slab size:
//   * turn costs (turn_penalty_factor > 0): the search is over EDGE states, because
//     the turn cost at a node depends on the edge that entered it;
//   * steps whose bounds do not fit the 32-bit packing;
//   * searches that outgrew the largest LDS table.
// Labels are 64-bit words key << 38 | (kTcCap - turn) << 17 | time: key = length + turn
// cost (mm), so one atomicMin keeps the lexicographic minimum of (key, length, time), the
// oracle's order (oracle.c rkey).  Labels are relative to the search root; relaxations
// beyond the task's relative bounds (length pd, time pt, turn cost kTcCap) are pruned.
//
// One workgroup (kGenThreads) per task, persistent over a device task list whose length
// is read on the device (no host round trip).  Each workgroup owns a slab: an open-
// addressing hash table {state | relaxed bit, label, round stamp} plus two frontier lists
// and the list of claimed slots (reset after every search, so a slab is never cleared as
// a whole).  Each round expands the frontier states whose labels are final by the IN
// criterion of the LDS search (key < smallest frontier key + the state's shortest
// in-edge: minin(node) in node mode, the state's own edge in edge mode) and carries the
// others to the next round, i.e. the label-setting search of the oracle, in parallel.
#pragma once
#include "otr_kernels.h"

namespace otr {

constexpr int kGenThreads = 256;
constexpr unsigned long long kGInf = 0xFFFFFFFFFFFFFFFFull;
constexpr uint32_t kGRel = 0x80000000u;  // key bit: the state has been expanded before
constexpr uint32_t kGIdMask = 0x7FFFFFFFu;

__host__ __device__ inline unsigned long long gpack(uint64_t k, uint64_t c, uint64_t t) {
  return (k << 38) | ((uint64_t)(kTcCap - c) << 17) | t;
}
__host__ __device__ inline uint32_t g_k(unsigned long long w) { return (uint32_t)(w >> 38); }
__host__ __device__ inline uint32_t g_c(unsigned long long w) { return kTcCap - (uint32_t)((w >> 17) & 0x1FFFFFull); }
__host__ __device__ inline uint32_t g_t(unsigned long long w) { return (uint32_t)(w & 0x1FFFFull); }
__host__ __device__ inline uint32_t g_d(unsigned long long w) { return g_k(w) - g_c(w); }

struct GSlabs {
  uint32_t* key;                // [n][cap] state | kGRel, kEmpty
  unsigned long long* lab;      // [n][cap]
  uint32_t* qmark;              // [n][cap] round + 1 when queued for that round
  uint32_t* fr;                 // [n][2][cap] frontier slot lists
  uint32_t* touched;            // [n][cap] claimed slots
  uint32_t cap;                 // power of two
  uint32_t n;                   // slabs (= grid size)
};

struct GenArgs {
  // task source: route tasks (mode 0) or winner paths (mode 1)
  int mode;
  const int64_t* list;          // indices of the tasks / steps to run
  const unsigned long long* list_count;
  // step data
  const int64_t* prev;
  const double* g;
  const int32_t* bt;            // time bound per state (0.1 s), -1 none
  const double* bound;
  const int32_t* cand_count;
  const uint32_t* cand_edge;
  const double* cand_p;
  const uint4* cprep;           // per candidate {part(p), src(e), minin(src), part(1 - p)}
  const uint2* cprep_t;         // per candidate {part_t(p), part_t(1 - p)}
  const int32_t* state_trace;
  const uint8_t* mode_of_trace;
  uint32_t turn_modes;          // bit m: mode m has turn costs
  const int32_t* turn;          // [OTR_MODES][181] turn cost table, mm
  // route mode
  const uint4* rec;                     // per route task: k_tasks' record (state s, source mask)
  const int64_t* trans_off;
  uint32_t* trans;
  uint32_t* trans_tc;
  // path mode
  const int64_t* steps;
  const int32_t* winner;
  int64_t* path_off;
  int32_t* path_len;
  uint32_t* path;
  unsigned long long* cursor;   // [kShards] bump cursors
  int64_t capacity;
  int32_t* cap_flag;
  // outcome per task / step: 0 done, 1 slab overflow (retry on a larger slab)
  int32_t* flag;
  unsigned long long* n_overflow;  // tasks that overflowed this slab size
  unsigned long long* counters;
};

__device__ inline unsigned long long ld_u64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t ld_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// slot of state e in the slab, claiming an empty one when absent (*claimed); -1 when full
__device__ inline int g_claim(uint32_t* key, uint32_t cap, uint32_t e, bool* claimed) {
  uint32_t h = hmix(e) & (cap - 1u);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    const uint32_t k = atomicCAS(&key[h], kEmpty, e);
    if (k == kEmpty) {
      *claimed = true;
      return (int)h;
    }
    if ((k & kGIdMask) == e) {
      *claimed = false;
      return (int)h;
    }
    h = (h + 1u) & (cap - 1u);
  }
  return -1;
}
__device__ inline int g_find(const uint32_t* key, uint32_t cap, uint32_t e) {
  uint32_t h = hmix(e) & (cap - 1u);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    const uint32_t k = ld_u32(&key[h]);
    if (k == kEmpty) return -1;
    if ((k & kGIdMask) == e) return (int)h;
    h = (h + 1u) & (cap - 1u);
  }
  return -1;
}

struct GTask {
  int64_t s, sp;
  uint32_t root;        // node (node mode) or edge (edge mode)
  bool edge_mode, time_on;
  uint32_t bmm;         // the step's length bound (mm)
  int32_t bt;           // the step's time bound (0.1 s), -1 none
  uint32_t pd, pt;      // the relative pruning bounds of this search (bound - exit part)
  int mode;
  const uint32_t* et;   // the mode's edge times
  const int32_t* turn;  // the mode's turn table
  uint32_t mode_bit;
};

// the relaxation of state a (label L) through edge b: relative (key, length, time, turn);
// a == kEmpty: no turn (node mode)
struct GOffer {
  uint32_t k, d, t, c;
};
__device__ inline GOffer g_offer(const DevGraph& G, const GTask& T, uint32_t a, unsigned long long L, uint32_t b) {
  GOffer o;
  const uint32_t len = G.len_mm[b];
  o.c = g_c(L);
  if (T.edge_mode && a != kEmpty) o.c += (uint32_t)T.turn[turn_degree(G.edge_head[a].y, G.edge_head[b].x)];
  o.d = g_d(L) + len;
  o.k = o.d + o.c;
  o.t = T.time_on ? g_t(L) + T.et[b] : 0u;
  return o;
}
__device__ inline bool g_feasible(const GTask& T, const GOffer& o) {
  return o.d <= T.pd && (!T.time_on || o.t <= T.pt) && o.c <= kTcCap;
}

// block-wide minimum of a u32 (kGenThreads threads)
__device__ inline uint32_t g_block_min(uint32_t v, uint32_t* s_red) {
  for (int off = OTR_WAVE / 2; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)v, off);
    v = o < v ? o : v;
  }
  __syncthreads();
  if (lane_id() == 0) s_red[threadIdx.x / OTR_WAVE] = v;
  __syncthreads();
  uint32_t m = s_red[0];
  for (int w = 1; w < kGenThreads / OTR_WAVE; ++w) m = s_red[w] < m ? s_red[w] : m;
  return m;
}

struct GShared {
  uint32_t n[2], touched, ovf, red[kGenThreads / OTR_WAVE];
};

// Workgroup-wide bounded search of one task in the slab (see the file comment).  Returns
// false (workgroup-uniform) on slab overflow.
__device__ bool g_search(const DevGraph& G, const GTask& T, uint32_t* key, unsigned long long* lab, uint32_t* qmark,
                         uint32_t* fr, uint32_t* touched, uint32_t cap, GShared* sh, unsigned long long* work) {
  const int tid = threadIdx.x;
  const uint32_t maxk = cap - cap / 8u;
  unsigned long long my_relaxed = 0;
  if (tid == 0) {
    sh->ovf = 0;
    sh->n[0] = 0;
    sh->n[1] = 0;
    // the root state, label 0, queued for round 0
    bool claimed = false;
    const int sl = g_claim(key, cap, T.root, &claimed);
    if (sl >= 0) {
      if (claimed) {
        const uint32_t k = sh->touched++;
        if (k < cap) touched[k] = (uint32_t)sl;
      }
      lab[sl] = gpack(0u, 0u, 0u);
      qmark[sl] = 1u;
      fr[0] = (uint32_t)sl;
      sh->n[0] = 1;
    } else {
      sh->ovf = 1;
    }
  }
  __threadfence_block();
  __syncthreads();
  // relax the final state a (label L) through edge b, queueing for round nr
  auto relax = [&](uint32_t a, unsigned long long L, uint32_t b, uint32_t nr, int nxt) {
    if (!(G.edge_attr[b] & T.mode_bit)) return;
    ++my_relaxed;
    const GOffer o = g_offer(G, T, T.edge_mode ? a : kEmpty, L, b);
    const uint32_t sid = T.edge_mode ? b : G.edge_dst[b];
    if (!g_feasible(T, o)) return;  // pruned (label-setting semantics)
    const unsigned long long w = gpack(o.k, o.c, o.t);
    bool claimed = false;
    const int sl = g_claim(key, cap, sid, &claimed);
    if (sl < 0) {
      sh->ovf = 1;
      return;
    }
    if (claimed) {
      const uint32_t k = atomicAdd(&sh->touched, 1u);
      if (k < cap) touched[k] = (uint32_t)sl;
      if (k >= maxk) sh->ovf = 1;
    }
    const unsigned long long old = atomicMin(&lab[sl], w);
    if (w < old && atomicExch(&qmark[sl], nr + 1u) != nr + 1u) {
      const uint32_t p = atomicAdd(&sh->n[nxt], 1u);
      if (p < cap) fr[(size_t)nxt * cap + p] = (uint32_t)sl;
      else sh->ovf = 1;
    }
  };
  uint32_t round = 0;
  int cur = 0;
  unsigned long long expanded = 0;  // states expanded (uniform): the search's "settled" count
  for (;;) {
    const uint32_t n = sh->n[cur];
    if (n == 0 || sh->ovf) break;
    const int nxt = cur ^ 1;
    __syncthreads();
    if (tid == 0) sh->n[nxt] = 0;
    const uint32_t nn = n < cap ? n : cap;
    // the frontier's smallest key: with each state's shortest in-edge it decides finality
    uint32_t kmin;
    {
      uint32_t m = 0xFFFFFFFFu;
      for (uint32_t i = tid; i < nn; i += kGenThreads) {
        const uint32_t sl = ld_u32(&fr[(size_t)cur * cap + i]);
        const uint32_t k = g_k(ld_u64(&lab[sl]));
        m = k < m ? k : m;
      }
      kmin = g_block_min(m, sh->red);
    }
    __syncthreads();
    for (uint32_t i = tid; i < nn; i += kGenThreads) {
      const uint32_t sl = ld_u32(&fr[(size_t)cur * cap + i]);
      const unsigned long long L = ld_u64(&lab[sl]);
      const uint32_t id = ld_u32(&key[sl]) & kGIdMask;
      const uint32_t mi = T.edge_mode ? G.len_mm[id] : G.node_minin[id];
      const uint32_t gap = id == T.root ? 1u : (mi ? mi : 1u);
      if ((uint64_t)g_k(L) >= (uint64_t)kmin + gap) {  // not final yet: carried to the next round
        if (atomicExch(&qmark[sl], round + 2u) != round + 2u) {
          const uint32_t p = atomicAdd(&sh->n[nxt], 1u);
          if (p < cap) fr[(size_t)nxt * cap + p] = sl;
          else sh->ovf = 1;
        }
        continue;
      }
      const uint32_t was = atomicOr(&key[sl], kGRel);
      const uint32_t a = was & kGIdMask;
      ++expanded;
      const uint32_t v = T.edge_mode ? G.edge_dst[a] : a;
      for (uint32_t e = G.node_row[v]; e < G.node_row[v + 1]; ++e) relax(a, L, e, round + 1u, nxt);
    }
    __threadfence_block();
    __syncthreads();
    ++round;
    cur = nxt;
  }
  __syncthreads();
  if (work) {  // this tier's counter bank (kinds 3 settled, 4 relaxed)
    const int shd = cshard();
    atomicAdd(&work[4 * kCShards + shd], my_relaxed);
    atomicAdd(&work[3 * kCShards + shd], expanded);
  }
  const bool ok = sh->ovf == 0;
  __syncthreads();
  return ok;
}

// The route to target (ej, pj): node mode the label of v = src(ej) (relative; the root
// node has 0); edge mode the lexicographic minimum over the labelled in-edges a of v of
// the offer with the turn (a, ej) — smallest a among equals (*via).  The target's entry
// part (tpart mm, tpt 0.1 s) is included and the offer must keep the relative bounds
// (oracle target_key).  Returns false when no feasible offer exists.
__device__ inline bool g_target(const DevGraph& G, const GTask& T, const uint32_t* key, const unsigned long long* lab,
                                uint32_t cap, uint32_t ej, uint32_t tpart, uint32_t tpt, GOffer* out, uint32_t* via) {
  const uint32_t v = G.edge_src[ej];
  if (!T.edge_mode) {
    const int sl = g_find(key, cap, v);
    if (sl < 0) return false;
    const unsigned long long L = ld_u64(&lab[sl]);
    if (L == kGInf) return false;
    GOffer o;
    o.c = 0;
    o.d = g_d(L) + tpart;
    o.k = o.d;
    o.t = T.time_on ? g_t(L) + tpt : 0u;
    *out = o;
    *via = kEmpty;
    return g_feasible(T, o);
  }
  bool found = false;
  unsigned long long best = kGInf;
  uint32_t bid = kEmpty;
  GOffer bo{};
  for (uint32_t r = G.rev_row[v]; r < G.rev_row[v + 1]; ++r) {
    const uint32_t a = G.rev_edge[r];
    const int sl = g_find(key, cap, a);
    if (sl < 0) continue;
    const unsigned long long L = ld_u64(&lab[sl]);
    if (L == kGInf) continue;
    GOffer o;
    o.c = g_c(L) + (uint32_t)T.turn[turn_degree(G.edge_head[a].y, G.edge_head[ej].x)];
    o.d = g_d(L) + tpart;
    o.k = o.d + o.c;
    o.t = T.time_on ? g_t(L) + tpt : 0u;
    if (!g_feasible(T, o)) continue;
    const unsigned long long w = gpack(o.k, o.c, o.t);
    if (!found || w < best || (w == best && a < bid)) {
      best = w;
      bid = a;
      bo = o;
      found = true;
    }
  }
  *out = bo;
  *via = bid;
  return found;
}

// the task of source candidate ei (node mode: the group's common root dst(ei)); the
// relative bounds use the exit part d0 (node mode: the group's smallest) and exit time t0
__device__ inline GTask g_task(const DevGraph& G, const GenArgs& a, int64_t s, int64_t sp, uint32_t ei, uint32_t d0,
                               uint32_t t0) {
  GTask T;
  T.s = s;
  T.sp = sp;
  const int tr = a.state_trace[s];
  const int md = a.mode_of_trace[tr] < OTR_MODES ? a.mode_of_trace[tr] : 0;
  T.mode = md;
  T.mode_bit = 1u << md;
  T.edge_mode = (a.turn_modes >> md) & 1u;
  T.bt = a.bt[s];
  T.time_on = T.bt >= 0;
  T.bmm = (uint32_t)bound_mm_of(a.bound[s]);
  T.root = T.edge_mode ? ei : G.edge_dst[ei];
  T.et = G.et(md);
  T.turn = a.turn + 181 * md;
  T.pd = T.bmm >= d0 ? T.bmm - d0 : 0u;
  T.pt = !T.time_on ? 0xFFFFFFFFu : (t0 <= (uint32_t)T.bt ? (uint32_t)T.bt - t0 : 0u);
  return T;
}

// reset the claimed slots of a slab (workgroup-wide), ready for the next search
__device__ inline void g_reset(uint32_t* key, unsigned long long* lab, uint32_t* qmark, const uint32_t* touched,
                               GShared* sh, uint32_t cap) {
  __syncthreads();
  const uint32_t n = sh->touched < cap ? sh->touched : cap;
  for (uint32_t i = threadIdx.x; i < n; i += kGenThreads) {
    const uint32_t sl = touched[i];
    key[sl] = kEmpty;
    lab[sl] = kGInf;
    qmark[sl] = 0u;
  }
  __threadfence_block();
  __syncthreads();
  if (threadIdx.x == 0) sh->touched = 0;
  __syncthreads();
}

// a feasible root: the sources' exit parts keep both bounds
__device__ inline bool g_root_ok(const GTask& T, uint32_t d0, uint32_t t0) {
  return d0 <= T.bmm && (!T.time_on || t0 <= (uint32_t)T.bt);
}

__global__ __launch_bounds__(kGenThreads) void k_general(DevGraph G, GenArgs a, GSlabs S) {
  __shared__ GShared sh;
  __shared__ uint32_t s_path[1];
  const uint32_t cap = S.cap;
  uint32_t* key = S.key + (size_t)blockIdx.x * cap;
  unsigned long long* lab = S.lab + (size_t)blockIdx.x * cap;
  uint32_t* qmark = S.qmark + (size_t)blockIdx.x * cap;
  uint32_t* fr = S.fr + (size_t)blockIdx.x * 2 * cap;
  uint32_t* touched = S.touched + (size_t)blockIdx.x * cap;
  const int64_t count = (int64_t)*a.list_count;
  const int tid = threadIdx.x;
  if (tid == 0) sh.touched = 0;  // the slab is clean (cleared at allocation, reset after every search)
  __syncthreads();
  // one search, leaving its labels in the slab; false on slab overflow
  auto run = [&](const GTask& T, unsigned long long* work) -> bool {
    return g_search(G, T, key, lab, qmark, fr, touched, cap, &sh, work);
  };
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    const int64_t item = a.list[k];
    if (a.mode == 0) {
      // ---- route task: transitions of every source of the task.  Node mode: one search
      // from the common root per group of sources with equal exit times (the time bound
      // prunes each group at its own bt - t0; the length bound at B - the group's smallest
      // exit part); turn costs: the task has one source edge
      const uint4 r0 = a.rec[3 * item], r1 = a.rec[3 * item + 1];
      const int64_t s = r0.x;
      const unsigned long long mask = ((unsigned long long)r1.w << 32) | r1.z;
      const int64_t sp = a.prev[s];
      const int Kb = a.cand_count[s];
      bool ok = true;
      for (unsigned long long todo = mask; todo && ok;) {
        const int i0 = __ffsll((long long)todo) - 1;
        const bool timed = a.bt[s] >= 0;
        const uint32_t t0 = timed ? a.cprep_t[sp * OTR_KMAX + i0].y : 0u;
        unsigned long long grp = 0;
        uint32_t d0 = 0xFFFFFFFFu;
        for (unsigned long long m = todo; m; m &= m - 1) {
          const int i = __ffsll((long long)m) - 1;
          if (timed && a.cprep_t[sp * OTR_KMAX + i].y != t0) continue;
          grp |= 1ull << i;
          const uint32_t w = a.cprep[sp * OTR_KMAX + i].w;
          d0 = w < d0 ? w : d0;
        }
        todo &= ~grp;
        const GTask T = g_task(G, a, s, sp, a.cand_edge[sp * OTR_KMAX + i0], d0, t0);
        bool need = false;
        for (int j = 0; j < Kb && !need; ++j) {
          const uint32_t ej = a.cand_edge[s * OTR_KMAX + j];
          const double pj = a.cand_p[s * OTR_KMAX + j];
          for (unsigned long long m = grp; m; m &= m - 1) {
            const int i = __ffsll((long long)m) - 1;
            if (!(ej == a.cand_edge[sp * OTR_KMAX + i] && pj >= a.cand_p[sp * OTR_KMAX + i])) need = true;
          }
        }
        bool searched = false;
        if (need && g_root_ok(T, d0, t0)) {
          ok = run(T, a.counters);
          searched = true;
        }
        if (!ok) break;
        if (a.counters && tid == 0 && searched) {  // kinds 5 transition entries, 6 searches
          const int shd = cshard();
          atomicAdd(&a.counters[5 * kCShards + shd], (unsigned long long)Kb * (unsigned long long)__popcll(grp));
          atomicAdd(&a.counters[6 * kCShards + shd], 1ull);
        }
        uint32_t* trow = a.trans + a.trans_off[s];
        uint32_t* crow = a.trans_tc + a.trans_off[s];
        for (int j = tid; j < Kb; j += kGenThreads) {
          const uint32_t ej = a.cand_edge[s * OTR_KMAX + j];
          const double pj = a.cand_p[s * OTR_KMAX + j];
          const uint4 cj = a.cprep[s * OTR_KMAX + j];
          const uint2 cjt = a.cprep_t[s * OTR_KMAX + j];
          GOffer o;
          uint32_t via;
          const bool reached = searched && g_target(G, T, key, lab, cap, ej, cj.x, cjt.x, &o, &via);
          for (unsigned long long m = grp; m; m &= m - 1) {
            const int i = __ffsll((long long)m) - 1;
            const uint32_t ei = a.cand_edge[sp * OTR_KMAX + i];
            const double pi = a.cand_p[sp * OTR_KMAX + i];
            int64_t rd = -1, rt = 0;
            uint32_t rc = 0;
            if (ej == ei && pj >= pi) {
              rd = part_mm(pj - pi, G.len_mm[ei]);
              rt = T.time_on ? part_mm(pj - pi, T.et[ei]) : 0;
            } else if (reached) {
              rd = (int64_t)a.cprep[sp * OTR_KMAX + i].w + o.d;
              rt = T.time_on ? (int64_t)t0 + o.t : 0;
              rc = o.c;
            }
            const bool valid = rd >= 0 && rd <= (int64_t)T.bmm && (!T.time_on || rt <= (int64_t)T.bt);
            trow[(int64_t)i * Kb + j] = valid ? (uint32_t)rd : kNoRoute;
            if (T.edge_mode) crow[(int64_t)i * Kb + j] = valid ? rc : 0u;  // allocated for turn modes only
          }
        }
        g_reset(key, lab, qmark, touched, &sh, cap);
      }
      if (ok) {
        if (tid == 0) a.flag[item] = 0;
      } else if (tid == 0) {
        a.flag[item] = 1;
        atomicAdd(a.n_overflow, 1ull);
      }
    } else {
      // ---- winner path of a step: search from the winner, then walk back
      const int64_t s = a.steps[item];
      const int64_t sp = a.prev[s];
      const int wi = a.winner[sp], wj = a.winner[s];
      const uint32_t ei = a.cand_edge[sp * OTR_KMAX + wi], ej = a.cand_edge[s * OTR_KMAX + wj];
      const double pj = a.cand_p[s * OTR_KMAX + wj];
      const uint4 ci = a.cprep[sp * OTR_KMAX + wi], cj = a.cprep[s * OTR_KMAX + wj];
      const GTask T = g_task(G, a, s, sp, ei, ci.w, a.cprep_t[sp * OTR_KMAX + wi].y);
      const bool ok = run(T, nullptr);
      if (!ok) {
        if (tid == 0) {
          a.flag[item] = 1;
          atomicAdd(a.n_overflow, 1ull);
        }
      } else {
        // one thread walks the predecessor states (rare path: dependent loads are fine);
        // the reversed edge list goes to frontier list 0 (free after the search)
        uint32_t* rev = fr;
        if (tid == 0) {
          int n = 0;
          bool good = true;
          if (!T.edge_mode) {
            // node labels: at v, the smallest-id in-edge whose tail's label plus the edge is
            // exactly v's label (oracle walk_path)
            uint32_t v = G.edge_src[ej];
            while (v != T.root) {
              const int sv = g_find(key, cap, v);
              const unsigned long long Lv = sv >= 0 ? ld_u64(&lab[sv]) : kGInf;
              uint32_t best = kEmpty;
              for (uint32_t r = G.rev_row[v]; r < G.rev_row[v + 1] && Lv != kGInf; ++r) {
                const uint32_t x = G.rev_edge[r];
                if (!(G.edge_attr[x] & T.mode_bit) || x >= best) continue;
                const int su = g_find(key, cap, G.edge_src[x]);
                if (su < 0) continue;
                const unsigned long long Lu = ld_u64(&lab[su]);
                if (Lu == kGInf) continue;
                const GOffer o = g_offer(G, T, kEmpty, Lu, x);
                if (g_feasible(T, o) && gpack(o.k, o.c, o.t) == Lv) best = x;
              }
              if (best == kEmpty || n >= (int)cap) {
                good = false;
                break;
              }
              rev[n++] = best;
              v = G.edge_src[best];
            }
          } else {
            GOffer o;
            uint32_t e;
            good = g_target(G, T, key, lab, cap, ej, cj.x, a.cprep_t[s * OTR_KMAX + wj].x, &o, &e);
            while (good && e != ei) {
              if (n >= (int)cap) {
                good = false;
                break;
              }
              rev[n++] = e;
              const int sa = g_find(key, cap, e);
              const unsigned long long La = ld_u64(&lab[sa]);
              const uint32_t v = G.edge_src[e];
              uint32_t best = kEmpty;
              for (uint32_t r = G.rev_row[v]; r < G.rev_row[v + 1]; ++r) {
                const uint32_t p = G.rev_edge[r];
                if (p >= best) continue;
                const int sp2 = g_find(key, cap, p);
                if (sp2 < 0) continue;
                const unsigned long long Lp = ld_u64(&lab[sp2]);
                if (Lp == kGInf) continue;
                const GOffer q = g_offer(G, T, p, Lp, e);
                if (g_feasible(T, q) && gpack(q.k, q.c, q.t) == La) best = p;
              }
              if (best == kEmpty) {
                good = false;
                break;
              }
              e = best;
            }
          }
          (void)pj;
          s_path[0] = good ? (uint32_t)n : 0xFFFFFFFFu;
        }
        __threadfence_block();
        __syncthreads();
        const uint32_t n = s_path[0];
        if (n == 0xFFFFFFFFu) {
          if (tid == 0) {
            a.flag[item] = 1;  // cannot happen for a valid winner; reported as an overflow
            atomicAdd(a.n_overflow, 1ull);
          }
        } else {
          __shared__ unsigned long long s_off;
          const int shard = (int)(blockIdx.x & (kShards - 1));
          const int64_t region = a.capacity / kShards;
          if (tid == 0) s_off = atomicAdd(&a.cursor[shard], (unsigned long long)n);
          __syncthreads();
          const int64_t off = (int64_t)s_off;
          if (off + (int64_t)n > region) {
            if (tid == 0) *a.cap_flag = 1;
          } else {
            const int64_t base = (int64_t)shard * region + off;
            for (uint32_t q = tid; q < n; q += kGenThreads) a.path[base + q] = ld_u32(&rev[n - 1 - q]);
            if (tid == 0) {
              a.path_off[s] = base;
              a.path_len[s] = (int32_t)n;
              a.flag[item] = 0;
            }
          }
        }
      }
    }
    g_reset(key, lab, qmark, touched, &sh, cap);
  }
}

}  // namespace otr
