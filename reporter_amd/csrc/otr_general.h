// otr_general.h — K3g/K6g: the bounded route search with its labels in HBM.
//
// The LDS search (otr_kernels.h, search_run) is the fast path: node labels packed in
// 32 bits (length mm << sh | time 0.1 s), at most 4096 slots per search.  Everything
// it cannot hold runs here, with no capacity limit below the slab size:
//   * turn costs (turn_penalty_factor > 0): the search is over EDGE states, because
//     the turn cost at a node depends on the edge that entered it;
//   * steps whose bounds do not fit the 32-bit packing;
//   * searches that outgrew the largest LDS table.
// Labels are 64-bit lexicographic keys d:25 | t:17 | c:22 (length mm, time 0.1 s, turn
// cost mm; oracle rkey with the ORC_* caps), so one atomicMin keeps the exact
// lexicographic minimum and the fixed point is independent of the processing order.
//
// One workgroup (kGenThreads) per task, persistent over a device task list whose length
// is read on the device (no host round trip).  Each workgroup owns a slab: an open-
// addressing hash table {state, label, round stamp} plus two frontier lists and the
// list of claimed slots (reset at the end of the task, so a slab is never cleared as a
// whole).  Rounds are label-correcting (a state is re-expanded whenever its label
// improves) over the frontier; the search ends when no label improved.
#pragma once
#include "otr_kernels.h"

namespace otr {

constexpr int kGenThreads = 256;
constexpr unsigned long long kGInf = 0xFFFFFFFFFFFFFFFFull;

__host__ __device__ inline unsigned long long gpack(uint64_t d, uint64_t t, uint64_t c) {
  return (d << 39) | (t << 22) | c;
}
__host__ __device__ inline uint32_t g_d(unsigned long long w) { return (uint32_t)(w >> 39); }
__host__ __device__ inline uint32_t g_t(unsigned long long w) { return (uint32_t)((w >> 22) & 0x1FFFFull); }
__host__ __device__ inline uint32_t g_c(unsigned long long w) { return (uint32_t)(w & 0x3FFFFFull); }

struct GSlabs {
  uint32_t* key;                // [n][cap] edge state, kEmpty
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
  const uint4* cprep;           // per candidate {part(p), src(e), h(src), part(1 - p)}
  const uint2* cprep_t;         // per candidate {part_t(p), part_t(1 - p)}
  const int32_t* state_trace;
  const uint8_t* mode_of_trace;
  uint32_t turn_modes;          // bit m: mode m has turn costs
  const int32_t* turn;          // [OTR_MODES][181] turn cost table, mm
  // route mode
  const int64_t* task_state;
  const unsigned long long* task_mask;
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
    if (k == e) {
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
    if (k == e) return (int)h;
    h = (h + 1u) & (cap - 1u);
  }
  return -1;
}

struct GTask {
  int64_t s, sp;
  uint32_t root;        // node (node mode) or edge (edge mode)
  bool edge_mode, time_on;
  uint32_t bmm;
  int32_t bt;
  int mode;
  const uint32_t* et;   // the mode's edge times
  const int32_t* turn;  // the mode's turn table
  uint32_t mode_bit;
};

// Workgroup-wide bounded label-correcting search of one task in slab `sl`.  Returns
// false (workgroup-uniform) on slab overflow.
__device__ bool g_search(const DevGraph& G, const GTask& T, uint32_t* key, unsigned long long* lab, uint32_t* qmark,
                         uint32_t* fr, uint32_t* touched, uint32_t cap, uint32_t* s_n, uint32_t* s_touched,
                         uint32_t* s_ovf, unsigned long long* work) {
  const int tid = threadIdx.x;
  const uint32_t maxk = cap - cap / 8u;
  unsigned long long my_relaxed = 0;
  if (tid == 0) {
    *s_touched = 0;
    *s_ovf = 0;
    s_n[0] = 0;
    s_n[1] = 0;
  }
  __syncthreads();
  // relax state a (or the virtual root node when a == kEmpty) with label L into edge b
  auto relax = [&](uint32_t a, unsigned long long L, uint32_t b, uint32_t round, int nxt) {
    const uint32_t attr = G.edge_attr[b];
    if (!(attr & T.mode_bit)) return;
    ++my_relaxed;
    const uint32_t nd = g_d(L) + G.len_mm[b];
    if (nd > T.bmm) return;
    uint32_t nt = 0, nc = 0;
    if (T.time_on) {
      const uint32_t x = g_t(L) + T.et[b];
      nt = x < kTCap ? x : kTCap;
    }
    if (T.edge_mode && a != kEmpty) {
      const int td = turn_degree(G.edge_head[a].y, G.edge_head[b].x);
      const uint32_t x = g_c(L) + (uint32_t)T.turn[td];
      nc = x < kTcCap ? x : kTcCap;
    } else if (T.edge_mode) {
      nc = g_c(L);
    }
    const unsigned long long w = gpack(nd, nt, nc);
    bool claimed = false;
    const int sl = g_claim(key, cap, b, &claimed);
    if (sl < 0) {
      *s_ovf = 1;
      return;
    }
    if (claimed) {
      const uint32_t k = atomicAdd(s_touched, 1u);
      if (k < cap) touched[k] = (uint32_t)sl;
      if (k >= maxk) *s_ovf = 1;
    }
    const unsigned long long old = atomicMin(&lab[sl], w);
    if (w < old && atomicExch(&qmark[sl], round + 1u) != round + 1u) {
      const uint32_t p = atomicAdd(&s_n[nxt], 1u);
      if (p < cap) fr[(size_t)nxt * cap + p] = (uint32_t)sl;
      else *s_ovf = 1;
    }
  };
  // round 0: the root's out-edges
  {
    uint32_t v;
    unsigned long long L0 = 0ull;
    uint32_t from = kEmpty;
    if (T.edge_mode) {
      // the root edge is a state with label 0 (labels are relative to its exit)
      if (tid == 0) {
        bool claimed = false;
        const int sl = g_claim(key, cap, T.root, &claimed);
        if (sl >= 0) {
          lab[sl] = 0ull;
          if (claimed) touched[atomicAdd(s_touched, 1u)] = (uint32_t)sl;
        } else {
          *s_ovf = 1;
        }
      }
      v = G.edge_dst[T.root];
      from = T.root;
    } else {
      v = T.root;
    }
    __syncthreads();
    const uint32_t e0 = G.node_row[v], e1 = G.node_row[v + 1];
    for (uint32_t e = e0 + tid; e < e1; e += kGenThreads) relax(from, L0, e, 0u, 0);
  }
  __syncthreads();
  uint32_t round = 0;
  int cur = 0;
  unsigned long long expanded = 0;  // states expanded (uniform): the search's "settled" count
  for (;;) {
    const uint32_t n = s_n[cur];
    if (n == 0 || *s_ovf) break;
    const int nxt = cur ^ 1;
    ++round;
    if (tid == 0) s_n[nxt] = 0;
    __syncthreads();
    const uint32_t nn = n < cap ? n : cap;
    expanded += nn;
    for (uint32_t i = tid; i < nn; i += kGenThreads) {
      const uint32_t sl = ld_u32(&fr[(size_t)cur * cap + i]);
      const uint32_t a = ld_u32(&key[sl]);
      const unsigned long long L = ld_u64(&lab[sl]);
      const uint32_t v = G.edge_dst[a];
      for (uint32_t e = G.node_row[v]; e < G.node_row[v + 1]; ++e) relax(a, L, e, round, nxt);
    }
    __threadfence_block();
    __syncthreads();
    cur = nxt;
  }
  __syncthreads();
  if (work) {  // this tier's counter bank (kinds 3 settled, 4 relaxed)
    const int sh = cshard();
    atomicAdd(&work[4 * kCShards + sh], my_relaxed);
    if (tid == 0) atomicAdd(&work[3 * kCShards + sh], expanded);
  }
  return *s_ovf == 0;
}

// the best label at node v: node mode the minimum over labelled in-edge states (the
// root node: 0); edge mode with the turn into edge ej added (min id among equals)
__device__ inline bool g_node_key(const DevGraph& G, const GTask& T, const uint32_t* key,
                                  const unsigned long long* lab, uint32_t cap, uint32_t ej,
                                  unsigned long long* out, uint32_t* via) {
  const uint32_t v = G.edge_src[ej];
  if (!T.edge_mode && v == T.root) {
    *out = 0ull;
    *via = kEmpty;
    return true;
  }
  bool found = false;
  unsigned long long best = kGInf;
  uint32_t bid = kEmpty;
  for (uint32_t r = G.rev_row[v]; r < G.rev_row[v + 1]; ++r) {
    const uint32_t a = G.rev_edge[r];
    const int sl = g_find(key, cap, a);
    if (sl < 0) continue;
    unsigned long long k = ld_u64(&lab[sl]);
    if (k == kGInf) continue;
    if (T.edge_mode) {
      const uint32_t x = g_c(k) + (uint32_t)T.turn[turn_degree(G.edge_head[a].y, G.edge_head[ej].x)];
      k = (k & ~0x3FFFFFull) | (x < kTcCap ? x : kTcCap);
    }
    if (!found || k < best || (k == best && a < bid)) {
      best = k;
      bid = a;
      found = true;
    }
  }
  *out = best;
  *via = bid;
  return found;
}

__device__ inline GTask g_task(const DevGraph& G, const GenArgs& a, int64_t s, int64_t sp, uint32_t ei) {
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
  return T;
}

// reset the claimed slots of a slab (workgroup-wide), ready for the next task
__device__ inline void g_reset(uint32_t* key, unsigned long long* lab, uint32_t* qmark, const uint32_t* touched,
                               uint32_t n_touched, uint32_t cap) {
  const uint32_t n = n_touched < cap ? n_touched : cap;
  for (uint32_t i = threadIdx.x; i < n; i += kGenThreads) {
    const uint32_t sl = touched[i];
    key[sl] = kEmpty;
    lab[sl] = kGInf;
    qmark[sl] = 0u;
  }
  __threadfence_block();
  __syncthreads();
}

__global__ __launch_bounds__(kGenThreads) void k_general(DevGraph G, GenArgs a, GSlabs S) {
  __shared__ uint32_t s_n[2], s_touched, s_ovf;
  __shared__ uint32_t s_path[1];
  const uint32_t cap = S.cap;
  uint32_t* key = S.key + (size_t)blockIdx.x * cap;
  unsigned long long* lab = S.lab + (size_t)blockIdx.x * cap;
  uint32_t* qmark = S.qmark + (size_t)blockIdx.x * cap;
  uint32_t* fr = S.fr + (size_t)blockIdx.x * 2 * cap;
  uint32_t* touched = S.touched + (size_t)blockIdx.x * cap;
  const int64_t count = (int64_t)*a.list_count;
  const int tid = threadIdx.x;
  for (int64_t k = blockIdx.x; k < count; k += gridDim.x) {
    const int64_t item = a.list[k];
    if (a.mode == 0) {
      // ---- route task: transitions of every source sharing the root node; with turn
      // costs (edge mode) every source edge is its own root: one search each
      const int64_t s = a.task_state[item];
      const unsigned long long mask = a.task_mask[item];
      const int64_t sp = a.prev[s];
      GTask T = g_task(G, a, s, sp, a.cand_edge[sp * OTR_KMAX + (__ffsll((long long)mask) - 1)]);
      bool ok = true;
      for (unsigned long long todo = mask; todo && ok;) {
        const int ia = __ffsll((long long)todo) - 1;
        const unsigned long long grp = T.edge_mode ? (1ull << ia) : todo;
        todo &= ~grp;
        if (T.edge_mode) T.root = a.cand_edge[sp * OTR_KMAX + ia];
        if (grp != mask) {  // a later source: a fresh slab
          __syncthreads();
          g_reset(key, lab, qmark, touched, s_touched, cap);
        }
        ok = g_search(G, T, key, lab, qmark, fr, touched, cap, s_n, &s_touched, &s_ovf, a.counters);
        if (!ok) break;
        const int Kb = a.cand_count[s];
        if (a.counters && tid == 0) {  // kinds 5 transition entries, 6 searches
          const int sh = cshard();
          atomicAdd(&a.counters[5 * kCShards + sh], (unsigned long long)Kb * (unsigned long long)__popcll(grp));
          atomicAdd(&a.counters[6 * kCShards + sh], 1ull);
        }
        uint32_t* trow = a.trans + a.trans_off[s];
        uint32_t* crow = a.trans_tc + a.trans_off[s];
        for (int j = tid; j < Kb; j += kGenThreads) {
          const uint32_t ej = a.cand_edge[s * OTR_KMAX + j];
          const double pj = a.cand_p[s * OTR_KMAX + j];
          const uint4 cj = a.cprep[s * OTR_KMAX + j];
          const uint2 cjt = a.cprep_t[s * OTR_KMAX + j];
          unsigned long long L;
          uint32_t via;
          const bool reached = g_node_key(G, T, key, lab, cap, ej, &L, &via);
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
              const uint4 ci = a.cprep[sp * OTR_KMAX + i];
              const uint2 cit = a.cprep_t[sp * OTR_KMAX + i];
              rd = (int64_t)ci.w + g_d(L) + cj.x;
              rt = T.time_on ? (int64_t)cit.y + g_t(L) + cjt.x : 0;
              rc = g_c(L);
            }
            const bool valid = rd >= 0 && rd <= (int64_t)T.bmm && (!T.time_on || rt <= (int64_t)T.bt);
            trow[(int64_t)i * Kb + j] = valid ? (uint32_t)rd : kNoRoute;
            if (T.edge_mode) crow[(int64_t)i * Kb + j] = rc;  // allocated for turn modes only
          }
        }
      }
      if (ok) {
        if (tid == 0) a.flag[item] = 0;
      } else if (tid == 0) {
        a.flag[item] = 1;
        atomicAdd(a.n_overflow, 1ull);
      }
    } else {
      // ---- winner path of a step: search from the winner's root, then walk back
      const int64_t s = a.steps[item];
      const int64_t sp = a.prev[s];
      const int wi = a.winner[sp], wj = a.winner[s];
      const uint32_t ei = a.cand_edge[sp * OTR_KMAX + wi], ej = a.cand_edge[s * OTR_KMAX + wj];
      const GTask T = g_task(G, a, s, sp, ei);
      const bool ok = g_search(G, T, key, lab, qmark, fr, touched, cap, s_n, &s_touched, &s_ovf, nullptr);
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
          unsigned long long L;
          uint32_t e;
          if (!T.edge_mode) {
            // node labels: at v, the smallest-id in-edge whose state label is v's label
            uint32_t v = G.edge_src[ej];
            const uint32_t S0 = T.root;
            while (v != S0) {
              uint32_t best = kEmpty;
              unsigned long long bl = kGInf;
              for (uint32_t r = G.rev_row[v]; r < G.rev_row[v + 1]; ++r) {
                const uint32_t x = G.rev_edge[r];
                const int sl = g_find(key, cap, x);
                if (sl < 0) continue;
                const unsigned long long k2 = ld_u64(&lab[sl]);
                if (k2 < bl || (k2 == bl && x < best)) {
                  bl = k2;
                  best = x;
                }
              }
              if (best == kEmpty || bl == kGInf || n >= (int)cap) {
                good = false;
                break;
              }
              rev[n++] = best;
              v = G.edge_src[best];
            }
          } else {
            good = g_node_key(G, T, key, lab, cap, ej, &L, &e);
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
                const int sp2 = g_find(key, cap, p);
                if (sp2 < 0) continue;
                const unsigned long long Lp = ld_u64(&lab[sp2]);
                if (Lp == kGInf) continue;
                // Lp + step(p -> e) == La ?
                const uint32_t nd = g_d(Lp) + G.len_mm[e];
                uint32_t nt = 0, nc = 0;
                if (T.time_on) {
                  const uint32_t x = g_t(Lp) + T.et[e];
                  nt = x < kTCap ? x : kTCap;
                }
                {
                  const uint32_t x = g_c(Lp) + (uint32_t)T.turn[turn_degree(G.edge_head[p].y, G.edge_head[e].x)];
                  nc = x < kTcCap ? x : kTcCap;
                }
                if (nd <= 0x1FFFFFFu && gpack(nd, nt, nc) == La && p < best) best = p;
              }
              if (best == kEmpty) {
                good = false;
                break;
              }
              e = best;
            }
          }
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
    __syncthreads();
    g_reset(key, lab, qmark, touched, s_touched, cap);
  }
}

}  // namespace otr
