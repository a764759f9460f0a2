/*
 * oracle.c — scalar CPU restatement of the matching hot path.  See oracle.h for the
 * provenance of every stage and the TEST-INFRASTRUCTURE-ONLY status.  Written as a
 * straightforward reading of the algorithm (binary-heap Dijkstra, dense Viterbi,
 * sequential stitching) so that it is easy to audit against DESIGN.md §3; the HIP
 * path (reporter_amd/csrc) is an independent parallel implementation of the same
 * rules.  Floating point: plain IEEE binary64, no contraction (-ffp-contract=off),
 * no libm transcendental on a decision path (cos is the Taylor polynomial below).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/otr_graph_format.h"

/* ---------------------------------------------------------------------------- */
/* graph                                                                         */
/* ---------------------------------------------------------------------------- */
struct orc_graph {
  otr_graph_header h;
  char* blob;
  const uint32_t *node_row, *rev_row, *rev_edge, *edge_src, *edge_dst, *edge_attr, *edge_shape, *edge_seg,
      *edge_way, *seg_len, *cell_row, *cell_edge;
  const int32_t *node_ll, *shape_ll;
  const float* edge_len;
  const uint64_t* seg_id;
  uint32_t* len_mm; /* routing length, whole millimetres */
};

orc_graph* orc_graph_load(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  orc_graph* g = (orc_graph*)calloc(1, sizeof(orc_graph));
  if (fread(&g->h, sizeof(g->h), 1, f) != 1 || memcmp(g->h.magic, OTR_GRAPH_MAGIC, 8) != 0) {
    fclose(f);
    free(g);
    return NULL;
  }
  size_t sz = (size_t)g->h.array_offset[OTR_A_END];
  g->blob = (char*)malloc(sz);
  fseek(f, 0, SEEK_SET);
  if (fread(g->blob, 1, sz, f) != sz) {
    fclose(f);
    free(g->blob);
    free(g);
    return NULL;
  }
  fclose(f);
#define A(i) (g->blob + g->h.array_offset[i])
  g->node_row = (const uint32_t*)A(OTR_A_NODE_ROW);
  g->node_ll = (const int32_t*)A(OTR_A_NODE_LL);
  g->rev_row = (const uint32_t*)A(OTR_A_REV_ROW);
  g->rev_edge = (const uint32_t*)A(OTR_A_REV_EDGE);
  g->edge_src = (const uint32_t*)A(OTR_A_EDGE_SRC);
  g->edge_dst = (const uint32_t*)A(OTR_A_EDGE_DST);
  g->edge_len = (const float*)A(OTR_A_EDGE_LEN);
  g->edge_attr = (const uint32_t*)A(OTR_A_EDGE_ATTR);
  g->edge_shape = (const uint32_t*)A(OTR_A_EDGE_SHAPE);
  g->edge_seg = (const uint32_t*)A(OTR_A_EDGE_SEG);
  g->edge_way = (const uint32_t*)A(OTR_A_EDGE_WAY);
  g->shape_ll = (const int32_t*)A(OTR_A_SHAPE_LL);
  g->seg_id = (const uint64_t*)A(OTR_A_SEG_ID);
  g->seg_len = (const uint32_t*)A(OTR_A_SEG_LEN);
  g->cell_row = (const uint32_t*)A(OTR_A_CELL_ROW);
  g->cell_edge = (const uint32_t*)A(OTR_A_CELL_EDGE);
#undef A
  g->len_mm = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)g->h.n_edges + 1));
  /* routing length in whole mm, at least 1 mm: with no zero-length edges every tight
   * in-edge strictly decreases the label, so predecessor walks always end */
  for (uint32_t e = 0; e < g->h.n_edges; ++e) {
    const long long mm = llround((double)g->edge_len[e] * 1000.0);
    g->len_mm[e] = (uint32_t)(mm < 1 ? 1 : mm);
  }
  return g;
}

void orc_graph_free(orc_graph* g) {
  if (!g) return;
  free(g->len_mm);
  free(g->blob);
  free(g);
}

/* ---------------------------------------------------------------------------- */
/* geometry                                                      */
/* ---------------------------------------------------------------------------- */
static const double kM = 20037581.187 / 180.0; /* metres per degree, Batch.java:36 */

/* cos of an angle in degrees, |deg| <= 90: Taylor series to x^22, Horner. */
static double cos_deg(double deg) {
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

/* equirectangular distance, Batch.java:37-41 */
static double gc_dist(double lat1, double lon1, double lat2, double lon2) {
  double x = (lon1 - lon2) * kM * cos_deg(0.5 * (lat1 + lat2));
  double y = (lat1 - lat2) * kM;
  return sqrt(x * x + y * y);
}

static double e6(int32_t v) { return (double)v * 1e-6; }

/* ---------------------------------------------------------------------------- */
/* small dynamic arrays                                                           */
/* ---------------------------------------------------------------------------- */
#define VEC(T) struct { T* d; size_t n, cap; }
#define VPUSH(v, x)                                                      \
  do {                                                                   \
    if ((v).n == (v).cap) {                                              \
      (v).cap = (v).cap ? 2 * (v).cap : 16;                              \
      (v).d = realloc((v).d, (v).cap * sizeof(*(v).d));                  \
    }                                                                    \
    (v).d[(v).n++] = (x);                                                \
  } while (0)

typedef struct {
  uint32_t e;
  double p, d2;
} cand_t;

static int cand_cmp(const void* a, const void* b) {
  const cand_t* x = (const cand_t*)a;
  const cand_t* y = (const cand_t*)b;
  if (x->d2 < y->d2) return -1;
  if (x->d2 > y->d2) return 1;
  return x->e < y->e ? -1 : (x->e > y->e);
}

/* ---------------------------------------------------------------------------- */
/* candidate search (UPSTREAM meili CandidateGridQuery::Query)     */
/* ---------------------------------------------------------------------------- */
static int find_candidates(const orc_graph* g, double plat, double plon, double radius, uint32_t mode_bit,
                           int kmax, cand_t* out) {
  const otr_graph_header* h = &g->h;
  const double mpl = kM * cos_deg(plat);
  const double cd = h->grid_cell_deg;
  const double dlat = radius / kM, dlon = radius / mpl;
  int64_t r0 = (int64_t)floor((plat - dlat - OTR_GRID_PAD_DEG - h->grid_min_lat) / cd);
  int64_t r1 = (int64_t)floor((plat + dlat + OTR_GRID_PAD_DEG - h->grid_min_lat) / cd);
  int64_t c0 = (int64_t)floor((plon - dlon - OTR_GRID_PAD_DEG - h->grid_min_lon) / cd);
  int64_t c1 = (int64_t)floor((plon + dlon + OTR_GRID_PAD_DEG - h->grid_min_lon) / cd);
  if (r0 < 0) r0 = 0;
  if (c0 < 0) c0 = 0;
  if (r1 > (int64_t)h->grid_rows - 1) r1 = (int64_t)h->grid_rows - 1;
  if (c1 > (int64_t)h->grid_cols - 1) c1 = (int64_t)h->grid_cols - 1;
  const double r2 = radius * radius;
  VEC(cand_t) found = {0};
  for (int64_t r = r0; r <= r1; ++r)
    for (int64_t c = c0; c <= c1; ++c) {
      uint32_t cell = (uint32_t)(r * h->grid_cols + c);
      for (uint32_t q = g->cell_row[cell]; q < g->cell_row[cell + 1]; ++q) {
        uint32_t e = g->cell_edge[q];
        if (!(g->edge_attr[e] & mode_bit)) continue;
        /* closest point on the edge polyline, local metric around the probe */
        double best = INFINITY, best_along = 0.0, bqx = 0.0, bqy = 0.0, acc = 0.0;
        for (uint32_t k = g->edge_shape[e]; k + 1 < g->edge_shape[e + 1]; ++k) {
          double ax = (e6(g->shape_ll[2 * k + 1]) - plon) * mpl;
          double ay = (e6(g->shape_ll[2 * k]) - plat) * kM;
          double bx = (e6(g->shape_ll[2 * k + 3]) - plon) * mpl;
          double by = (e6(g->shape_ll[2 * k + 2]) - plat) * kM;
          double dx = bx - ax, dy = by - ay;
          double l2 = dx * dx + dy * dy;
          double t = 0.0;
          if (l2 > 0.0) {
            t = -(ax * dx + ay * dy) / l2;
            if (t < 0.0) t = 0.0;
            if (t > 1.0) t = 1.0;
          }
          double qx = ax + t * dx, qy = ay + t * dy;
          double d2 = qx * qx + qy * qy;
          double sl = sqrt(l2);
          if (d2 < best) {
            best = d2;
            best_along = acc + t * sl;
            bqx = qx;
            bqy = qy;
          }
          acc = acc + sl;
        }
        if (!(best <= r2)) continue;
        /* ownership: only the cell holding the snapped point reports the edge */
        double slat = plat + bqy / kM, slon = plon + bqx / mpl;
        int64_t sr = (int64_t)floor((slat - h->grid_min_lat) / cd);
        int64_t sc = (int64_t)floor((slon - h->grid_min_lon) / cd);
        if (sr != r || sc != c) continue;
        cand_t cd_ = {e, acc > 0.0 ? best_along / acc : 0.0, best};
        VPUSH(found, cd_);
      }
    }
  qsort(found.d, found.n, sizeof(cand_t), cand_cmp);
  int n = (int)found.n < kmax ? (int)found.n : kmax;
  for (int i = 0; i < n; ++i) out[i] = found.d[i];
  free(found.d);
  return n;
}

/* ---------------------------------------------------------------------------- */
/* bounded one-to-many Dijkstra (UPSTREAM meili routing.cc)        */
/* ---------------------------------------------------------------------------- */
#define NO_LABEL INT64_MAX
typedef struct {
  uint32_t* key;  /* node id, UINT32_MAX empty */
  int64_t* dist;  /* label, millimetres */
  uint8_t* done;
  uint32_t cap, n;
} nodemap_t;

static uint32_t hmix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

static void nm_init(nodemap_t* m, uint32_t cap) {
  m->cap = cap;
  m->n = 0;
  m->key = (uint32_t*)malloc(cap * sizeof(uint32_t));
  m->dist = (int64_t*)malloc(cap * sizeof(int64_t));
  m->done = (uint8_t*)malloc(cap);
  memset(m->key, 0xFF, cap * sizeof(uint32_t));
}
static void nm_free(nodemap_t* m) {
  free(m->key);
  free(m->dist);
  free(m->done);
}
static uint32_t nm_find(const nodemap_t* m, uint32_t k) {
  uint32_t s = hmix(k) & (m->cap - 1);
  while (m->key[s] != 0xFFFFFFFFu) {
    if (m->key[s] == k) return s;
    s = (s + 1) & (m->cap - 1);
  }
  return 0xFFFFFFFFu;
}
static void nm_grow(nodemap_t* m);
static uint32_t nm_insert(nodemap_t* m, uint32_t k, int* isnew) {
  if (2 * (m->n + 1) > m->cap) nm_grow(m);
  uint32_t s = hmix(k) & (m->cap - 1);
  while (m->key[s] != 0xFFFFFFFFu) {
    if (m->key[s] == k) {
      *isnew = 0;
      return s;
    }
    s = (s + 1) & (m->cap - 1);
  }
  m->key[s] = k;
  m->dist[s] = NO_LABEL;
  m->done[s] = 0;
  m->n++;
  *isnew = 1;
  return s;
}
static void nm_grow(nodemap_t* m) {
  nodemap_t o = *m;
  nm_init(m, o.cap * 2);
  for (uint32_t i = 0; i < o.cap; ++i)
    if (o.key[i] != 0xFFFFFFFFu) {
      int nw;
      uint32_t s = nm_insert(m, o.key[i], &nw);
      m->dist[s] = o.dist[i];
      m->done[s] = o.done[i];
    }
  nm_free(&o);
}

typedef struct {
  int64_t d;
  uint32_t node;
} heap_item;
typedef VEC(heap_item) heap_t;
static void hpush(heap_t* h, heap_item x) {
  VPUSH(*h, x);
  size_t i = h->n - 1;
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (h->d[p].d <= h->d[i].d) break;
    heap_item t = h->d[p];
    h->d[p] = h->d[i];
    h->d[i] = t;
    i = p;
  }
}
static heap_item hpop(heap_t* h) {
  heap_item top = h->d[0];
  h->d[0] = h->d[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < h->n && h->d[l].d < h->d[m].d) m = l;
    if (r < h->n && h->d[r].d < h->d[m].d) m = r;
    if (m == i) break;
    heap_item t = h->d[m];
    h->d[m] = h->d[i];
    h->d[i] = t;
    i = m;
  }
  return top;
}

/* Labels every node reachable from `start` (label 0) with its shortest-path length in
 * whole millimetres (integer, so exact and order-independent), keeping only labels
 * <= bound_mm. */
static void dijkstra(const orc_graph* g, uint32_t start, int64_t bound_mm, uint32_t mode_bit, nodemap_t* m) {
  m->n = 0;
  memset(m->key, 0xFF, m->cap * sizeof(uint32_t));
  heap_t hp = {0};
  int nw;
  uint32_t s = nm_insert(m, start, &nw);
  m->dist[s] = 0;
  heap_item it0 = {0, start};
  hpush(&hp, it0);
  while (hp.n) {
    heap_item it = hpop(&hp);
    uint32_t su = nm_find(m, it.node);
    if (m->done[su] || it.d > m->dist[su]) continue;
    m->done[su] = 1;
    int64_t du = m->dist[su];
    uint32_t u = it.node;
    for (uint32_t e = g->node_row[u]; e < g->node_row[u + 1]; ++e) {
      if (!(g->edge_attr[e] & mode_bit)) continue;
      int64_t nd = du + (int64_t)g->len_mm[e];
      if (nd > bound_mm) continue;
      uint32_t sv = nm_insert(m, g->edge_dst[e], &nw);
      if (nd < m->dist[sv]) {
        m->dist[sv] = nd;
        heap_item x = {nd, g->edge_dst[e]};
        hpush(&hp, x);
      }
    }
  }
  free(hp.d);
}

/* metres → whole millimetres of the routing bound and the partial edge lengths */
static int64_t bound_mm_of(double bound) { return (int64_t)floor(bound * 1000.0); }
static int64_t part_mm(double frac, uint32_t len_mm) { return (int64_t)llround(frac * (double)len_mm); }

/* route length in mm from candidate (ei,pi) to (ej,pj) given labels rooted at dst(ei):
 * same edge forward: round((pj-pi)*len); else round((1-pi)*len_i) + label(src(ej)) +
 * round(pj*len_j).  INT64_MAX when src(ej) was not reached. */
static int64_t route_from_labels(const orc_graph* g, const nodemap_t* m, uint32_t ei, double pi, uint32_t ej,
                                 double pj) {
  if (ej == ei && pj >= pi) return part_mm(pj - pi, g->len_mm[ei]);
  uint32_t s = nm_find(m, g->edge_src[ej]);
  if (s == 0xFFFFFFFFu) return NO_LABEL;
  return part_mm(1.0 - pi, g->len_mm[ei]) + m->dist[s] + part_mm(pj, g->len_mm[ej]);
}

int orc_route_dist(const orc_graph* g, uint32_t src_edge, double src_p, uint32_t dst_edge, double dst_p,
                   double bound, uint32_t mode_bit, double* out_dist) {
  nodemap_t m;
  nm_init(&m, 1024);
  int64_t r = NO_LABEL;
  const int64_t bmm = bound_mm_of(bound);
  if (dst_edge == src_edge && dst_p >= src_p) {
    r = part_mm(dst_p - src_p, g->len_mm[src_edge]);
  } else {
    dijkstra(g, g->edge_dst[src_edge], bmm, mode_bit, &m);
    r = route_from_labels(g, &m, src_edge, src_p, dst_edge, dst_p);
  }
  nm_free(&m);
  *out_dist = r <= bmm ? (double)r / 1000.0 : INFINITY;
  return 0;
}

/* ---------------------------------------------------------------------------- */
/* report() — reporter_service.py:79-179                                          */
/* ---------------------------------------------------------------------------- */
int orc_report(int32_t n, const uint8_t* has_id, const uint64_t* seg_id, const double* start,
               const double* end, const uint8_t* internal, const int32_t* queue, const uint8_t* has_length,
               const int32_t* length, const int32_t* begin_shape, int64_t trace_end_time, double threshold,
               uint32_t report_levels_mask, uint32_t transition_levels_mask, uint64_t* rep_id, uint64_t* rep_next,
               double* rep_t0, double* rep_t1, int32_t* rep_length, int32_t* rep_queue, orc_report_out* out) {
  memset(out, 0, sizeof(*out));
  const double end_time = (double)trace_end_time;
  int32_t last_idx = n - 1; /* :85-87 */
  while (last_idx >= 0 && end_time - start[last_idx] < threshold) last_idx--;
  out->shape_used = -1; /* :90-92, emitted only when truthy :165 */
  if (last_idx >= 0 && begin_shape[last_idx] != 0) out->shape_used = begin_shape[last_idx];
  int prior_valid = 0, prior_has_len = 0, first_seg = 1;
  uint64_t prior_id = 0;
  double prior_start = 0, prior_end = 0;
  int32_t prior_len = 0, prior_queue = 0, prior_level = -1;
  int32_t nrep = 0;
  for (int32_t idx = 0; idx <= last_idx; ++idx) {
    int lvl = has_id[idx] ? (int)(seg_id[idx] & 7u) : -1; /* :119 */
    if (idx != 0 && start[idx] == -1.0 && end[idx - 1] == -1.0) out->counts[2]++; /* :115-116 */
    int lvl_trans = lvl >= 0 && ((transition_levels_mask >> lvl) & 1u);
    if (prior_valid && prior_has_len && prior_len > 0 && !internal[idx]) { /* :122 */
      if (prior_level >= 0 && ((report_levels_mask >> prior_level) & 1u)) {
        double t0 = prior_start;
        double t1 = lvl_trans ? start[idx] : prior_end;
        double dt = t1 - t0;
        if (dt <= 0 || isinf(dt) || isnan(dt)) {
          out->counts[4]++;
        } else if (((double)prior_len / dt) * 3.6 > 160) {
          out->counts[3]++;
        } else {
          rep_id[nrep] = prior_id;
          rep_next[nrep] = (lvl_trans && has_id[idx]) ? seg_id[idx] : ORC_NO_ID;
          rep_t0[nrep] = t0;
          rep_t1[nrep] = t1;
          rep_length[nrep] = prior_len;
          rep_queue[nrep] = prior_queue;
          nrep++;
          out->counts[0]++;
          out->lengths[0] = (double)prior_len / 1000.0; /* round(len*0.001, 3), int len */
          out->length_set[0] = 1;
        }
      } else {
        out->counts[1]++;
        out->lengths[1] = (double)prior_len / 1000.0;
        out->length_set[1] = 1;
      }
    }
    if (internal[idx] && !first_seg) {
      /* :145-147 prior kept */
    } else {
      prior_valid = has_id[idx];
      prior_id = seg_id[idx];
      prior_start = start[idx];
      prior_end = end[idx];
      prior_has_len = has_length[idx];
      prior_len = length[idx];
      prior_level = lvl;
      prior_queue = queue[idx];
    }
    first_seg = 0;
    if (!has_id[idx] && !internal[idx]) out->counts[5]++; /* :161-162 */
  }
  out->n_rep = nrep;
  return 0;
}

/* ---------------------------------------------------------------------------- */
/* per-trace matching                                                            */
/* ---------------------------------------------------------------------------- */
typedef struct {
  VEC(int64_t) state_probe;
  VEC(int32_t) cand_count;
  VEC(cand_t) cands; /* ORC_KMAX per state */
  VEC(int32_t) winner;
  VEC(int32_t) subpath;
  VEC(uint32_t) route;
  /* segments */
  VEC(uint64_t) seg_id;
  VEC(double) seg_start, seg_end;
  VEC(int32_t) seg_length, seg_queue, seg_bshape, seg_eshape;
  VEC(uint8_t) seg_internal;
  VEC(int64_t) seg_way_n;
  VEC(uint32_t) seg_way;
  /* report */
  int32_t n_rep;
  uint64_t *rep_id, *rep_next;
  double *rep_t0, *rep_t1;
  int32_t *rep_length, *rep_queue;
  orc_report_out rep;
} trace_out;

typedef struct {
  uint32_t e, pad;
  int64_t s0, s1; /* route positions, whole millimetres */
} portion_t;

typedef struct {
  const orc_graph* g;
  const orc_params* p;
  const int64_t* trace_off;
  const double *lat, *lon;
  const int64_t* time;
  const float* acc;
  const uint8_t* mode;
  uint32_t rl, tl;
  trace_out* outs;
  int32_t n_traces;
  int32_t next; /* work counter */
  pthread_mutex_t mu;
} job_t;

/* time at route position s (mm): linear between the states around it */
static double time_at(const int64_t* pos, const double* tm, int n, int64_t s) {
  int k = 0;
  while (k < n - 2 && s > pos[k + 1]) ++k;
  if (pos[k + 1] > pos[k])
    return tm[k] + (tm[k + 1] - tm[k]) * ((double)(s - pos[k]) / (double)(pos[k + 1] - pos[k]));
  return tm[k];
}

static void match_trace(job_t* J, int32_t t) {
  const orc_graph* g = J->g;
  const orc_params* P = J->p;
  trace_out* O = &J->outs[t];
  memset(O, 0, sizeof(*O));
  const int64_t b = J->trace_off[t], n = J->trace_off[t + 1] - b;
  const double *lat = J->lat + b, *lon = J->lon + b;
  const int64_t* tm = J->time + b;
  const uint32_t mode_bit = 1u << J->mode[t];
  const int kmax = P->max_candidates < ORC_KMAX ? P->max_candidates : ORC_KMAX;
  const double inv2s2 = 1.0 / (P->sigma_z * P->sigma_z * 2.0);
  const double inv_beta = 1.0 / P->beta;
  if (n <= 0) goto report;
  /* 1. state selection: interpolation_distance from the last state point (§3.3) */
  {
    int64_t last = 0;
    for (int64_t i = 0; i < n; ++i) {
      int st = 0;
      if (i == 0 || i == n - 1) st = 1;
      else if (gc_dist(lat[last], lon[last], lat[i], lon[i]) >= P->interpolation_distance) st = 1;
      if (st) {
        last = i;
        VPUSH(O->state_probe, b + i);
      }
    }
  }
  const int ns = (int)O->state_probe.n;
  /* 2. candidates + emission */
  for (int s = 0; s < ns; ++s) {
    int64_t i = O->state_probe.d[s] - b;
    double a = (J->acc && J->acc[b + i] >= 0) ? (double)J->acc[b + i] : P->gps_accuracy;
    double radius = P->search_radius > a ? P->search_radius : a;
    if (radius > P->max_search_radius) radius = P->max_search_radius;
    cand_t buf[ORC_KMAX];
    int k = find_candidates(g, lat[i], lon[i], radius, mode_bit, kmax, buf);
    VPUSH(O->cand_count, k);
    for (int q = 0; q < ORC_KMAX; ++q) {
      cand_t c = q < k ? buf[q] : (cand_t){0xFFFFFFFFu, 0.0, 0.0};
      VPUSH(O->cands, c);
    }
    VPUSH(O->winner, -1);
    VPUSH(O->subpath, -1);
  }
  /* 3. active states, transitions, Viterbi (§3.4-3.6) */
  int* act = (int*)malloc(sizeof(int) * (ns + 1));
  int na = 0;
  for (int s = 0; s < ns; ++s)
    if (O->cand_count.d[s] > 0) act[na++] = s;
  double* cost = (double*)malloc(sizeof(double) * ORC_KMAX);
  double* ncost = (double*)malloc(sizeof(double) * ORC_KMAX);
  int8_t* bp = (int8_t*)malloc((size_t)(na + 1) * ORC_KMAX);
  uint8_t* brk = (uint8_t*)calloc((size_t)na + 1, 1); /* brk[k]: sub-path starts at active k */
  int* end_winner = (int*)malloc(sizeof(int) * (na + 1));
  nodemap_t nm;
  nm_init(&nm, 1024);
  double* trans = (double*)malloc(sizeof(double) * ORC_KMAX * ORC_KMAX);
  if (na > 0) {
    const cand_t* c0 = &O->cands.d[(size_t)act[0] * ORC_KMAX];
    for (int j = 0; j < O->cand_count.d[act[0]]; ++j) cost[j] = c0[j].d2 * inv2s2;
    brk[0] = 1;
  }
  for (int k = 1; k < na; ++k) {
    int sa = act[k - 1], sb = act[k];
    int64_t ia = O->state_probe.d[sa] - b, ib = O->state_probe.d[sb] - b;
    int Ka = O->cand_count.d[sa], Kb = O->cand_count.d[sb];
    const cand_t* ca = &O->cands.d[(size_t)sa * ORC_KMAX];
    const cand_t* cb = &O->cands.d[(size_t)sb * ORC_KMAX];
    double gcd = gc_dist(lat[ia], lon[ia], lat[ib], lon[ib]);
    int forced = gcd > P->breakage_distance;
    double gfl = gcd > P->interpolation_distance ? gcd : P->interpolation_distance;
    double bound = P->max_route_distance_factor * gfl;
    if (bound > P->breakage_distance) bound = P->breakage_distance;
    const int64_t bmm = bound_mm_of(bound);
    uint32_t searched = 0xFFFFFFFFu; /* labels rooted at this node are in nm */
    for (int i = 0; i < Ka; ++i) {
      for (int j = 0; j < Kb; ++j) trans[i * ORC_KMAX + j] = INFINITY;
      if (forced) continue;
      int need = 0;
      for (int j = 0; j < Kb; ++j) {
        if (cb[j].e == ca[i].e && cb[j].p >= ca[i].p) {
          int64_t r = part_mm(cb[j].p - ca[i].p, g->len_mm[ca[i].e]);
          if (r <= bmm) trans[i * ORC_KMAX + j] = fabs((double)r / 1000.0 - gcd) * inv_beta;
        } else {
          need = 1;
        }
      }
      if (!need) continue;
      /* one search per root node: labels do not depend on the source edge */
      if (g->edge_dst[ca[i].e] != searched) {
        searched = g->edge_dst[ca[i].e];
        dijkstra(g, searched, bmm, mode_bit, &nm);
      }
      for (int j = 0; j < Kb; ++j) {
        if (cb[j].e == ca[i].e && cb[j].p >= ca[i].p) continue;
        int64_t r = route_from_labels(g, &nm, ca[i].e, ca[i].p, cb[j].e, cb[j].p);
        if (r <= bmm) trans[i * ORC_KMAX + j] = fabs((double)r / 1000.0 - gcd) * inv_beta;
      }
    }
    int any = 0;
    for (int j = 0; j < Kb; ++j) {
      double best = INFINITY;
      int bi = -1;
      for (int i = 0; i < Ka; ++i) {
        double tr = trans[i * ORC_KMAX + j];
        if (tr == INFINITY || cost[i] == INFINITY) continue;
        double c = cost[i] + tr;
        if (c < best) {
          best = c;
          bi = i;
        }
      }
      bp[(size_t)k * ORC_KMAX + j] = (int8_t)bi;
      ncost[j] = bi >= 0 ? best + cb[j].d2 * inv2s2 : INFINITY;
      if (bi >= 0) any = 1;
    }
    if (!any) { /* breakage: previous sub-path ends at k-1, a new one starts at k */
      brk[k] = 1;
      for (int j = 0; j < Kb; ++j) {
        ncost[j] = cb[j].d2 * inv2s2;
        bp[(size_t)k * ORC_KMAX + j] = -1;
      }
    }
    if (brk[k]) {
      int w = 0;
      for (int i = 1; i < Ka; ++i)
        if (cost[i] < cost[w]) w = i;
      end_winner[k - 1] = w;
    }
    double* tmp = cost;
    cost = ncost;
    ncost = tmp;
  }
  if (na > 0) {
    int Kl = O->cand_count.d[act[na - 1]], w = 0;
    for (int j = 1; j < Kl; ++j)
      if (cost[j] < cost[w]) w = j;
    end_winner[na - 1] = w;
    /* backtrack */
    int cur = -1;
    for (int k = na - 1; k >= 0; --k) {
      if (k == na - 1 || brk[k + 1]) cur = end_winner[k];
      O->winner.d[act[k]] = cur;
      if (!brk[k]) cur = bp[(size_t)k * ORC_KMAX + cur];
    }
    int sp = -1;
    for (int k = 0; k < na; ++k) {
      if (brk[k]) ++sp;
      O->subpath.d[act[k]] = sp;
    }
  }
  /* 4. route stitching + OSMLR segments (§3.7-3.8) */
  {
    VEC(portion_t) por = {0};
    int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (na + 1));
    double* stm = (double*)malloc(sizeof(double) * (na + 1));
    int k = 0;
    int first_sub = 1;
    while (k < na) {
      int a = k, e_ = k + 1;
      while (e_ < na && !brk[e_]) ++e_;
      /* sub-path: active states a..e_-1 */
      int bidx = e_ - 1;
      k = e_;
      if (bidx == a) { first_sub = 0; continue; }
      if (O->route.n) VPUSH(O->route, 0xFFFFFFFFu);
      por.n = 0;
      const cand_t* c = &O->cands.d[(size_t)act[a] * ORC_KMAX + O->winner.d[act[a]]];
      uint32_t cur_e = c->e;
      int64_t cur_s0 = 0;
      pos[0] = 0;
      stm[0] = (double)tm[O->state_probe.d[act[a]] - b];
      VPUSH(O->route, cur_e);
      for (int q = a + 1; q <= bidx; ++q) {
        const cand_t* ci = &O->cands.d[(size_t)act[q - 1] * ORC_KMAX + O->winner.d[act[q - 1]]];
        const cand_t* cj = &O->cands.d[(size_t)act[q] * ORC_KMAX + O->winner.d[act[q]]];
        stm[q - a] = (double)tm[O->state_probe.d[act[q]] - b];
        if (cj->e == ci->e && cj->p >= ci->p) {
          pos[q - a] = pos[q - a - 1] + part_mm(cj->p - ci->p, g->len_mm[ci->e]);
          continue;
        }
        int64_t end_s = pos[q - a - 1] + part_mm(1.0 - ci->p, g->len_mm[ci->e]);
        portion_t pt = {cur_e, 0, cur_s0, end_s};
        VPUSH(por, pt);
        int64_t s = end_s;
        /* path: re-run the bounded search from the winner and walk predecessors */
        int64_t ia = O->state_probe.d[act[q - 1]] - b, ib = O->state_probe.d[act[q]] - b;
        double gcd = gc_dist(lat[ia], lon[ia], lat[ib], lon[ib]);
        double gfl = gcd > P->interpolation_distance ? gcd : P->interpolation_distance;
        double bound = P->max_route_distance_factor * gfl;
        if (bound > P->breakage_distance) bound = P->breakage_distance;
        uint32_t S = g->edge_dst[ci->e], T = g->edge_src[cj->e];
        dijkstra(g, S, bound_mm_of(bound), mode_bit, &nm);
        VEC(uint32_t) path = {0};
        uint32_t v = T;
        while (v != S && path.n <= g->h.n_nodes) {
          uint32_t sv = nm_find(&nm, v);
          int64_t dv = nm.dist[sv];
          uint32_t best_e = 0xFFFFFFFFu;
          for (uint32_t r = g->rev_row[v]; r < g->rev_row[v + 1]; ++r) {
            uint32_t ed = g->rev_edge[r];
            if (!(g->edge_attr[ed] & mode_bit)) continue;
            uint32_t su = nm_find(&nm, g->edge_src[ed]);
            if (su == 0xFFFFFFFFu) continue;
            if (nm.dist[su] + (int64_t)g->len_mm[ed] == dv && ed < best_e) best_e = ed;
          }
          if (best_e == 0xFFFFFFFFu) break; /* unreachable by construction */
          VPUSH(path, best_e);
          v = g->edge_src[best_e];
        }
        for (size_t z = path.n; z-- > 0;) {
          uint32_t ed = path.d[z];
          portion_t pp = {ed, 0, s, s + (int64_t)g->len_mm[ed]};
          VPUSH(por, pp);
          VPUSH(O->route, ed);
          s = s + (int64_t)g->len_mm[ed];
        }
        free(path.d);
        cur_e = cj->e;
        cur_s0 = s;
        VPUSH(O->route, cur_e);
        pos[q - a] = s + part_mm(cj->p, g->len_mm[cj->e]);
      }
      portion_t last = {cur_e, 0, cur_s0, pos[bidx - a]};
      VPUSH(por, last);
      /* trace index range owned by this sub-path, for begin/end_shape_index */
      int64_t lo = first_sub ? 0 : O->state_probe.d[act[a]] - b;
      int64_t hi = (k < na) ? O->state_probe.d[act[k]] - b - 1 : n - 1;
      first_sub = 0;
      const int nst = bidx - a + 1;
      /* group portions into traffic segments */
      size_t q = 0;
      while (q < por.n) {
        uint32_t e0 = por.d[q].e;
        uint32_t key = g->edge_seg[e0];
        int internal = (g->edge_attr[e0] & OTR_ATTR_INTERNAL) != 0;
        size_t r = q + 1;
        while (r < por.n) {
          uint32_t er = por.d[r].e, ep = por.d[r - 1].e;
          if (key != OTR_NO_SEGMENT) {
            if (g->edge_seg[er] != key || (g->edge_attr[ep] & OTR_ATTR_SEG_END) ||
                (g->edge_attr[er] & OTR_ATTR_SEG_BEGIN))
              break;
          } else {
            int ir = (g->edge_attr[er] & OTR_ATTR_INTERNAL) != 0;
            if (g->edge_seg[er] != OTR_NO_SEGMENT || ir != internal) break;
          }
          ++r;
        }
        size_t lq = r - 1;
        int64_t s0 = por.d[q].s0, s1 = por.d[lq].s1;
        double st = -1.0, et = -1.0;
        int32_t length = -1;
        if (key != OTR_NO_SEGMENT) {
          if (q != 0 && (g->edge_attr[e0] & OTR_ATTR_SEG_BEGIN)) st = time_at(pos, stm, nst, s0);
          if (lq != por.n - 1 && (g->edge_attr[por.d[lq].e] & OTR_ATTR_SEG_END)) et = time_at(pos, stm, nst, s1);
          if (st != -1.0 && et != -1.0) length = (int32_t)g->seg_len[key];
          VPUSH(O->seg_id, g->seg_id[key]);
        } else {
          if (q != 0) st = time_at(pos, stm, nst, s0);
          if (lq != por.n - 1) et = time_at(pos, stm, nst, s1);
          VPUSH(O->seg_id, ORC_NO_ID);
        }
        VPUSH(O->seg_start, st);
        VPUSH(O->seg_end, et);
        VPUSH(O->seg_length, length);
        VPUSH(O->seg_queue, 0);
        VPUSH(O->seg_internal, (uint8_t)(key == OTR_NO_SEGMENT && internal));
        int64_t nw = 0;
        uint32_t lastw = 0;
        for (size_t z = q; z <= lq; ++z) {
          uint32_t w = g->edge_way[por.d[z].e];
          if (nw == 0 || w != lastw) {
            VPUSH(O->seg_way, w);
            ++nw;
            lastw = w;
          }
        }
        VPUSH(O->seg_way_n, nw);
        /* shape indices: last trace index whose route position <= s (§3.8) */
        for (int which = 0; which < 2; ++which) {
          int64_t sq = which ? s1 : s0;
          int64_t best = lo;
          int st_ptr = -1;
          for (int64_t ti = lo; ti <= hi; ++ti) {
            while (st_ptr + 1 < nst && O->state_probe.d[act[a + st_ptr + 1]] - b <= ti) ++st_ptr;
            if (st_ptr >= 0 && pos[st_ptr] <= sq) best = ti;
          }
          if (which) VPUSH(O->seg_eshape, (int32_t)best);
          else VPUSH(O->seg_bshape, (int32_t)best);
        }
        q = r;
      }
    }
    free(por.d);
    free(pos);
    free(stm);
  }
  nm_free(&nm);
  free(trans);
  free(act);
  free(cost);
  free(ncost);
  free(bp);
  free(brk);
  free(end_winner);
report:
  /* 5. report() over this trace's segments */
  {
    int32_t nsg = (int32_t)O->seg_id.n;
    uint8_t* has_id = (uint8_t*)malloc((size_t)nsg + 1);
    uint8_t* has_len = (uint8_t*)malloc((size_t)nsg + 1);
    for (int32_t i = 0; i < nsg; ++i) {
      has_id[i] = O->seg_id.d[i] != ORC_NO_ID;
      has_len[i] = 1;
    }
    O->rep_id = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)nsg + 1));
    O->rep_next = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)nsg + 1));
    O->rep_t0 = (double*)malloc(sizeof(double) * ((size_t)nsg + 1));
    O->rep_t1 = (double*)malloc(sizeof(double) * ((size_t)nsg + 1));
    O->rep_length = (int32_t*)malloc(sizeof(int32_t) * ((size_t)nsg + 1));
    O->rep_queue = (int32_t*)malloc(sizeof(int32_t) * ((size_t)nsg + 1));
    int64_t end_t = n > 0 ? tm[n - 1] : 0;
    orc_report(nsg, has_id, O->seg_id.d, O->seg_start.d, O->seg_end.d, O->seg_internal.d, O->seg_queue.d, has_len,
               O->seg_length.d, O->seg_bshape.d, end_t, (double)P->threshold_sec, J->rl, J->tl, O->rep_id,
               O->rep_next, O->rep_t0, O->rep_t1, O->rep_length, O->rep_queue, &O->rep);
    O->n_rep = O->rep.n_rep;
    free(has_id);
    free(has_len);
  }
}

static void* worker(void* arg) {
  job_t* J = (job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&J->mu);
    int32_t t = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (t >= J->n_traces) break;
    match_trace(J, t);
  }
  return NULL;
}

#define CAT(field, T, count_expr)                                                 \
  do {                                                                            \
    size_t tot = 0;                                                               \
    for (int32_t t = 0; t < n_traces; ++t) tot += (count_expr);                   \
    out->field = (T*)malloc(sizeof(T) * (tot + 1));                                \
    size_t o = 0;                                                                 \
    for (int32_t t = 0; t < n_traces; ++t) {                                      \
      size_t c = (count_expr);                                                    \
      if (c) memcpy(out->field + o, SRC_##field, sizeof(T) * c);                  \
      o += c;                                                                     \
    }                                                                             \
  } while (0)

int orc_match_batch(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off,
                    const double* lat, const double* lon, const int64_t* time, const float* accuracy,
                    const uint8_t* mode, uint32_t report_levels_mask, uint32_t transition_levels_mask,
                    int32_t n_threads, orc_result* out) {
  memset(out, 0, sizeof(*out));
  job_t J;
  memset(&J, 0, sizeof(J));
  J.g = g;
  J.p = p;
  J.trace_off = trace_off;
  J.lat = lat;
  J.lon = lon;
  J.time = time;
  J.acc = accuracy;
  J.mode = mode;
  J.rl = report_levels_mask;
  J.tl = transition_levels_mask;
  J.n_traces = n_traces;
  J.outs = (trace_out*)calloc((size_t)n_traces + 1, sizeof(trace_out));
  pthread_mutex_init(&J.mu, NULL);
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &J);
  for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&J.mu);
  trace_out* T = J.outs;
  out->n_traces = n_traces;
  out->trace_state_off = (int64_t*)malloc(sizeof(int64_t) * (n_traces + 1));
  out->trace_route_off = (int64_t*)malloc(sizeof(int64_t) * (n_traces + 1));
  out->trace_seg_off = (int64_t*)malloc(sizeof(int64_t) * (n_traces + 1));
  out->trace_rep_off = (int64_t*)malloc(sizeof(int64_t) * (n_traces + 1));
  out->shape_used = (int32_t*)malloc(sizeof(int32_t) * (n_traces + 1));
  out->stats = (int32_t*)malloc(sizeof(int32_t) * 7 * (n_traces + 1));
  out->stats_len = (double*)malloc(sizeof(double) * 2 * (n_traces + 1));
  out->trace_state_off[0] = out->trace_route_off[0] = out->trace_seg_off[0] = out->trace_rep_off[0] = 0;
  for (int32_t t = 0; t < n_traces; ++t) {
    out->trace_state_off[t + 1] = out->trace_state_off[t] + (int64_t)T[t].state_probe.n;
    out->trace_route_off[t + 1] = out->trace_route_off[t] + (int64_t)T[t].route.n;
    out->trace_seg_off[t + 1] = out->trace_seg_off[t] + (int64_t)T[t].seg_id.n;
    out->trace_rep_off[t + 1] = out->trace_rep_off[t] + T[t].n_rep;
    out->shape_used[t] = T[t].rep.shape_used;
    for (int k = 0; k < 6; ++k) out->stats[7 * t + k] = T[t].rep.counts[k];
    out->stats[7 * t + 6] = 0;
    out->stats_len[2 * t] = T[t].rep.lengths[0];
    out->stats_len[2 * t + 1] = T[t].rep.lengths[1];
  }
  out->n_states = out->trace_state_off[n_traces];
  out->n_route = out->trace_route_off[n_traces];
  out->n_seg = out->trace_seg_off[n_traces];
  out->n_rep = out->trace_rep_off[n_traces];
#define SRC_state_probe T[t].state_probe.d
#define SRC_cand_count T[t].cand_count.d
#define SRC_winner T[t].winner.d
#define SRC_subpath T[t].subpath.d
#define SRC_route_edge T[t].route.d
#define SRC_seg_id T[t].seg_id.d
#define SRC_seg_start T[t].seg_start.d
#define SRC_seg_end T[t].seg_end.d
#define SRC_seg_length T[t].seg_length.d
#define SRC_seg_queue T[t].seg_queue.d
#define SRC_seg_internal T[t].seg_internal.d
#define SRC_seg_begin_shape T[t].seg_bshape.d
#define SRC_seg_end_shape T[t].seg_eshape.d
#define SRC_seg_way T[t].seg_way.d
#define SRC_rep_id T[t].rep_id
#define SRC_rep_next T[t].rep_next
#define SRC_rep_t0 T[t].rep_t0
#define SRC_rep_t1 T[t].rep_t1
#define SRC_rep_length T[t].rep_length
#define SRC_rep_queue T[t].rep_queue
  CAT(state_probe, int64_t, T[t].state_probe.n);
  CAT(cand_count, int32_t, T[t].cand_count.n);
  CAT(winner, int32_t, T[t].winner.n);
  CAT(subpath, int32_t, T[t].subpath.n);
  CAT(route_edge, uint32_t, T[t].route.n);
  CAT(seg_id, uint64_t, T[t].seg_id.n);
  CAT(seg_start, double, T[t].seg_start.n);
  CAT(seg_end, double, T[t].seg_end.n);
  CAT(seg_length, int32_t, T[t].seg_length.n);
  CAT(seg_queue, int32_t, T[t].seg_queue.n);
  CAT(seg_internal, uint8_t, T[t].seg_internal.n);
  CAT(seg_begin_shape, int32_t, T[t].seg_bshape.n);
  CAT(seg_end_shape, int32_t, T[t].seg_eshape.n);
  CAT(seg_way, uint32_t, T[t].seg_way.n);
  CAT(rep_id, uint64_t, (size_t)T[t].n_rep);
  CAT(rep_next, uint64_t, (size_t)T[t].n_rep);
  CAT(rep_t0, double, (size_t)T[t].n_rep);
  CAT(rep_t1, double, (size_t)T[t].n_rep);
  CAT(rep_length, int32_t, (size_t)T[t].n_rep);
  CAT(rep_queue, int32_t, (size_t)T[t].n_rep);
  /* candidates: ORC_KMAX slots per state */
  out->cand_edge = (uint32_t*)malloc(sizeof(uint32_t) * ORC_KMAX * ((size_t)out->n_states + 1));
  out->cand_p = (double*)malloc(sizeof(double) * ORC_KMAX * ((size_t)out->n_states + 1));
  out->cand_sqd = (double*)malloc(sizeof(double) * ORC_KMAX * ((size_t)out->n_states + 1));
  {
    size_t o = 0;
    for (int32_t t = 0; t < n_traces; ++t)
      for (size_t q = 0; q < T[t].cands.n; ++q, ++o) {
        out->cand_edge[o] = T[t].cands.d[q].e;
        out->cand_p[o] = T[t].cands.d[q].p;
        out->cand_sqd[o] = T[t].cands.d[q].d2;
      }
  }
  out->seg_way_off = (int64_t*)malloc(sizeof(int64_t) * ((size_t)out->n_seg + 1));
  {
    size_t o = 0;
    out->seg_way_off[0] = 0;
    for (int32_t t = 0; t < n_traces; ++t)
      for (size_t q = 0; q < T[t].seg_way_n.n; ++q, ++o) out->seg_way_off[o + 1] = out->seg_way_off[o] + T[t].seg_way_n.d[q];
  }
  for (int32_t t = 0; t < n_traces; ++t) {
    trace_out* O = &T[t];
    free(O->state_probe.d); free(O->cand_count.d); free(O->cands.d); free(O->winner.d); free(O->subpath.d);
    free(O->route.d); free(O->seg_id.d); free(O->seg_start.d); free(O->seg_end.d); free(O->seg_length.d);
    free(O->seg_queue.d); free(O->seg_bshape.d); free(O->seg_eshape.d); free(O->seg_internal.d);
    free(O->seg_way_n.d); free(O->seg_way.d); free(O->rep_id); free(O->rep_next); free(O->rep_t0);
    free(O->rep_t1); free(O->rep_length); free(O->rep_queue);
  }
  free(T);
  return 0;
}

void orc_result_free(orc_result* r) {
  void* ptrs[] = {r->trace_state_off, r->state_probe, r->cand_count, r->cand_edge, r->cand_p, r->cand_sqd,
                  r->winner, r->subpath, r->trace_route_off, r->route_edge, r->trace_seg_off, r->seg_id,
                  r->seg_start, r->seg_end, r->seg_length, r->seg_queue, r->seg_internal, r->seg_begin_shape,
                  r->seg_end_shape, r->seg_way_off, r->seg_way, r->trace_rep_off, r->rep_id, r->rep_next,
                  r->rep_t0, r->rep_t1, r->rep_length, r->rep_queue, r->shape_used, r->stats, r->stats_len};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
  memset(r, 0, sizeof(*r));
}
