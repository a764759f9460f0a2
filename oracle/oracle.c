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
  int16_t *h_begin, *h_end; /* headings of the first / last shape segment, degrees (§3.5) */
};

static double cos_deg(double deg);

/* heading (integer degrees clockwise from north, 0..359) of the shape segment a → b in
 * the local equirectangular metric; -1 for a zero-length segment */
static int seg_heading(const int32_t* a, const int32_t* b) {
  const double la1 = (double)a[0] * 1e-6, lo1 = (double)a[1] * 1e-6;
  const double la2 = (double)b[0] * 1e-6, lo2 = (double)b[1] * 1e-6;
  const double m = 20037581.187 / 180.0; /* metres per degree, Batch.java:36 */
  const double x = (lo2 - lo1) * m * cos_deg(0.5 * (la1 + la2));
  const double y = (la2 - la1) * m;
  if (x == 0.0 && y == 0.0) return -1;
  double deg = atan2(x, y) * (180.0 / 3.14159265358979323846);
  if (deg < 0.0) deg = deg + 360.0;
  return (int)(llround(deg) % 360);
}

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
  g->h_begin = (int16_t*)malloc(sizeof(int16_t) * ((size_t)g->h.n_edges + 1));
  g->h_end = (int16_t*)malloc(sizeof(int16_t) * ((size_t)g->h.n_edges + 1));
  for (uint32_t e = 0; e < g->h.n_edges; ++e) {
    const uint32_t k0 = g->edge_shape[e], k1 = g->edge_shape[e + 1];
    int hb = -1, he = -1;
    for (uint32_t k = k0; k + 1 < k1 && hb < 0; ++k) hb = seg_heading(g->shape_ll + 2 * k, g->shape_ll + 2 * k + 2);
    for (uint32_t k = k1 - 1; k > k0 && he < 0; --k) he = seg_heading(g->shape_ll + 2 * k - 2, g->shape_ll + 2 * k);
    g->h_begin[e] = (int16_t)(hb < 0 ? 0 : hb);
    g->h_end[e] = (int16_t)(he < 0 ? 0 : he);
  }
  return g;
}

void orc_graph_free(orc_graph* g) {
  if (!g) return;
  free(g->len_mm);
  free(g->h_begin);
  free(g->h_end);
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
/* bounded one-to-many routing (UPSTREAM meili routing.cc)     */
/* ---------------------------------------------------------------------------- */
/* A route label is (k, d, t): k = the search key = length + accumulated turn cost (mm;
 * k = d when the mode has no turn costs), d = length in whole mm, t = route time in 0.1 s
 * (tracked only while the step's time bound is active, else 0).  Labels are compared
 * lexicographically on (k, d, t).  The search is label-setting in that order (UPSTREAM
 * meili find_shortest_path: a priority queue on the distance-plus-turn sort cost), it
 * starts at the source candidate with the exit part of its edge, and it PRUNES every
 * relaxation whose route exceeds a bound: length > B_mm, time > bt (the step's
 * max_route_time_factor bound), or turn cost > ORC_TCCAP.  A label is therefore the
 * lexicographic minimum over the feasible offers of the FINAL labels of its
 * predecessors — a unique fixed point (by induction on k: every step adds >= 1 mm), which
 * the GPU's parallel search must reproduce exactly. */
typedef struct {
  int64_t k, d, t;
} rkey;

static int rk_lt(rkey a, rkey b) {
  if (a.k != b.k) return a.k < b.k;
  if (a.d != b.d) return a.d < b.d;
  return a.t < b.t;
}
static int rk_eq(rkey a, rkey b) { return a.k == b.k && a.d == b.d && a.t == b.t; }

typedef struct {
  uint32_t* key;  /* node or edge id, UINT32_MAX empty */
  rkey* lab;
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
  m->lab = (rkey*)malloc(cap * sizeof(rkey));
  m->done = (uint8_t*)malloc(cap);
  memset(m->key, 0xFF, cap * sizeof(uint32_t));
}
static void nm_free(nodemap_t* m) {
  free(m->key);
  free(m->lab);
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
  m->lab[s].k = INT64_MAX;
  m->lab[s].d = INT64_MAX;
  m->lab[s].t = INT64_MAX;
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
      m->lab[s] = o.lab[i];
      m->done[s] = o.done[i];
    }
  nm_free(&o);
}

typedef struct {
  rkey k;
  uint32_t id;
} heap_item;
typedef VEC(heap_item) heap_t;
static int hi_lt(const heap_item* a, const heap_item* b) { return rk_lt(a->k, b->k); }
static void hpush(heap_t* h, heap_item x) {
  VPUSH(*h, x);
  size_t i = h->n - 1;
  while (i > 0) {
    size_t p = (i - 1) / 2;
    if (!hi_lt(&h->d[i], &h->d[p])) break;
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
    if (l < h->n && hi_lt(&h->d[l], &h->d[m])) m = l;
    if (r < h->n && hi_lt(&h->d[r], &h->d[m])) m = r;
    if (m == i) break;
    heap_item t = h->d[m];
    h->d[m] = h->d[i];
    h->d[i] = t;
    i = m;
  }
  return top;
}

/* metres → whole millimetres of the routing bound and the partial edge lengths; the
 * same for route times (0.1 s) of partial edges */
static int64_t bound_mm_of(double bound) { return (int64_t)floor(bound * 1000.0); }
static int64_t part_mm(double frac, uint32_t len_mm) { return (int64_t)llround(frac * (double)len_mm); }

/* per-mode routing data */
typedef struct {
  uint32_t* time_ds; /* [E] route time of each edge at the mode's speed, 0.1 s */
  int32_t turn[181]; /* turn cost by turn degree (0 = U-turn, 180 = straight), mm */
  int turn_on;
  uint32_t mode_bit;
} mode_data;

/* e^(-1/45) by its Taylor series; the turn table multiplies it up (deterministic, no libm) */
void orc_turn_table(const orc_params* p, int32_t* tab) {
  const double x = -1.0 / 45.0;
  double r = 1.0, term = 1.0;
  for (int k = 1; k <= 20; ++k) {
    term = term * x / (double)k;
    r = r + term;
  }
  double f = 1.0;
  for (int i = 0; i <= 180; ++i) {
    const double v = 1000.0 * p->turn_penalty_factor * f; /* turn_penalty_factor * exp(-i/45) m */
    tab[i] = p->turn_penalty_factor > 0.0 ? (int32_t)llround(v) : 0;
    f = f * r;
  }
}

/* route time of one edge at the mode's speed: 0.1 s units, len_mm * 0.036 / kph */
static uint32_t edge_time_ds(const orc_graph* g, const orc_params* p, uint32_t e) {
  double kph = (double)OTR_ATTR_SPEED(g->edge_attr[e]);
  if (!(kph > 0.0)) kph = 30.0; /* unknown speed */
  if (p->speed_kph > 0.0 && p->speed_kph < kph) kph = p->speed_kph;
  const double v = (double)g->len_mm[e] * 0.036 / kph;
  return v < 2.0e9 ? (uint32_t)llround(v) : 2000000000u;
}

static void mode_data_init(const orc_graph* g, const orc_params* p, int mode, mode_data* md) {
  md->time_ds = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)g->h.n_edges + 1));
  for (uint32_t e = 0; e < g->h.n_edges; ++e) md->time_ds[e] = edge_time_ds(g, p, e);
  orc_turn_table(p, md->turn);
  md->turn_on = p->turn_penalty_factor > 0.0;
  md->mode_bit = 1u << mode;
}

/* turn degree at a node from in-edge a to out-edge b: the angle between the heading
 * back along a and the heading out along b, folded to 0..180 (0 = U-turn) */
static int turn_degree(const orc_graph* g, uint32_t a, uint32_t b) {
  const int back = (g->h_end[a] + 180) % 360;
  const int td = (g->h_begin[b] - back + 360) % 360;
  return td <= 180 ? td : 360 - td;
}

/* One step's routing context */
typedef struct {
  const orc_graph* g;
  const mode_data* md;
  int time_on;      /* the step's time bound is active: t components are tracked */
  int64_t bt;       /* the time bound, 0.1 s */
  int64_t bmm;      /* the distance bound, mm */
} rctx;

/* a label is feasible when its route keeps every bound (the search prunes the others) */
static int feasible(const rctx* X, rkey L) {
  return L.d <= X->bmm && (!X->time_on || L.t <= X->bt) && L.k - L.d <= ORC_TCCAP;
}

/* label L extended by edge e (and, with turn costs, by the turn from in-edge turn_from
 * into e); `frac_mm`/`frac_t` >= 0 replace the whole edge by a part of it (a target's
 * entry part) */
static rkey step_key(const rctx* X, rkey L, uint32_t e, int turn_from /* in-edge or -1 */) {
  rkey k;
  const int64_t len = (int64_t)X->g->len_mm[e];
  const int64_t c = (X->md->turn_on && turn_from >= 0) ? X->md->turn[turn_degree(X->g, (uint32_t)turn_from, e)] : 0;
  k.d = L.d + len;
  k.k = L.k + len + c;
  k.t = X->time_on ? L.t + (int64_t)X->md->time_ds[e] : 0;
  return k;
}

/* The source candidate's start label: the exit part of its edge (length, time) */
static rkey start_key(const rctx* X, uint32_t ei, double pi) {
  rkey L;
  L.d = part_mm(1.0 - pi, X->g->len_mm[ei]);
  L.k = L.d;
  L.t = X->time_on ? part_mm(1.0 - pi, X->md->time_ds[ei]) : 0;
  return L;
}

/* Label-setting search (binary heap, lexicographic (k, d, t)) from source candidate
 * (ei, pi), pruning infeasible relaxations.  Node mode (turn costs off): states are
 * nodes, the root node dst(ei) starts with the exit part.  Edge mode (turn costs on):
 * states are edges (arrived at dst(e) through e), the root state is edge ei; moving from
 * a to b adds turn(a, b). */
static void search(const rctx* X, uint32_t ei, double pi, nodemap_t* m) {
  const orc_graph* g = X->g;
  const int edge_mode = X->md->turn_on;
  m->n = 0;
  memset(m->key, 0xFF, m->cap * sizeof(uint32_t));
  const rkey L0 = start_key(X, ei, pi);
  if (!feasible(X, L0)) return;
  const uint32_t root = edge_mode ? ei : g->edge_dst[ei];
  heap_t hp = {0};
  int nw;
  uint32_t s = nm_insert(m, root, &nw);
  m->lab[s] = L0;
  heap_item it0 = {L0, root};
  hpush(&hp, it0);
  while (hp.n) {
    heap_item it = hpop(&hp);
    uint32_t su = nm_find(m, it.id);
    if (m->done[su] || !rk_eq(it.k, m->lab[su])) continue;
    m->done[su] = 1;
    const rkey L = m->lab[su];
    const uint32_t u = edge_mode ? g->edge_dst[it.id] : it.id;
    for (uint32_t e = g->node_row[u]; e < g->node_row[u + 1]; ++e) {
      if (!(g->edge_attr[e] & X->md->mode_bit)) continue;
      const rkey k = step_key(X, L, e, edge_mode ? (int)it.id : -1);
      if (!feasible(X, k)) continue; /* pruned during the search */
      const uint32_t id = edge_mode ? e : g->edge_dst[e];
      uint32_t sv = nm_insert(m, id, &nw);
      if (rk_lt(k, m->lab[sv])) {
        m->lab[sv] = k;
        heap_item x = {k, id};
        hpush(&hp, x);
      }
    }
  }
  free(hp.d);
}

/* the entry part of target edge ej appended to label L (after the turn into ej) */
static rkey entry_key(const rctx* X, rkey L, uint32_t ej, double pj, int64_t turn) {
  rkey r;
  const int64_t dp = part_mm(pj, X->g->len_mm[ej]);
  r.d = L.d + dp;
  r.k = L.k + turn + dp;
  r.t = X->time_on ? L.t + part_mm(pj, X->md->time_ds[ej]) : 0;
  return r;
}

/* Route to target (ej, pj) of the search rooted at source edge ei:
 * the target is a state whose offers come from v = src(ej): node mode v's label; edge
 * mode every labelled in-edge a of v with the turn (a, ej) — the lexicographic minimum
 * over the FEASIBLE offers (entry part included), smallest a among equals (*via). */
static int target_key(const rctx* X, const nodemap_t* m, uint32_t ej, double pj, rkey* out, uint32_t* via) {
  const orc_graph* g = X->g;
  const uint32_t v = g->edge_src[ej];
  if (!X->md->turn_on) {
    uint32_t s = nm_find(m, v);
    if (s == 0xFFFFFFFFu) return 0;
    const rkey r = entry_key(X, m->lab[s], ej, pj, 0);
    if (!feasible(X, r)) return 0;
    *out = r;
    return 1;
  }
  int found = 0;
  rkey best = {0, 0, 0};
  uint32_t bid = 0xFFFFFFFFu;
  for (uint32_t q = g->rev_row[v]; q < g->rev_row[v + 1]; ++q) {
    const uint32_t a = g->rev_edge[q];
    const uint32_t s = nm_find(m, a);
    if (s == 0xFFFFFFFFu) continue;
    const rkey r = entry_key(X, m->lab[s], ej, pj, X->md->turn[turn_degree(g, a, ej)]);
    if (!feasible(X, r)) continue;
    if (!found || rk_lt(r, best) || (rk_eq(r, best) && a < bid)) {
      best = r;
      bid = a;
      found = 1;
    }
  }
  if (found) {
    *out = best;
    *via = bid;
  }
  return found;
}

/* route of a transition: same edge forward: the part between the two
 * fractions (valid when within the bounds); else the target's label in the search from
 * (ei, pi).  Returns 1 when a valid route exists. */
static int route_of(const rctx* X, const nodemap_t* m, uint32_t ei, double pi, uint32_t ej, double pj,
                    rkey* out) {
  const orc_graph* g = X->g;
  if (ej == ei && pj >= pi) {
    rkey r;
    r.d = part_mm(pj - pi, g->len_mm[ei]);
    r.k = r.d;
    r.t = X->time_on ? part_mm(pj - pi, X->md->time_ds[ei]) : 0;
    *out = r;
    return feasible(X, r);
  }
  uint32_t via;
  return target_key(X, m, ej, pj, out, &via);
}

/* the step's routing context: distance bound from the great-circle distance, time
 * bound max_route_time_factor * (time difference), 0.1 s */
static void step_ctx(rctx* X, const orc_graph* g, const mode_data* md, const orc_params* P, double gcd,
                     int64_t dt) {
  X->g = g;
  X->md = md;
  const double gfl = gcd > P->interpolation_distance ? gcd : P->interpolation_distance;
  double bound = P->max_route_distance_factor * gfl;
  if (bound > P->breakage_distance) bound = P->breakage_distance;
  X->bmm = bound_mm_of(bound);
  X->time_on = 0;
  X->bt = 0;
  if (P->max_route_time_factor > 0.0 && dt > 0) {
    const double b = floor(P->max_route_time_factor * (double)dt * 10.0);
    if (b <= (double)ORC_TB_MAX) {
      X->time_on = 1;
      X->bt = (int64_t)b;
    }
  }
}

/* winner path: edges strictly between ei and ej, walking back from ej
 * through the smallest-id in-edge (in-state) whose final label extended by the step is
 * exactly the label reached.  Appends to *path in travel order. */
typedef VEC(uint32_t) u32vec;
static int walk_path(const rctx* X, const nodemap_t* m, uint32_t ei, uint32_t ej, double pj, u32vec* path) {
  const orc_graph* g = X->g;
  u32vec rev = {0};
  int ok = 1;
  if (!X->md->turn_on) {
    const uint32_t S = g->edge_dst[ei];
    uint32_t v = g->edge_src[ej];
    while (v != S && rev.n <= g->h.n_nodes) {
      const uint32_t sv = nm_find(m, v);
      if (sv == 0xFFFFFFFFu) {
        ok = 0;
        break;
      }
      const rkey Lv = m->lab[sv];
      uint32_t best_e = 0xFFFFFFFFu;
      for (uint32_t r = g->rev_row[v]; r < g->rev_row[v + 1]; ++r) {
        const uint32_t ed = g->rev_edge[r];
        if (!(g->edge_attr[ed] & X->md->mode_bit)) continue;
        const uint32_t su = nm_find(m, g->edge_src[ed]);
        if (su == 0xFFFFFFFFu) continue;
        if (rk_eq(step_key(X, m->lab[su], ed, -1), Lv) && ed < best_e) best_e = ed;
      }
      if (best_e == 0xFFFFFFFFu) {
        ok = 0;
        break;
      }
      VPUSH(rev, best_e);
      v = g->edge_src[best_e];
    }
  } else {
    rkey L;
    uint32_t a;
    if (!target_key(X, m, ej, pj, &L, &a)) ok = 0;
    while (ok && a != ei && rev.n <= g->h.n_edges) {
      VPUSH(rev, a);
      const uint32_t sa = nm_find(m, a);
      const rkey La = m->lab[sa];
      const uint32_t v = g->edge_src[a];
      uint32_t best = 0xFFFFFFFFu;
      for (uint32_t r = g->rev_row[v]; r < g->rev_row[v + 1]; ++r) {
        const uint32_t p = g->rev_edge[r];
        const uint32_t sp = nm_find(m, p);
        if (sp == 0xFFFFFFFFu) continue;
        if (rk_eq(step_key(X, m->lab[sp], a, (int)p), La) && p < best) best = p;
      }
      if (best == 0xFFFFFFFFu) {
        ok = 0;
        break;
      }
      a = best;
    }
  }
  for (size_t z = rev.n; ok && z-- > 0;) VPUSH(*path, rev.d[z]);
  free(rev.d);
  return ok;
}

int orc_edge_info(const orc_graph* g, const orc_params* p, uint32_t edge, int32_t* h_begin, int32_t* h_end,
                  int64_t* time_ds) {
  if (edge >= g->h.n_edges) return 0;
  *h_begin = g->h_begin[edge];
  *h_end = g->h_end[edge];
  *time_ds = edge_time_ds(g, p, edge);
  return 1;
}

int orc_route(const orc_graph* g, const orc_params* p, int mode, uint32_t src_edge, double src_p, uint32_t dst_edge,
              double dst_p, double bound, int64_t dt_sec, double* out_dist, int64_t* out_time_ds,
              int64_t* out_turn_mm) {
  mode_data md;
  mode_data_init(g, p, mode, &md);
  rctx X;
  /* bound given directly: a great-circle distance whose bound it is */
  orc_params q = *p;
  q.max_route_distance_factor = 1.0;
  q.interpolation_distance = 0.0;
  q.breakage_distance = bound;
  step_ctx(&X, g, &md, &q, bound, dt_sec);
  nodemap_t m;
  nm_init(&m, 1024);
  if (!(dst_edge == src_edge && dst_p >= src_p)) search(&X, src_edge, src_p, &m);
  rkey r;
  const int ok = route_of(&X, &m, src_edge, src_p, dst_edge, dst_p, &r);
  nm_free(&m);
  free(md.time_ds);
  *out_dist = ok ? (double)r.d / 1000.0 : INFINITY;
  *out_time_ds = ok ? r.t : -1;
  *out_turn_mm = ok ? r.k - r.d : -1;
  return ok;
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
  const orc_params* p;   /* ORC_MODES parameter sets */
  const mode_data* md;   /* ORC_MODES routing data */
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

/* queue_length (README.md:283,295: "the distance from the end of the segment where the
 * speed drops below the threshold"): the state-to-state piece holding the
 * segment's exit position s1 and the slow pieces right before it, clipped to [s0, s1];
 * a piece is slow when its mean speed (route mm over the state times) is below
 * queue_kph.  Whole metres, half up. */
static int piece_slow(const int64_t* pos, const double* tm, int k, double kph) {
  return (double)(pos[k + 1] - pos[k]) * 0.0036 < kph * (tm[k + 1] - tm[k]);
}
static int32_t queue_at(const int64_t* pos, const double* tm, int n, int64_t s0, int64_t s1, double kph) {
  if (n < 2) return 0;
  int k = 0;
  while (k < n - 2 && s1 > pos[k + 1]) ++k;
  if (!piece_slow(pos, tm, k, kph)) return 0;
  while (k > 0 && pos[k] > s0 && piece_slow(pos, tm, k - 1, kph)) --k;
  const int64_t q0 = pos[k] > s0 ? pos[k] : s0;
  return (int32_t)((s1 - q0 + 500) / 1000);
}

static void match_trace(job_t* J, int32_t t) {
  const orc_graph* g = J->g;
  const int mode = J->mode[t] < ORC_MODES ? J->mode[t] : 0;
  const orc_params* P = &J->p[mode];
  const mode_data* MD = &J->md[mode];
  trace_out* O = &J->outs[t];
  memset(O, 0, sizeof(*O));
  const int64_t b = J->trace_off[t], n = J->trace_off[t + 1] - b;
  const double *lat = J->lat + b, *lon = J->lon + b;
  const int64_t* tm = J->time + b;
  const uint32_t mode_bit = MD->mode_bit;
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
    rctx X;
    step_ctx(&X, g, MD, P, gcd, tm[ib] - tm[ia]);
    for (int i = 0; i < Ka; ++i) {
      for (int j = 0; j < Kb; ++j) trans[i * ORC_KMAX + j] = INFINITY;
      if (forced) continue;
      int need = 0;
      for (int j = 0; j < Kb; ++j)
        if (!(cb[j].e == ca[i].e && cb[j].p >= ca[i].p)) need = 1;
      /* one search per source candidate: its exit part counts toward the bounds that
       * prune the search */
      if (need) search(&X, ca[i].e, ca[i].p, &nm);
      for (int j = 0; j < Kb; ++j) {
        rkey r;
        if (route_of(&X, &nm, ca[i].e, ca[i].p, cb[j].e, cb[j].p, &r))
          trans[i * ORC_KMAX + j] = ((double)(r.k - r.d) / 1000.0 + fabs((double)r.d / 1000.0 - gcd)) * inv_beta;
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
        rctx X;
        step_ctx(&X, g, MD, P, gcd, tm[ib] - tm[ia]);
        search(&X, ci->e, ci->p, &nm);
        u32vec path = {0};
        walk_path(&X, &nm, ci->e, cj->e, cj->p, &path); /* the winner's route is valid by construction */
        for (size_t z = 0; z < path.n; ++z) {
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
        VPUSH(O->seg_queue, et != -1.0 ? queue_at(pos, stm, nst, s0, s1, P->queue_kph) : 0);
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
  /* per-mode route times and turn tables (only for the modes present) */
  mode_data md[ORC_MODES];
  memset(md, 0, sizeof(md));
  for (int m = 0; m < ORC_MODES; ++m) {
    int used = 0;
    for (int32_t t = 0; t < n_traces && !used; ++t) used = (mode[t] < ORC_MODES ? mode[t] : 0) == m;
    if (used) mode_data_init(g, &p[m], m, &md[m]);
    else md[m].mode_bit = 1u << m;
  }
  J.md = md;
  J.outs = (trace_out*)calloc((size_t)n_traces + 1, sizeof(trace_out));
  pthread_mutex_init(&J.mu, NULL);
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
  for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &J);
  for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&J.mu);
  for (int m = 0; m < ORC_MODES; ++m) free(md[m].time_ds);
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
