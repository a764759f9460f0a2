/*
 * edge_stats.c — design statistics of the edge-state (turn-cost) route searches, on the
 * CPU.  Includes the oracle's translation unit (TEST/ANALYSIS INFRASTRUCTURE ONLY, never
 * the product) and simulates the GPU's exact-round search (otr_edge.h edge_search: IN
 * criterion k < kmin + gap(state), early exit once every target is resolved) for every
 * source candidate of every step of a trace sample, reporting what sizes the LDS tiers:
 * table keys per search, settled states, rounds, and per step the union of the sources'
 * states (what a multi-source search would hold).
 *
 * Build: gcc -O2 -shared -fPIC -o tools/libedgestats.so tools/edge_stats.c -lm -lpthread
 * Use:   python tools/edge_stats.py
 */
#include "../oracle/oracle.c"

typedef struct {
  int64_t searches, keys, settled, rounds, rounds_tmin, settled_tmin, steps, union_keys, sum_keys, sources;
  int64_t union_settle_events, sum_settle_events; /* (state, round) pairs: combined vs separate */
  int64_t hist_keys[64];                          /* keys per search, 32-key buckets */
  int64_t hist_union[64];                         /* union keys per step, 64-key buckets */
  int64_t hist_rounds[64];                        /* rounds per search */
  int64_t pend_max, max_rounds_sum, relaxed, groups;
  int64_t hist_bmm_keys[24][24]; /* [route bound / 100 m][keys / 32] */
  int64_t settled_out, rounds_out, scans_tmin, scans_out; /* + the OUT criterion; pending entries examined */
  int64_t settled_tterm, rounds_tterm;                     /* + the time-bound target resolution */
  int64_t settled_ast, rounds_ast, settled_ast1, rounds_ast1; /* + A* lower-bound resolution: per target / one anchor */
} es_stats;

typedef struct {
  uint32_t* stamp; /* per edge: generation of the search that touched it */
  rkey* lab;
  uint8_t* flag; /* 1 pending, 2 settled */
  uint32_t* ustamp; /* per edge: step generation (union) */
  uint64_t* umask;  /* per edge: rounds (< 64) in which some source of the step settled it */
  uint32_t gen, ugen;
  int64_t ukeys, uevents;
  uint32_t* pend;
  uint32_t* nxt;
} es_ws;

static const int64_t kInf = INT64_MAX / 4;

static void es_touch(es_ws* W, uint32_t e) {
  if (W->ustamp[e] != W->ugen) {
    W->ustamp[e] = W->ugen;
    W->umask[e] = 0;
    W->ukeys++;
  }
}


/* A* lower-bound target resolution (analysis): planar chord metric, rho_d / rho_t = the
 * smallest length / time per chord-mm over every edge, so every path's length (time) is
 * >= rho * the chord between its ends */
static double g_rho_d, g_rho_t, g_kx, g_ky;
static double pl_chord_mm(const orc_graph* g, uint32_t u, uint32_t v) {
  const double dx = (double)(g->node_ll[2 * u + 1] - g->node_ll[2 * v + 1]) * g_kx;
  const double dy = (double)(g->node_ll[2 * u] - g->node_ll[2 * v]) * g_ky;
  return sqrt(dx * dx + dy * dy);
}
static int g_ast; /* 1: per-target anchors, 2: one anchor (the first needed target's node) */
static uint32_t g_anchor;
static int g_tterm; /* also resolve a target once every pending label's time + its entry time breaks the bound */

/* one simulated search; returns keys; *settled, *rounds out */
static int64_t es_search(const rctx* X, es_ws* W, uint32_t ei, double pi, int ntg, const uint32_t* tv,
                         const int64_t* tpart, const int64_t* tpt, const uint32_t* tej, int64_t tmin,
                         int64_t* settled, int64_t* rounds, int64_t* relaxed, int64_t* pend_max, int record,
                         const int64_t* minout, int64_t* scans) {
  const orc_graph* g = X->g;
  const mode_data* md = X->md;
  *settled = 0;
  *rounds = 0;
  const int64_t d0 = part_mm(1.0 - pi, g->len_mm[ei]);
  const int64_t t0 = X->time_on ? part_mm(1.0 - pi, md->time_ds[ei]) : 0;
  if (d0 > X->bmm || (X->time_on && t0 > X->bt)) return 0;
  const int64_t pd = X->bmm - d0, pt = X->time_on ? X->bt - t0 : kInf;
  W->gen++;
  int64_t keys = 1;
  uint32_t np = 0;
  W->stamp[ei] = W->gen;
  W->lab[ei] = (rkey){0, 0, 0};
  W->flag[ei] = 1;
  W->pend[np++] = ei;
  if (record) es_touch(W, ei);
  rkey tl[ORC_KMAX];
  for (int j = 0; j < ntg; ++j) tl[j] = (rkey){kInf, kInf, kInf};
  int64_t kmin = 0, dmin = 0, tminp = 0;
  for (;;) {
    if (np == 0) break;
    int unres = 0;
    for (int j = 0; j < ntg; ++j) {
      if (tv[j] == 0xFFFFFFFFu) continue;
      int res = (tl[j].k < kInf && tl[j].k < kmin + tpart[j] + tmin) || dmin + tpart[j] > pd ||
                      (g_tterm && X->time_on && tminp + tpt[j] > pt);
      if (!res && g_ast) {
        /* every later offer to j descends from a pending state b (head v): length >= d(b) +
           rho_d * chord(v, src(j)), time likewise */
        double ad = 1e300, at = 1e300;
        const uint32_t anc = g_ast == 1 ? tv[j] : g_anchor;
        const double rj = g_ast == 1 ? 0.0 : pl_chord_mm(g, g_anchor, tv[j]);
        for (uint32_t q = 0; q < np; ++q) {
          const uint32_t b = W->pend[q];
          const double ch = pl_chord_mm(g, g->edge_dst[b], anc) - rj;
          const double xd = (double)W->lab[b].d + g_rho_d * ch, xt = (double)W->lab[b].t + g_rho_t * ch;
          if (xd < ad) ad = xd;
          if (xt < at) at = xt;
        }
        if (ad + (double)tpart[j] > (double)pd + 1e-3 || (X->time_on && at + (double)tpt[j] > (double)pt + 1e-3)) res = 1;
      }
      if (!res) unres = 1;
    }
    if (!unres) break;
    const int64_t r = *rounds;
    ++*rounds;
    int64_t knext = kInf, dnext = kInf, tnext = kInf;
    uint32_t nf = 0, kept = 0;
    /* OUT criterion (minout != NULL): every later offer leaves a pending state u through
       one of its head's out-edges: key >= k(u) + minout(head(u)) + tmin */
    int64_t othr = minout ? kInf : -1; /* (-1: no state passes by OUT alone) */
    if (minout)
      for (uint32_t q = 0; q < np; ++q) {
        const uint32_t b = W->pend[q];
        const int64_t o = W->lab[b].k + minout[g->edge_dst[b]] + tmin;
        if (o < othr) othr = o;
      }
    if (scans) *scans += np;
    for (uint32_t q = 0; q < np; ++q) {
      const uint32_t b = W->pend[q];
      const int64_t len = b == ei ? 0 : (int64_t)g->len_mm[b];
      const int64_t mq = len >> 8 < 255 ? len >> 8 : 255;
      const int64_t gap = (mq ? mq << 8 : 1) + (b == ei ? 0 : tmin);
      if (W->lab[b].k < kmin + gap || W->lab[b].k < othr) W->nxt[nf++] = b;
      else {
        W->pend[kept++] = b;
        if (W->lab[b].k < knext) knext = W->lab[b].k;
        if (W->lab[b].d < dnext) dnext = W->lab[b].d;
        if (W->lab[b].t < tnext) tnext = W->lab[b].t;
      }
    }
    np = kept;
    for (uint32_t f = 0; f < nf; ++f) {
      const uint32_t b = W->nxt[f];
      W->flag[b] = 2;
      ++*settled;
      if (record && r < 64 && !(W->umask[b] >> r & 1)) {
        W->umask[b] |= 1ull << r;
        W->uevents++;
      }
      const rkey L = W->lab[b];
      const uint32_t v = g->edge_dst[b];
      for (int j = 0; j < ntg; ++j)
        if (tv[j] == v) {
          const int64_t c = md->turn[turn_degree(g, b, tej[j])];
          rkey o = {L.k + tpart[j] + c, L.d + tpart[j], X->time_on ? L.t + tpt[j] : 0};
          if (o.d <= pd && o.t <= pt && o.k - o.d <= ORC_TCCAP && rk_lt(o, tl[j])) tl[j] = o;
        }
      for (uint32_t e = g->node_row[v]; e < g->node_row[v + 1]; ++e) {
        if (!(g->edge_attr[e] & md->mode_bit)) continue;
        ++*relaxed;
        const int64_t c = md->turn[turn_degree(g, b, e)];
        rkey o = {L.k + g->len_mm[e] + c, L.d + g->len_mm[e], X->time_on ? L.t + md->time_ds[e] : 0};
        if (!(o.d <= pd && o.t <= pt && o.k - o.d <= ORC_TCCAP)) continue;
        if (W->stamp[e] != W->gen) {
          W->stamp[e] = W->gen;
          W->lab[e] = (rkey){kInf, kInf, kInf};
          W->flag[e] = 0;
          ++keys;
          if (record) es_touch(W, e);
        }
        if (rk_lt(o, W->lab[e])) {
          W->lab[e] = o;
          if (o.k < knext) knext = o.k;
          if (o.d < dnext) dnext = o.d;
          if (o.t < tnext) tnext = o.t;
          if (W->flag[e] == 0) {
            W->flag[e] = 1;
            W->pend[np++] = e;
          }
        }
      }
    }
    if (np > *pend_max) *pend_max = np;
    kmin = knext;
    dmin = dnext;
    tminp = tnext;
  }
  return keys;
}

int es_run(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off, const double* lat,
           const double* lon, const int64_t* tms, int group, es_stats* S) {
  memset(S, 0, sizeof(*S));
  const uint32_t E = g->h.n_edges;
  es_ws W;
  memset(&W, 0, sizeof(W));
  W.stamp = calloc(E + 1, 4);
  W.lab = malloc(sizeof(rkey) * (E + 1));
  W.flag = calloc(E + 1, 1);
  W.ustamp = calloc(E + 1, 4);
  W.umask = calloc(E + 1, 8);
  W.pend = malloc(4 * (size_t)(E + 1));
  W.nxt = malloc(4 * (size_t)(E + 1));
  mode_data md;
  mode_data_init(g, &p[0], 0, &md);
  {
    double lat0 = 0;
    for (uint32_t v = 0; v < g->h.n_nodes; ++v) lat0 += g->node_ll[2 * v] * 1e-6;
    lat0 /= g->h.n_nodes;
    g_ky = kM * 1e-6 * 1000.0;
    g_kx = kM * 1e-6 * 1000.0 * cos_deg(lat0) * 0.98; /* (margin for the latitude spread) */
    g_rho_d = 1e300;
    g_rho_t = 1e300;
    int64_t zt = 0;
    for (uint32_t e = 0; e < E; ++e) {
      if (!(g->edge_attr[e] & md.mode_bit)) continue;
      const double ch = pl_chord_mm(g, g->edge_src[e], g->edge_dst[e]);
      if (ch <= 0) continue;
      const double rd = (double)g->len_mm[e] / ch, rt = (double)md.time_ds[e] / ch;
      if (rd < g_rho_d) g_rho_d = rd;
      if (rt < g_rho_t) g_rho_t = rt;
      if (md.time_ds[e] == 0) zt++;
    }
    fprintf(stderr, "rho_d %.6f rho_t %.8f (1/rho_t %.1f mm per 0.1 s) zero-time edges %lld\n", g_rho_d, g_rho_t,
            1.0 / g_rho_t, (long long)zt);
  }
  int64_t tmin = md.turn[0];
  for (int i = 0; i <= 180; ++i)
    if (md.turn[i] < tmin) tmin = md.turn[i];
  /* per node: the shortest out-edge the mode may use (quantized down to 256 mm) */
  int64_t* minout = malloc(8 * (size_t)(g->h.n_nodes + 1));
  for (uint32_t v = 0; v < g->h.n_nodes; ++v) {
    int64_t m = kInf / 2;
    for (uint32_t e = g->node_row[v]; e < g->node_row[v + 1]; ++e)
      if ((g->edge_attr[e] & md.mode_bit) && (int64_t)g->len_mm[e] < m) m = g->len_mm[e];
    minout[v] = m >= kInf / 2 ? m : (m >> 8) << 8;
  }
  const int kmax = p[0].max_candidates < ORC_KMAX ? p[0].max_candidates : ORC_KMAX;
  static cand_t cands[4096][ORC_KMAX];
  static int kc[4096], act[4096];
  static int64_t sp[4096];
  for (int32_t t = 0; t < n_traces; ++t) {
    const int64_t b = trace_off[t], n = trace_off[t + 1] - b;
    int ns = 0;
    int64_t last = 0;
    for (int64_t i = 0; i < n && ns < 4096; ++i) {
      int st = i == 0 || i == n - 1 ||
               gc_dist(lat[b + last], lon[b + last], lat[b + i], lon[b + i]) >= p[0].interpolation_distance;
      if (st) {
        last = i;
        sp[ns++] = b + i;
      }
    }
    int na = 0;
    for (int s = 0; s < ns; ++s) {
      double a = p[0].gps_accuracy;
      double radius = p[0].search_radius > a ? p[0].search_radius : a;
      if (radius > p[0].max_search_radius) radius = p[0].max_search_radius;
      kc[s] = find_candidates(g, lat[sp[s]], lon[sp[s]], radius, md.mode_bit, kmax, cands[s]);
      if (kc[s] > 0) act[na++] = s;
    }
    for (int k = 1; k < na; ++k) {
      const int sa = act[k - 1], sb = act[k];
      const double gcd = gc_dist(lat[sp[sa]], lon[sp[sa]], lat[sp[sb]], lon[sp[sb]]);
      if (gcd > p[0].breakage_distance) continue;
      rctx X;
      step_ctx(&X, g, &md, &p[0], gcd, tms[sp[sb]] - tms[sp[sa]]);
      uint32_t tv[ORC_KMAX], tej[ORC_KMAX];
      int64_t tpart[ORC_KMAX], tpt[ORC_KMAX];
      const int Kb = kc[sb];
      W.ugen++;
      W.ukeys = 0;
      W.uevents = 0;
      int64_t step_sum = 0, nsrc = 0, max_rounds = 0;
      for (int i = 0; i < kc[sa]; ++i) {
        const cand_t* ci = &cands[sa][i];
        int need = 0;
        for (int j = 0; j < Kb; ++j) {
          const cand_t* cj = &cands[sb][j];
          const int nd = !(cj->e == ci->e && cj->p >= ci->p);
          tv[j] = nd ? g->edge_src[cj->e] : 0xFFFFFFFFu;
          tej[j] = cj->e;
          tpart[j] = part_mm(cj->p, g->len_mm[cj->e]);
          tpt[j] = X.time_on ? part_mm(cj->p, md.time_ds[cj->e]) : 0;
          need |= nd;
        }
        if (!need) continue;
        if (group > 0 && nsrc > 0 && nsrc % group == 0) { /* a new group: its own union */
          S->union_keys += W.ukeys;
          S->union_settle_events += W.uevents;
          S->hist_union[W.ukeys / 64 < 63 ? W.ukeys / 64 : 63]++;
          S->groups++;
          W.ugen++;
          W.ukeys = 0;
          W.uevents = 0;
        }
        int64_t st, rd, st2, rd2, rl = 0, rl2 = 0;
        const int64_t keys =
            es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, 0, &st, &rd, &rl, &S->pend_max, 1, NULL, NULL);
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st2, &rd2, &rl2, &S->pend_max, 0, NULL,
                        &S->scans_tmin);
        int64_t st3, rd3, rl3 = 0;
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st3, &rd3, &rl3, &S->pend_max, 0, minout,
                        &S->scans_out);
        if (getenv("ES_DEBUG") && (st3 != st2 || rd3 != rd2)) {
          static int shown = 0;
          if (shown++ < 5) fprintf(stderr, "search %lld: tmin st %lld rd %lld | out st %lld rd %lld\n",
                                   (long long)S->searches, (long long)st2, (long long)rd2, (long long)st3, (long long)rd3);
        }
        S->settled_out += st3;
        S->rounds_out += rd3;
        g_tterm = 1;
        int64_t st4, rd4, rl4 = 0;
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st4, &rd4, &rl4, &S->pend_max, 0, NULL, NULL);
        int64_t st5, rd5, rl5 = 0, st6, rd6, rl6 = 0;
        g_ast = 1;
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st5, &rd5, &rl5, &S->pend_max, 0, NULL, NULL);
        g_ast = 2;
        g_anchor = 0xFFFFFFFFu;
        for (int j = 0; j < Kb && g_anchor == 0xFFFFFFFFu; ++j) if (tv[j] != 0xFFFFFFFFu) g_anchor = tv[j];
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st6, &rd6, &rl6, &S->pend_max, 0, NULL, NULL);
        g_ast = 0;
        S->settled_ast += st5;
        S->rounds_ast += rd5;
        S->settled_ast1 += st6;
        S->rounds_ast1 += rd6;
        g_tterm = 0;
        S->settled_tterm += st4;
        S->rounds_tterm += rd4;
        S->searches++;
        S->keys += keys;
        S->settled += st;
        S->relaxed += rl;
        S->rounds += rd;
        S->settled_tmin += st2;
        S->rounds_tmin += rd2;
        S->sum_settle_events += st;
        S->hist_keys[keys / 32 < 63 ? keys / 32 : 63]++;
        {
          const int64_t bb = X.bmm / 100000 < 23 ? X.bmm / 100000 : 23, kb = keys / 32 < 23 ? keys / 32 : 23;
          S->hist_bmm_keys[bb][kb]++;
        }
        S->hist_rounds[rd < 63 ? rd : 63]++;
        step_sum += keys;
        nsrc++;
        if (rd > max_rounds) max_rounds = rd;
      }
      if (!nsrc) continue;
      S->steps++;
      S->sum_keys += step_sum;
      S->union_keys += W.ukeys;
      S->union_settle_events += W.uevents;
      S->hist_union[W.ukeys / 64 < 63 ? W.ukeys / 64 : 63]++;
      S->groups++;
      S->sources += nsrc;
      S->max_rounds_sum += max_rounds;
    }
  }
  free(W.stamp);
  free(W.lab);
  free(W.flag);
  free(W.ustamp);
  free(W.umask);
  free(W.pend);
  free(W.nxt);
  free(minout);
  free(md.time_ds);
  return 0;
}

/* Viterbi-side pruning statistics (analysis): with step t-1's accumulated costs known,
 * how many source candidates of step t need a search at all?  Sources in ascending cost
 * order; a source is skippable when its cost is infinite (no predecessor reached it) or
 * when every target already has a cheaper offer U_j < cost(i) (transitions are >= 0). */
typedef struct {
  int64_t steps, sources, inf_sources, skip_local, searched_local, brk;
} vp_stats;

int vp_run(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off, const double* lat,
           const double* lon, const int64_t* tms, vp_stats* S) {
  memset(S, 0, sizeof(*S));
  mode_data md;
  mode_data_init(g, &p[0], 0, &md);
  const double inv2s2 = 1.0 / (p[0].sigma_z * p[0].sigma_z * 2.0), inv_beta = 1.0 / p[0].beta;
  const int kmax = p[0].max_candidates < ORC_KMAX ? p[0].max_candidates : ORC_KMAX;
  static cand_t cands[4096][ORC_KMAX];
  static int kc[4096], act[4096];
  static int64_t sp[4096];
  nodemap_t nm;
  nm_init(&nm, 1024);
  double trans[ORC_KMAX * ORC_KMAX];
  for (int32_t t = 0; t < n_traces; ++t) {
    const int64_t b = trace_off[t], n = trace_off[t + 1] - b;
    int ns = 0;
    int64_t last = 0;
    for (int64_t i = 0; i < n && ns < 4096; ++i) {
      int st = i == 0 || i == n - 1 ||
               gc_dist(lat[b + last], lon[b + last], lat[b + i], lon[b + i]) >= p[0].interpolation_distance;
      if (st) {
        last = i;
        sp[ns++] = b + i;
      }
    }
    int na = 0;
    for (int s = 0; s < ns; ++s) {
      double a = p[0].gps_accuracy;
      double radius = p[0].search_radius > a ? p[0].search_radius : a;
      if (radius > p[0].max_search_radius) radius = p[0].max_search_radius;
      kc[s] = find_candidates(g, lat[sp[s]], lon[sp[s]], radius, md.mode_bit, kmax, cands[s]);
      if (kc[s] > 0) act[na++] = s;
    }
    double cost[ORC_KMAX], ncost[ORC_KMAX];
    if (na > 0)
      for (int j = 0; j < kc[act[0]]; ++j) cost[j] = cands[act[0]][j].d2 * inv2s2;
    for (int k = 1; k < na; ++k) {
      const int sa = act[k - 1], sb = act[k];
      const int Ka = kc[sa], Kb = kc[sb];
      const cand_t *ca = cands[sa], *cb = cands[sb];
      const double gcd = gc_dist(lat[sp[sa]], lon[sp[sa]], lat[sp[sb]], lon[sp[sb]]);
      const int forced = gcd > p[0].breakage_distance;
      rctx X;
      step_ctx(&X, g, &md, &p[0], gcd, tms[sp[sb]] - tms[sp[sa]]);
      int needed[ORC_KMAX];
      for (int i = 0; i < Ka; ++i) {
        for (int j = 0; j < Kb; ++j) trans[i * ORC_KMAX + j] = INFINITY;
        needed[i] = 0;
        if (forced) continue;
        int need = 0;
        for (int j = 0; j < Kb; ++j)
          if (!(cb[j].e == ca[i].e && cb[j].p >= ca[i].p)) need = 1;
        needed[i] = need;
        if (need) search(&X, ca[i].e, ca[i].p, &nm);
        for (int j = 0; j < Kb; ++j) {
          rkey r;
          if (route_of(&X, &nm, ca[i].e, ca[i].p, cb[j].e, cb[j].p, &r))
            trans[i * ORC_KMAX + j] = ((double)(r.k - r.d) / 1000.0 + fabs((double)r.d / 1000.0 - gcd)) * inv_beta;
        }
      }
      /* the statistics */
      if (!forced) {
        S->steps++;
        int ord[ORC_KMAX];
        for (int i = 0; i < Ka; ++i) ord[i] = i;
        for (int x = 1; x < Ka; ++x) /* insertion sort by (cost, index) */
          for (int y = x; y > 0 && cost[ord[y]] < cost[ord[y - 1]]; --y) {
            const int tmp = ord[y];
            ord[y] = ord[y - 1];
            ord[y - 1] = tmp;
          }
        double U[ORC_KMAX];
        for (int j = 0; j < Kb; ++j) U[j] = INFINITY;
        /* same-edge forward targets need no search: their offers count toward U first */
        for (int i = 0; i < Ka; ++i)
          for (int j = 0; j < Kb; ++j)
            if (cb[j].e == ca[i].e && cb[j].p >= ca[i].p && trans[i * ORC_KMAX + j] != INFINITY &&
                cost[i] != INFINITY && cost[i] + trans[i * ORC_KMAX + j] < U[j])
              U[j] = cost[i] + trans[i * ORC_KMAX + j];
        for (int x = 0; x < Ka; ++x) {
          const int i = ord[x];
          if (!needed[i]) continue;
          S->sources++;
          if (cost[i] == INFINITY) {
            S->inf_sources++;
            continue;
          }
          int skip = 1;
          for (int j = 0; j < Kb && skip; ++j) {
            if (cb[j].e == ca[i].e && cb[j].p >= ca[i].p) continue;
            if (!(U[j] < cost[i])) skip = 0;
          }
          if (skip) {
            S->skip_local++;
            continue;
          }
          S->searched_local++;
          for (int j = 0; j < Kb; ++j)
            if (trans[i * ORC_KMAX + j] != INFINITY && cost[i] + trans[i * ORC_KMAX + j] < U[j])
              U[j] = cost[i] + trans[i * ORC_KMAX + j];
        }
      }
      int any = 0;
      for (int j = 0; j < Kb; ++j) {
        double best = INFINITY;
        int bi = -1;
        for (int i = 0; i < Ka; ++i) {
          const double tr = trans[i * ORC_KMAX + j];
          if (tr == INFINITY || cost[i] == INFINITY) continue;
          const double c = cost[i] + tr;
          if (c < best) {
            best = c;
            bi = i;
          }
        }
        ncost[j] = bi >= 0 ? best + cb[j].d2 * inv2s2 : INFINITY;
        if (bi >= 0) any = 1;
      }
      if (!any) {
        S->brk++;
        for (int j = 0; j < Kb; ++j) ncost[j] = cb[j].d2 * inv2s2;
      }
      memcpy(cost, ncost, sizeof(cost));
    }
  }
  nm_free(&nm);
  free(md.time_ds);
  return 0;
}

/* Node-mode (no turn costs) search sizes with and without the A* target resolution
 * (analysis): a sequential label-setting search per source candidate; settled nodes until
 * every needed target is resolved — (a) the GPU's rule (its node settled, or no pending
 * length / time can still reach it), (b) + the chord lower bound of every pending node to
 * the target node (rho_d, rho_t as for the edge search). */
typedef struct {
  int64_t searches, settled_base, settled_astar, exhausted_base, exhausted_astar, settled_order, exhausted_order;
  int64_t settled_tt, exhausted_tt; /* mode 3: the base rule + the time rule (no feasible label and the
                                       smallest pending time + the entry time breaks the time bound) */
} ns_stats;
static double g_ns_c = 0.5; /* heuristic weight (of rho_d) of the A*-ordered variant */
void ns_set_c(double c) { g_ns_c = c; }

int ns_run(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off, const double* lat,
           const double* lon, const int64_t* tms, const float* acc, ns_stats* S) {
  memset(S, 0, sizeof(*S));
  const uint32_t E = g->h.n_edges, N = g->h.n_nodes;
  mode_data md;
  mode_data_init(g, &p[0], 0, &md);
  {
    double lat0 = 0;
    for (uint32_t v = 0; v < N; ++v) lat0 += g->node_ll[2 * v] * 1e-6;
    lat0 /= N;
    g_ky = kM * 1e-6 * 1000.0;
    g_kx = kM * 1e-6 * 1000.0 * cos_deg(lat0) * 0.98;
    g_rho_d = 1e300;
    g_rho_t = 1e300;
    for (uint32_t e = 0; e < E; ++e) {
      if (!(g->edge_attr[e] & md.mode_bit)) continue;
      const double ch = pl_chord_mm(g, g->edge_src[e], g->edge_dst[e]);
      if (ch <= 0) continue;
      if ((double)g->len_mm[e] / ch < g_rho_d) g_rho_d = (double)g->len_mm[e] / ch;
      if ((double)md.time_ds[e] / ch < g_rho_t) g_rho_t = (double)md.time_ds[e] / ch;
    }
  }
  const int kmax = p[0].max_candidates < ORC_KMAX ? p[0].max_candidates : ORC_KMAX;
  static cand_t cands[4096][ORC_KMAX];
  static int kc[4096], act[4096];
  static int64_t sp[4096];
  uint32_t* stamp = calloc(N + 1, 4);
  rkey* lab = malloc(sizeof(rkey) * (N + 1));
  uint8_t* done = calloc(N + 1, 1);
  uint32_t gen = 0;
  for (int32_t t = 0; t < n_traces; ++t) {
    const int64_t b = trace_off[t], n = trace_off[t + 1] - b;
    int ns = 0;
    int64_t last = 0;
    for (int64_t i = 0; i < n && ns < 4096; ++i) {
      int st = i == 0 || i == n - 1 ||
               gc_dist(lat[b + last], lon[b + last], lat[b + i], lon[b + i]) >= p[0].interpolation_distance;
      if (st) {
        last = i;
        sp[ns++] = b + i;
      }
    }
    int na = 0;
    for (int s = 0; s < ns; ++s) {
      double a = acc ? (double)acc[sp[s]] : p[0].gps_accuracy;
      double radius = p[0].search_radius > a ? p[0].search_radius : a;
      if (radius > p[0].max_search_radius) radius = p[0].max_search_radius;
      kc[s] = find_candidates(g, lat[sp[s]], lon[sp[s]], radius, md.mode_bit, kmax, cands[s]);
      if (kc[s] > 0) act[na++] = s;
    }
    for (int k = 1; k < na; ++k) {
      const int sa = act[k - 1], sb = act[k];
      const double gcd = gc_dist(lat[sp[sa]], lon[sp[sa]], lat[sp[sb]], lon[sp[sb]]);
      if (gcd > p[0].breakage_distance) continue;
      rctx X;
      step_ctx(&X, g, &md, &p[0], gcd, tms[sp[sb]] - tms[sp[sa]]);
      const int Kb = kc[sb];
      for (int i = 0; i < kc[sa]; ++i) {
        const cand_t* ci = &cands[sa][i];
        uint32_t tv[ORC_KMAX];
        int64_t tpart[ORC_KMAX], tpt[ORC_KMAX];
        int need = 0;
        for (int j = 0; j < Kb; ++j) {
          const cand_t* cj = &cands[sb][j];
          const int nd = !(cj->e == ci->e && cj->p >= ci->p);
          tv[j] = nd ? g->edge_src[cj->e] : 0xFFFFFFFFu;
          tpart[j] = part_mm(cj->p, g->len_mm[cj->e]);
          tpt[j] = X.time_on ? part_mm(cj->p, md.time_ds[cj->e]) : 0;
          need |= nd;
        }
        if (!need) continue;
        const rkey L0 = start_key(&X, ci->e, ci->p);
        if (!feasible(&X, L0)) continue;
        const int64_t pd = X.bmm, pt = X.time_on ? X.bt : kInf;
        S->searches++;
        /* the anchor: the target probe; R: the farthest target node from it */
        const uint32_t anc_dummy = 0;
        (void)anc_dummy;
        double Ax = 0, Ay = 0, R = 0;
        {
          const int64_t ib = sp[sb];
          Ax = lon[ib] * 1e6 * g_kx;
          Ay = lat[ib] * 1e6 * g_ky;
          for (int j = 0; j < Kb; ++j) {
            if (tv[j] == 0xFFFFFFFFu) continue;
            const double dx = (double)g->node_ll[2 * tv[j] + 1] * g_kx - Ax, dy = (double)g->node_ll[2 * tv[j]] * g_ky - Ay;
            const double r = sqrt(dx * dx + dy * dy);
            if (r > R) R = r;
          }
        }
#define NS_H(x) (mode == 2 ? g_ns_c * g_rho_d * fmax(0.0, sqrt(((double)g->node_ll[2 * (x) + 1] * g_kx - Ax) * ((double)g->node_ll[2 * (x) + 1] * g_kx - Ax) + ((double)g->node_ll[2 * (x)] * g_ky - Ay) * ((double)g->node_ll[2 * (x)] * g_ky - Ay)) - R - 1.0) : 0.0)
        for (int mode = 0; mode < 4; ++mode) {
          ++gen;
          heap_t hp = {0};
          const uint32_t root = g->edge_dst[ci->e];
          stamp[root] = gen;
          lab[root] = L0;
          done[root] = 0;
          heap_item it0 = {L0, root};
          if (mode == 2) it0.k.k = L0.k + (int64_t)NS_H(root);
          hpush(&hp, it0);
          int64_t settled = 0;
          int exhausted = 1;
          for (;;) {
            /* resolution check (every settle for the base rule, every 4 for A*) */
            if (hp.n == 0) break;
            int unres = 0;
            const rkey top = hp.d[0].k;
            for (int j = 0; j < Kb && !unres; ++j) {
              if (tv[j] == 0xFFFFFFFFu) continue;
              if (stamp[tv[j]] == gen && done[tv[j]]) continue;
              if ((mode < 2 || mode == 3) && top.d + tpart[j] > pd) continue;
              int r = 0;
              if (mode == 3 && X.time_on) {
                const int has = stamp[tv[j]] == gen && lab[tv[j]].t + tpt[j] <= pt;  /* a feasible label */
                if (!has) {
                  int64_t tmn = kInf;
                  for (size_t q = 0; q < hp.n; ++q)
                    if (hp.d[q].k.t < tmn) tmn = hp.d[q].k.t;
                  if (tmn + tpt[j] > pt) r = 1;
                }
              }
              if (mode >= 1 && (settled & 3) == 0) {
                double ad = 1e300, at = 1e300;
                for (size_t q = 0; q < hp.n; ++q) {
                  const uint32_t x = hp.d[q].id;
                  const double ch = pl_chord_mm(g, x, tv[j]);
                  const double xd = (double)hp.d[q].k.d + g_rho_d * ch, xt = (double)hp.d[q].k.t + g_rho_t * ch;
                  if (xd < ad) ad = xd;
                  if (xt < at) at = xt;
                }
                if (ad + (double)tpart[j] > (double)pd + 1e-3 || (X.time_on && at + (double)tpt[j] > (double)pt + 1e-3))
                  r = 1;
              }
              if (!r) unres = 1;
            }
            if (!unres) {
              exhausted = 0;
              break;
            }
            heap_item it = hpop(&hp);
            rkey itk = it.k;
            if (mode == 2) itk.k = itk.d; /* (node mode: k = d; the heap key carries k + h) */
            if (done[it.id] || !rk_eq(itk, lab[it.id])) continue;
            done[it.id] = 1;
            ++settled;
            const rkey L = lab[it.id];
            for (uint32_t e = g->node_row[it.id]; e < g->node_row[it.id + 1]; ++e) {
              if (!(g->edge_attr[e] & md.mode_bit)) continue;
              const rkey kk = step_key(&X, L, e, -1);
              if (!feasible(&X, kk)) continue;
              const uint32_t v = g->edge_dst[e];
              if (stamp[v] != gen) {
                stamp[v] = gen;
                done[v] = 0;
                lab[v] = (rkey){kInf, kInf, kInf};
              }
              if (rk_lt(kk, lab[v])) {
                lab[v] = kk;
                heap_item x = {kk, v};
                if (mode == 2) x.k.k = kk.k + (int64_t)NS_H(v);
                hpush(&hp, x);
              }
            }
          }
          free(hp.d);
          if (mode == 0) {
            S->settled_base += settled;
            S->exhausted_base += exhausted;
          } else if (mode == 3) {
            S->settled_tt += settled;
            S->exhausted_tt += exhausted;
          } else if (mode == 2) {
            S->settled_order += settled;
            S->exhausted_order += exhausted;
          } else {
            S->settled_astar += settled;
            S->exhausted_astar += exhausted;
          }
        }
      }
    }
  }
  free(stamp);
  free(lab);
  free(done);
  free(md.time_ds);
  return 0;
}

/* Edge-state exact rounds in A* order (analysis): f(b) = k(b) + c*rho_d*hq(b), hq(b) =
 * max(0, |head(b) - A| - R) (A: the target probe, R: its farthest target node); state b
 * is final once f(b) < fmin + (1 - c) * gap(b) + tmin (every later offer to b comes from a
 * pending u with f(u) >= fmin through b itself); targets final once tlab < fmin + tpart +
 * tmin; unreachable once every pending d + rho_d * hq (t + rho_t * hq) breaks the bound.
 * A round that settles nothing falls back to the key-order criterion (progress). */
typedef struct {
  int64_t searches, settled, rounds, stalls, settled_base, rounds_base;
} ea_stats;

static int64_t ea_search(const rctx* X, es_ws* W, uint32_t ei, double pi, int ntg, const uint32_t* tv,
                         const int64_t* tpart, const int64_t* tpt, const uint32_t* tej, int64_t tmin, double Ax,
                         double Ay, double R, double c, int64_t* settled, int64_t* rounds, int64_t* stalls,
                         double* hq) {
  const orc_graph* g = X->g;
  const mode_data* md = X->md;
  *settled = 0;
  *rounds = 0;
  const int64_t d0 = part_mm(1.0 - pi, g->len_mm[ei]);
  const int64_t t0 = X->time_on ? part_mm(1.0 - pi, md->time_ds[ei]) : 0;
  if (d0 > X->bmm || (X->time_on && t0 > X->bt)) return 0;
  const int64_t pd = X->bmm - d0, pt = X->time_on ? X->bt - t0 : kInf;
#define EA_HQ(e)                                                                                           \
  do {                                                                                                     \
    const uint32_t w_ = g->edge_dst[e];                                                                    \
    const double dx_ = (double)g->node_ll[2 * w_ + 1] * g_kx - Ax, dy_ = (double)g->node_ll[2 * w_] * g_ky - Ay; \
    hq[e] = fmax(0.0, sqrt(dx_ * dx_ + dy_ * dy_) - R);                                                     \
  } while (0)
  W->gen++;
  uint32_t np = 0;
  W->stamp[ei] = W->gen;
  W->lab[ei] = (rkey){0, 0, 0};
  W->flag[ei] = 1;
  EA_HQ(ei);
  W->pend[np++] = ei;
  rkey tl[ORC_KMAX];
  for (int j = 0; j < ntg; ++j) tl[j] = (rkey){kInf, kInf, kInf};
  const double ch = c * g_rho_d;
  for (;;) {
    if (np == 0) break;
    double fmin = 1e300, dlb = 1e300, tlb = 1e300;
    int64_t kmin = kInf;
    for (uint32_t q = 0; q < np; ++q) {
      const uint32_t b = W->pend[q];
      const double h = hq[b];
      const double f = (double)W->lab[b].k + ch * h;
      if (f < fmin) fmin = f;
      if ((double)W->lab[b].d + g_rho_d * h < dlb) dlb = (double)W->lab[b].d + g_rho_d * h;
      if ((double)W->lab[b].t + g_rho_t * h < tlb) tlb = (double)W->lab[b].t + g_rho_t * h;
      if (W->lab[b].k < kmin) kmin = W->lab[b].k;
    }
    int unres = 0;
    for (int j = 0; j < ntg; ++j) {
      if (tv[j] == 0xFFFFFFFFu) continue;
      const int res = (tl[j].k < kInf && (double)tl[j].k < fmin + (double)tpart[j] + (double)tmin) ||
                      dlb + (double)tpart[j] > (double)pd || (X->time_on && tlb + (double)tpt[j] > (double)pt);
      if (!res) unres = 1;
    }
    if (!unres) break;
    ++*rounds;
    uint32_t nf = 0, kept = 0;
    for (int pass = 0; pass < 2 && nf == 0; ++pass) {
      kept = 0;
      for (uint32_t q = 0; q < np; ++q) {
        const uint32_t b = W->pend[q];
        const int64_t len = b == ei ? 0 : (int64_t)g->len_mm[b];
        const int64_t mq = len >> 8 < 255 ? len >> 8 : 255;
        const int64_t gap = (mq ? mq << 8 : 1);
        const int take = pass == 0 ? ((double)W->lab[b].k + ch * hq[b] < fmin + (1.0 - c) * (double)gap + (b == ei ? 0 : tmin) - 1.0)
                                   : (W->lab[b].k < kmin + gap + (b == ei ? 0 : tmin));
        if (take) W->nxt[nf++] = b;
        else W->pend[kept++] = b;
      }
      if (nf == 0) ++*stalls;
    }
    np = kept;
    for (uint32_t f = 0; f < nf; ++f) {
      const uint32_t b = W->nxt[f];
      W->flag[b] = 2;
      ++*settled;
      const rkey L = W->lab[b];
      const uint32_t v = g->edge_dst[b];
      for (int j = 0; j < ntg; ++j)
        if (tv[j] == v) {
          const int64_t cc = md->turn[turn_degree(g, b, tej[j])];
          rkey o = {L.k + tpart[j] + cc, L.d + tpart[j], X->time_on ? L.t + tpt[j] : 0};
          if (o.d <= pd && o.t <= pt && o.k - o.d <= ORC_TCCAP && rk_lt(o, tl[j])) tl[j] = o;
        }
      for (uint32_t e = g->node_row[v]; e < g->node_row[v + 1]; ++e) {
        if (!(g->edge_attr[e] & md->mode_bit)) continue;
        const int64_t cc = md->turn[turn_degree(g, b, e)];
        rkey o = {L.k + g->len_mm[e] + cc, L.d + g->len_mm[e], X->time_on ? L.t + md->time_ds[e] : 0};
        if (!(o.d <= pd && o.t <= pt && o.k - o.d <= ORC_TCCAP)) continue;
        if (W->stamp[e] != W->gen) {
          W->stamp[e] = W->gen;
          W->lab[e] = (rkey){kInf, kInf, kInf};
          W->flag[e] = 0;
          EA_HQ(e);
        }
        if (rk_lt(o, W->lab[e])) {
          if (W->flag[e] == 2) { fprintf(stderr, "ea: settled label improved (not exact)\n"); }
          W->lab[e] = o;
          if (W->flag[e] == 0) {
            W->flag[e] = 1;
            W->pend[np++] = e;
          }
        }
      }
    }
  }
  return 0;
}

int ea_run(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off, const double* lat,
           const double* lon, const int64_t* tms, double c, ea_stats* S) {
  memset(S, 0, sizeof(*S));
  const uint32_t E = g->h.n_edges;
  es_ws W;
  memset(&W, 0, sizeof(W));
  W.stamp = calloc(E + 1, 4);
  W.lab = malloc(sizeof(rkey) * (E + 1));
  W.flag = calloc(E + 1, 1);
  W.ustamp = calloc(E + 1, 4);
  W.umask = calloc(E + 1, 8);
  W.pend = malloc(4 * (size_t)(E + 1));
  W.nxt = malloc(4 * (size_t)(E + 1));
  double* hq = malloc(sizeof(double) * (E + 1));
  mode_data md;
  mode_data_init(g, &p[0], 0, &md);
  {
    double lat0 = 0;
    for (uint32_t v = 0; v < g->h.n_nodes; ++v) lat0 += g->node_ll[2 * v] * 1e-6;
    lat0 /= g->h.n_nodes;
    g_ky = kM * 1e-6 * 1000.0;
    g_kx = kM * 1e-6 * 1000.0 * cos_deg(lat0) * 0.98;
    g_rho_d = 1e300;
    g_rho_t = 1e300;
    for (uint32_t e = 0; e < E; ++e) {
      if (!(g->edge_attr[e] & md.mode_bit)) continue;
      const double chd = pl_chord_mm(g, g->edge_src[e], g->edge_dst[e]);
      if (chd <= 0) continue;
      if ((double)g->len_mm[e] / chd < g_rho_d) g_rho_d = (double)g->len_mm[e] / chd;
      if ((double)md.time_ds[e] / chd < g_rho_t) g_rho_t = (double)md.time_ds[e] / chd;
    }
  }
  int64_t tmin = md.turn[0];
  for (int i = 0; i <= 180; ++i)
    if (md.turn[i] < tmin) tmin = md.turn[i];
  const int kmax = p[0].max_candidates < ORC_KMAX ? p[0].max_candidates : ORC_KMAX;
  static cand_t cands[4096][ORC_KMAX];
  static int kc[4096], act[4096];
  static int64_t sp[4096];
  for (int32_t t = 0; t < n_traces; ++t) {
    const int64_t b = trace_off[t], n = trace_off[t + 1] - b;
    int ns = 0;
    int64_t last = 0;
    for (int64_t i = 0; i < n && ns < 4096; ++i) {
      int st = i == 0 || i == n - 1 ||
               gc_dist(lat[b + last], lon[b + last], lat[b + i], lon[b + i]) >= p[0].interpolation_distance;
      if (st) {
        last = i;
        sp[ns++] = b + i;
      }
    }
    int na = 0;
    for (int s = 0; s < ns; ++s) {
      double a = p[0].gps_accuracy;
      double radius = p[0].search_radius > a ? p[0].search_radius : a;
      if (radius > p[0].max_search_radius) radius = p[0].max_search_radius;
      kc[s] = find_candidates(g, lat[sp[s]], lon[sp[s]], radius, md.mode_bit, kmax, cands[s]);
      if (kc[s] > 0) act[na++] = s;
    }
    for (int k = 1; k < na; ++k) {
      const int sa = act[k - 1], sb = act[k];
      const double gcd = gc_dist(lat[sp[sa]], lon[sp[sa]], lat[sp[sb]], lon[sp[sb]]);
      if (gcd > p[0].breakage_distance) continue;
      rctx X;
      step_ctx(&X, g, &md, &p[0], gcd, tms[sp[sb]] - tms[sp[sa]]);
      uint32_t tv[ORC_KMAX], tej[ORC_KMAX];
      int64_t tpart[ORC_KMAX], tpt[ORC_KMAX];
      const int Kb = kc[sb];
      const double Ax = lon[sp[sb]] * 1e6 * g_kx, Ay = lat[sp[sb]] * 1e6 * g_ky;
      double R = 0;
      for (int j = 0; j < Kb; ++j) {
        const uint32_t v = g->edge_src[cands[sb][j].e];
        const double dx = (double)g->node_ll[2 * v + 1] * g_kx - Ax, dy = (double)g->node_ll[2 * v] * g_ky - Ay;
        if (sqrt(dx * dx + dy * dy) > R) R = sqrt(dx * dx + dy * dy);
      }
      R += 1.0;
      for (int i = 0; i < kc[sa]; ++i) {
        const cand_t* ci = &cands[sa][i];
        int need = 0;
        for (int j = 0; j < Kb; ++j) {
          const cand_t* cj = &cands[sb][j];
          const int nd = !(cj->e == ci->e && cj->p >= ci->p);
          tv[j] = nd ? g->edge_src[cj->e] : 0xFFFFFFFFu;
          tej[j] = cj->e;
          tpart[j] = part_mm(cj->p, g->len_mm[cj->e]);
          tpt[j] = X.time_on ? part_mm(cj->p, md.time_ds[cj->e]) : 0;
          need |= nd;
        }
        if (!need) continue;
        int64_t st, rd, stl = 0, pm = 0, rl = 0;
        (void)es_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, &st, &rd, &rl, &pm, 0, NULL, NULL);
        S->settled_base += st;
        S->rounds_base += rd;
        (void)ea_search(&X, &W, ci->e, ci->p, Kb, tv, tpart, tpt, tej, tmin, Ax, Ay, R, c, &st, &rd, &stl, hq);
        S->searches++;
        S->settled += st;
        S->rounds += rd;
        S->stalls += stl;
      }
    }
  }
  free(W.stamp);
  free(W.lab);
  free(W.flag);
  free(W.ustamp);
  free(W.umask);
  free(W.pend);
  free(W.nxt);
  free(hq);
  free(md.time_ds);
  return 0;
}

/* Node-mode exact rounds (the GPU's k_route rounds, analysis): key order (k < kmin +
 * max(1, minin)) vs A* order (f = k + c*rho_d*hq, f < fmin + (1 - c) * minin - 1 mm, with
 * the key-order criterion as the fallback of a round that settles nothing). */
typedef struct {
  int64_t searches, settled_base, rounds_base, settled_a, rounds_a, stalls_a;
} nr_stats;

static int g_nr_term = 3; /* A* rounds' unreachability: 1 the length bound (d + rho hq), 2 the time bound */
void nr_set_term(int t) { g_nr_term = t; }
int nr_run(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off, const double* lat,
           const double* lon, const int64_t* tms, const float* acc, double c, nr_stats* S) {
  memset(S, 0, sizeof(*S));
  const uint32_t E = g->h.n_edges, N = g->h.n_nodes;
  mode_data md;
  mode_data_init(g, &p[0], 0, &md);
  {
    double lat0 = 0;
    for (uint32_t v = 0; v < N; ++v) lat0 += g->node_ll[2 * v] * 1e-6;
    lat0 /= N;
    g_ky = kM * 1e-6 * 1000.0;
    g_kx = kM * 1e-6 * 1000.0 * cos_deg(lat0) * 0.98;
    g_rho_d = 1e300;
    g_rho_t = 1e300;
    for (uint32_t e = 0; e < E; ++e) {
      if (!(g->edge_attr[e] & md.mode_bit)) continue;
      const double ch = pl_chord_mm(g, g->edge_src[e], g->edge_dst[e]);
      if (ch <= 0) continue;
      if ((double)g->len_mm[e] / ch < g_rho_d) g_rho_d = (double)g->len_mm[e] / ch;
      if ((double)md.time_ds[e] / ch < g_rho_t) g_rho_t = (double)md.time_ds[e] / ch;
    }
  }
  int64_t* minin = malloc(8 * (size_t)(N + 1));
  for (uint32_t v = 0; v < N; ++v) minin[v] = kInf;
  for (uint32_t e = 0; e < E; ++e)
    if ((g->edge_attr[e] & md.mode_bit) && (int64_t)g->len_mm[e] < minin[g->edge_dst[e]]) minin[g->edge_dst[e]] = g->len_mm[e];
  for (uint32_t v = 0; v < N; ++v)
    if (minin[v] < 1) minin[v] = 1;
  const int kmax = p[0].max_candidates < ORC_KMAX ? p[0].max_candidates : ORC_KMAX;
  static cand_t cands[4096][ORC_KMAX];
  static int kc[4096], act[4096];
  static int64_t sp[4096];
  uint32_t* stamp = calloc(N + 1, 4);
  rkey* lab = malloc(sizeof(rkey) * (N + 1));
  uint8_t* flag = calloc(N + 1, 1);
  double* hq = malloc(sizeof(double) * (N + 1));
  uint32_t* pend = malloc(4 * (size_t)(N + 1));
  uint32_t* nxt = malloc(4 * (size_t)(N + 1));
  uint32_t gen = 0;
  for (int32_t t = 0; t < n_traces; ++t) {
    const int64_t b = trace_off[t], n = trace_off[t + 1] - b;
    int ns = 0;
    int64_t last = 0;
    for (int64_t i = 0; i < n && ns < 4096; ++i) {
      int st = i == 0 || i == n - 1 ||
               gc_dist(lat[b + last], lon[b + last], lat[b + i], lon[b + i]) >= p[0].interpolation_distance;
      if (st) {
        last = i;
        sp[ns++] = b + i;
      }
    }
    int na = 0;
    for (int s = 0; s < ns; ++s) {
      double a = acc ? (double)acc[sp[s]] : p[0].gps_accuracy;
      double radius = p[0].search_radius > a ? p[0].search_radius : a;
      if (radius > p[0].max_search_radius) radius = p[0].max_search_radius;
      kc[s] = find_candidates(g, lat[sp[s]], lon[sp[s]], radius, md.mode_bit, kmax, cands[s]);
      if (kc[s] > 0) act[na++] = s;
    }
    for (int k = 1; k < na; ++k) {
      const int sa = act[k - 1], sb = act[k];
      const double gcd = gc_dist(lat[sp[sa]], lon[sp[sa]], lat[sp[sb]], lon[sp[sb]]);
      if (gcd > p[0].breakage_distance) continue;
      rctx X;
      step_ctx(&X, g, &md, &p[0], gcd, tms[sp[sb]] - tms[sp[sa]]);
      const int Kb = kc[sb];
      const double Ax = lon[sp[sb]] * 1e6 * g_kx, Ay = lat[sp[sb]] * 1e6 * g_ky;
      double R = 0;
      for (int j = 0; j < Kb; ++j) {
        const uint32_t v = g->edge_src[cands[sb][j].e];
        const double dx = (double)g->node_ll[2 * v + 1] * g_kx - Ax, dy = (double)g->node_ll[2 * v] * g_ky - Ay;
        if (sqrt(dx * dx + dy * dy) > R) R = sqrt(dx * dx + dy * dy);
      }
      R += 1.0;
      for (int i = 0; i < kc[sa]; ++i) {
        const cand_t* ci = &cands[sa][i];
        uint32_t tv[ORC_KMAX];
        int64_t tpart[ORC_KMAX], tpt[ORC_KMAX];
        int need = 0;
        for (int j = 0; j < Kb; ++j) {
          const cand_t* cj = &cands[sb][j];
          const int nd = !(cj->e == ci->e && cj->p >= ci->p);
          tv[j] = nd ? g->edge_src[cj->e] : 0xFFFFFFFFu;
          tpart[j] = part_mm(cj->p, g->len_mm[cj->e]);
          tpt[j] = X.time_on ? part_mm(cj->p, md.time_ds[cj->e]) : 0;
          need |= nd;
        }
        if (!need) continue;
        const rkey L0 = start_key(&X, ci->e, ci->p);
        if (!feasible(&X, L0)) continue;
        const int64_t pd = X.bmm, pt = X.time_on ? X.bt : kInf;
        S->searches++;
        for (int mode = 0; mode < 2; ++mode) {
          const double ch = mode ? c * g_rho_d : 0.0;
          ++gen;
          uint32_t np = 0;
          const uint32_t root = g->edge_dst[ci->e];
          stamp[root] = gen;
          lab[root] = L0;
          flag[root] = 1;
          {
            const double dx = (double)g->node_ll[2 * root + 1] * g_kx - Ax, dy = (double)g->node_ll[2 * root] * g_ky - Ay;
            hq[root] = fmax(0.0, sqrt(dx * dx + dy * dy) - R);
          }
          pend[np++] = root;
          int64_t settled = 0, rounds = 0, stalls = 0;
          for (;;) {
            if (np == 0) break;
            double fmin = 1e300, dlb = 1e300, tlb = 1e300;
            int64_t kmin = kInf, dmn = kInf, tmn = kInf;
            for (uint32_t q = 0; q < np; ++q) {
              const uint32_t v = pend[q];
              const double f = (double)lab[v].k + ch * hq[v];
              if (f < fmin) fmin = f;
              if ((double)lab[v].d + g_rho_d * hq[v] < dlb) dlb = (double)lab[v].d + g_rho_d * hq[v];
              if ((double)lab[v].t + g_rho_t * hq[v] < tlb) tlb = (double)lab[v].t + g_rho_t * hq[v];
              if (lab[v].k < kmin) kmin = lab[v].k;
              if (lab[v].d < dmn) dmn = lab[v].d;
              if (lab[v].t < tmn) tmn = lab[v].t;
            }
            int unres = 0;
            for (int j = 0; j < Kb && !unres; ++j) {
              const uint32_t v = tv[j];
              if (v == 0xFFFFFFFFu) continue;
              if (stamp[v] == gen && flag[v] == 2) continue;
              if (mode == 0) {
                const int64_t lt = stamp[v] == gen ? lab[v].d : kInf;
                const int64_t lo = lt < kmin + minin[v] ? lt : kmin + minin[v];
                if (stamp[v] == gen && lab[v].k < kmin + minin[v]) continue;
                if (lo + tpart[j] > pd) continue;
                if (X.time_on && tmn + tpt[j] > pt) continue;
              } else {
                if (stamp[v] == gen && (double)lab[v].k < fmin + (1.0 - c) * (double)minin[v] - 1.0) continue;
                {
                  const double lt = stamp[v] == gen ? (double)lab[v].d : 1e300;
                  const double nx = fmin + (1.0 - c) * (double)minin[v] - 1.0;
                  if ((lt < nx ? lt : nx) + (double)tpart[j] > (double)pd) continue;
                }
                if ((g_nr_term & 1) && dlb + (double)tpart[j] > (double)pd) continue;
                if ((g_nr_term & 2) && X.time_on && tlb + (double)tpt[j] > (double)pt) continue;
              }
              unres = 1;
            }
            if (!unres) break;
            ++rounds;
            uint32_t nf = 0, kept = 0;
            for (int pass = mode ? 0 : 1; pass < 2 && nf == 0; ++pass) {
              kept = 0;
              for (uint32_t q = 0; q < np; ++q) {
                const uint32_t v = pend[q];
                const int take = pass == 0 ? ((double)lab[v].k + ch * hq[v] < fmin + (1.0 - c) * (double)minin[v] - 1.0)
                                           : (lab[v].k < kmin + minin[v]);
                if (take) nxt[nf++] = v;
                else pend[kept++] = v;
              }
              if (nf == 0 && pass == 0) ++stalls;
            }
            np = kept;
            for (uint32_t f = 0; f < nf; ++f) {
              const uint32_t u = nxt[f];
              flag[u] = 2;
              ++settled;
              const rkey L = lab[u];
              for (uint32_t e = g->node_row[u]; e < g->node_row[u + 1]; ++e) {
                if (!(g->edge_attr[e] & md.mode_bit)) continue;
                const rkey kk = step_key(&X, L, e, -1);
                if (!feasible(&X, kk)) continue;
                const uint32_t v = g->edge_dst[e];
                if (stamp[v] != gen) {
                  stamp[v] = gen;
                  flag[v] = 0;
                  lab[v] = (rkey){kInf, kInf, kInf};
                  const double dx = (double)g->node_ll[2 * v + 1] * g_kx - Ax, dy = (double)g->node_ll[2 * v] * g_ky - Ay;
                  hq[v] = fmax(0.0, sqrt(dx * dx + dy * dy) - R);
                }
                if (rk_lt(kk, lab[v])) {
                  if (flag[v] == 2) fprintf(stderr, "nr: settled label improved (mode %d)\n", mode);
                  lab[v] = kk;
                  if (flag[v] == 0) {
                    flag[v] = 1;
                    pend[np++] = v;
                  }
                }
              }
            }
          }
          if (mode == 0) {
            S->settled_base += settled;
            S->rounds_base += rounds;
          } else {
            S->settled_a += settled;
            S->rounds_a += rounds;
            S->stalls_a += stalls;
          }
        }
      }
    }
  }
  free(stamp);
  free(lab);
  free(flag);
  free(hq);
  free(pend);
  free(nxt);
  free(minin);
  free(md.time_ds);
  return 0;
}
