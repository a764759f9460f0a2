// otrgen.cpp — seeded synthetic road graphs and GPS traces (libotrgen.so).
//
// Workload definition for the benches and tests.  The reference's
// generator (py/generate_test_trace.py) needs a live Valhalla service for routes;
// this restates it offline:
//   * graph: perturbed street grid with a level 0/1/2 hierarchy, one-ways, removed
//     links, footways, turn channels (internal) and service roads (no OSMLR), plus
//     OSMLR segments = chains of 1-5 edges, ids packed level|tile|index exactly as
//     simple_reporter.py:36-49 / get_tiles.py:30-72 lay them out.
//   * traces: a random drive at edge speed, one position per second
//     (get_coords_per_second, generate_test_trace.py:120-149), every sampleRate-th
//     second plus the last kept (:71-74), quadrant-rejected Gaussian noise averaged
//     over `noiseLookback = ceil(30 / (sampleRate+2))` draws with Python-2 integer
//     division (0 ⇒ mean of ALL draws, since lst[-0:] is the whole list) (:59,79-91),
//     lat/lon rounded to 6 dp (:94-95), integer times (:93).
// Not product code: the product never links this library.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/otr_graph_format.h"

namespace {

constexpr double kMetersPerDeg = 20037581.187 / 180.0;  // Batch.java:36

struct Rng {  // splitmix64 → xoshiro256**
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (int i = 0; i < 4; ++i) {
      seed += 0x9E3779B97F4A7C15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) % n); }
  double normal() {  // Box-Muller
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

struct Link {  // undirected street link between grid nodes a→b (a < b in walk order)
  uint32_t a, b;
  int level;
  uint32_t line;      // road line id (row/col line)
  uint32_t pos;       // position along the line
  int dir;            // 0 both, +1 a→b only, -1 b→a only
  bool internal, unassociated;
  uint32_t access;
  uint64_t mid_off;  // intermediate shape points (lat_e6, lon_e6): mids[mid_off, mid_off + nmid)
  uint32_t nmid;
};

struct DEdge {
  uint32_t src, dst, link;
  bool fwd;
};

double seg_len_m(int32_t la, int32_t lo, int32_t lb, int32_t lob) {
  double lat1 = la * 1e-6, lon1 = lo * 1e-6, lat2 = lb * 1e-6, lon2 = lob * 1e-6;
  double x = (lon1 - lon2) * kMetersPerDeg * std::cos(0.5 * (lat1 + lat2) * M_PI / 180.0);
  double y = (lat1 - lat2) * kMetersPerDeg;
  return std::sqrt(x * x + y * y);
}

// get_tiles.py:51-72, world bbox (-180,-90,180,90): tile id = row * ncols + col
uint32_t tile_index(int level, double lat, double lon) {
  double size = level == 0 ? 4.0 : (level == 1 ? 1.0 : 0.25);
  int ncols = (int)std::ceil(360.0 / size);
  int row = (int)((lat + 90.0) / size);
  int col = (int)((lon + 180.0) / size);
  return (uint32_t)(row * ncols + col);
}

template <class T>
void write_arr(FILE* f, const std::vector<T>& v, uint64_t* off) {
  long pos = ftell(f);
  long pad = (64 - pos % 64) % 64;
  static const char zeros[64] = {0};
  fwrite(zeros, 1, pad, f);
  *off = (uint64_t)(pos + pad);
  if (!v.empty()) fwrite(v.data(), sizeof(T), v.size(), f);
}

}  // namespace

extern "C" {

// Generates a street-grid graph and writes it to `path`.  Returns 0 on success.
int otrgen_graph(const char* path, int rows, int cols, double spacing_m, double center_lat,
                 double center_lon, double p_remove, uint64_t seed, double cell_deg) {
  // country-scale graphs (C5, ~50M nodes) take minutes: progress on stderr
  const bool big = (uint64_t)rows * (uint64_t)cols > 4000000ull;
  auto say = [&](const char* what) {
    if (big) {
      fprintf(stderr, "otrgen: %s\n", what);
      fflush(stderr);
    }
  };
  Rng rng(seed);
  const double mlon = kMetersPerDeg * std::cos(center_lat * M_PI / 180.0);
  const uint32_t n_nodes = (uint32_t)rows * (uint32_t)cols;
  std::vector<int32_t> node_ll(2 * (size_t)n_nodes);
  const double jit = 0.12 * spacing_m;
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
      double lat = center_lat + ((r - rows / 2) * spacing_m + (rng.uni() * 2 - 1) * jit) / kMetersPerDeg;
      double lon = center_lon + ((c - cols / 2) * spacing_m + (rng.uni() * 2 - 1) * jit) / mlon;
      size_t n = (size_t)r * cols + c;
      node_ll[2 * n] = (int32_t)std::llround(lat * 1e6);
      node_ll[2 * n + 1] = (int32_t)std::llround(lon * 1e6);
    }
  auto line_level = [](int k) { return k % 16 == 0 ? 0 : (k % 4 == 0 ? 1 : 2); };
  std::vector<Link> links;
  links.reserve(2 * (size_t)n_nodes);
  std::vector<std::pair<int32_t, int32_t>> mids;
  mids.reserve(2 * (size_t)n_nodes);
  // horizontal lines (rows), then vertical lines (cols)
  for (int pass = 0; pass < 2; ++pass) {
    int nl = pass == 0 ? rows : cols, len = pass == 0 ? cols : rows;
    for (int k = 0; k < nl; ++k) {
      int level = line_level(k);
      uint32_t line = (uint32_t)(pass * rows + k);
      int oneway = 0;
      if (level == 2 && (k % 7) == 3) oneway = (k / 7) % 2 ? 1 : -1;
      for (int p = 0; p + 1 < len; ++p) {
        Link L;
        L.a = pass == 0 ? (uint32_t)(k * cols + p) : (uint32_t)(p * cols + k);
        L.b = pass == 0 ? (uint32_t)(k * cols + p + 1) : (uint32_t)((p + 1) * cols + k);
        L.level = level;
        L.line = line;
        L.pos = (uint32_t)p;
        L.dir = oneway;
        double u = rng.uni();
        if (level == 2 && u < p_remove) continue;
        L.internal = level == 2 && rng.uni() < 0.03;
        L.unassociated = !L.internal && level == 2 && rng.uni() < 0.08;
        L.access = level == 0 ? OTR_ACCESS_AUTO
                              : (OTR_ACCESS_AUTO | OTR_ACCESS_BICYCLE | OTR_ACCESS_PEDESTRIAN);
        if (level == 2 && !L.internal && rng.uni() < 0.04) L.access = OTR_ACCESS_PEDESTRIAN | OTR_ACCESS_BICYCLE;
        int nmid = (int)rng.below(3);
        int32_t la = node_ll[2 * L.a], loa = node_ll[2 * L.a + 1];
        int32_t lb = node_ll[2 * L.b], lob = node_ll[2 * L.b + 1];
        L.mid_off = mids.size();
        L.nmid = (uint32_t)nmid;
        for (int m = 1; m <= nmid; ++m) {
          double f = (double)m / (nmid + 1);
          double off = (rng.uni() * 2 - 1) * 4.0;  // metres, perpendicular wiggle
          double lat = (la + f * (lb - la)) * 1e-6, lon = (loa + f * (lob - loa)) * 1e-6;
          if (pass == 0) lat += off / kMetersPerDeg; else lon += off / mlon;
          mids.push_back({(int32_t)std::llround(lat * 1e6), (int32_t)std::llround(lon * 1e6)});
        }
        links.push_back(L);
      }
    }
  }
  // no sinks: a one-way link into a node with no way out for cars becomes two-way
  for (int pass = 0; pass < 4; ++pass) {
    std::vector<uint32_t> outdeg(n_nodes, 0);
    for (const Link& L : links) {
      if (!(L.access & OTR_ACCESS_AUTO)) continue;
      if (L.dir >= 0) outdeg[L.a]++;
      if (L.dir <= 0) outdeg[L.b]++;
    }
    bool changed = false;
    for (Link& L : links) {
      if (L.dir == 0 || !(L.access & OTR_ACCESS_AUTO)) continue;
      uint32_t head = L.dir > 0 ? L.b : L.a;
      if (outdeg[head] == 0) { L.dir = 0; changed = true; }
    }
    if (!changed) break;
  }
  say("links done");
  // directed edges
  std::vector<DEdge> de;
  de.reserve(2 * links.size());
  for (uint32_t i = 0; i < links.size(); ++i) {
    const Link& L = links[i];
    if (L.dir >= 0) de.push_back({L.a, L.b, i, true});
    if (L.dir <= 0) de.push_back({L.b, L.a, i, false});
  }
  std::sort(de.begin(), de.end(), [](const DEdge& x, const DEdge& y) {
    return x.src != y.src ? x.src < y.src : x.dst < y.dst;
  });
  say("directed edges sorted");
  if (de.size() >= 0xFFFFFFFFull) return -3;
  const uint32_t n_edges = (uint32_t)de.size();
  std::vector<uint32_t> node_row(n_nodes + 1, 0), edge_src(n_edges), edge_dst(n_edges), edge_attr(n_edges),
      edge_shape(n_edges + 1), edge_seg(n_edges, OTR_NO_SEGMENT), edge_way(n_edges);
  std::vector<float> edge_len(n_edges);
  std::vector<int32_t> shape_ll;
  shape_ll.reserve(2 * (size_t)n_edges * 3);
  for (uint32_t e = 0; e < n_edges; ++e) {
    const DEdge& d = de[e];
    const Link& L = links[d.link];
    node_row[d.src + 1]++;
    edge_src[e] = d.src;
    edge_dst[e] = d.dst;
    uint32_t speed = L.level == 0 ? 90 : (L.level == 1 ? 50 : 30);
    if (L.internal) speed = 20;
    uint32_t attr = (L.access & OTR_ATTR_ACCESS_MASK) | (speed << OTR_ATTR_SPEED_SHIFT) |
                    ((uint32_t)L.level << OTR_ATTR_LEVEL_SHIFT);
    if (L.internal) attr |= OTR_ATTR_INTERNAL;
    edge_attr[e] = attr;
    edge_way[e] = 100000u + L.line * 64u + L.pos / 20u;
    edge_shape[e] = (uint32_t)(shape_ll.size() / 2);
    std::pair<int32_t, int32_t> pts[4];
    size_t np = 0;
    pts[np++] = {node_ll[2 * (size_t)d.src], node_ll[2 * (size_t)d.src + 1]};
    if (d.fwd) for (uint32_t m = 0; m < L.nmid; ++m) pts[np++] = mids[L.mid_off + m];
    else for (uint32_t m = L.nmid; m-- > 0;) pts[np++] = mids[L.mid_off + m];
    pts[np++] = {node_ll[2 * (size_t)d.dst], node_ll[2 * (size_t)d.dst + 1]};
    double len = 0;
    for (size_t k = 0; k < np; ++k) {
      shape_ll.push_back(pts[k].first);
      shape_ll.push_back(pts[k].second);
      if (k) len += seg_len_m(pts[k - 1].first, pts[k - 1].second, pts[k].first, pts[k].second);
    }
    edge_len[e] = (float)std::max(len, 0.5);
  }
  edge_shape[n_edges] = (uint32_t)(shape_ll.size() / 2);
  for (uint32_t n = 0; n < n_nodes; ++n) node_row[n + 1] += node_row[n];
  auto find_edge = [&](uint32_t s, uint32_t t) -> int64_t {
    for (uint32_t e = node_row[s]; e < node_row[s + 1]; ++e)
      if (edge_dst[e] == t) return e;
    return -1;
  };
  // OSMLR segments: walk each line in each direction, chain associated links 1-5 at a time.
  std::vector<uint64_t> seg_id;
  std::vector<uint32_t> seg_len;
  std::map<std::pair<int, uint32_t>, uint32_t> tile_counter;
  {
    // group links per line, ordered by pos
    std::vector<std::vector<uint32_t>> per_line((size_t)rows + cols);
    for (uint32_t i = 0; i < links.size(); ++i) per_line[links[i].line].push_back(i);
    for (auto& lv : per_line) {
      for (int fwd = 1; fwd >= 0; --fwd) {
        std::vector<int64_t> chain;  // directed edge ids along this direction, -1 = break
        if (fwd) {
          int64_t prev_pos = -2;
          for (uint32_t li : lv) {
            const Link& L = links[li];
            if ((int64_t)L.pos != prev_pos + 1) chain.push_back(-1);
            prev_pos = L.pos;
            int64_t e = (L.dir >= 0 && !L.internal && !L.unassociated) ? find_edge(L.a, L.b) : -1;
            chain.push_back(e);
          }
        } else {
          int64_t prev_pos = -2;
          for (auto it = lv.rbegin(); it != lv.rend(); ++it) {
            const Link& L = links[*it];
            if ((int64_t)L.pos != prev_pos - 1 && prev_pos != -2) chain.push_back(-1);
            prev_pos = L.pos;
            int64_t e = (L.dir <= 0 && !L.internal && !L.unassociated) ? find_edge(L.b, L.a) : -1;
            chain.push_back(e);
          }
        }
        size_t k = 0;
        while (k < chain.size()) {
          if (chain[k] < 0) { ++k; continue; }
          size_t want = 1 + rng.below(5), j = k;
          while (j < chain.size() && chain[j] >= 0 && j - k < want) ++j;
          uint32_t sidx = (uint32_t)seg_id.size();
          uint32_t e0 = (uint32_t)chain[k];
          int level = (int)OTR_ATTR_LEVEL(edge_attr[e0]);
          double lat0 = node_ll[2 * edge_src[e0]] * 1e-6, lon0 = node_ll[2 * edge_src[e0] + 1] * 1e-6;
          uint32_t tile = tile_index(level, lat0, lon0);
          uint32_t& cnt = tile_counter[{level, tile}];
          uint64_t id = ((uint64_t)cnt << 25) | ((uint64_t)tile << 3) | (uint64_t)level;
          ++cnt;
          double sl = 0;
          for (size_t q = k; q < j; ++q) {
            uint32_t e = (uint32_t)chain[q];
            edge_seg[e] = sidx;
            sl += edge_len[e];
            if (q == k) edge_attr[e] |= OTR_ATTR_SEG_BEGIN;
            if (q + 1 == j) edge_attr[e] |= OTR_ATTR_SEG_END;
          }
          seg_id.push_back(id);
          seg_len.push_back((uint32_t)std::llround(sl));
          k = j;
        }
      }
    }
  }
  // reverse CSR
  std::vector<uint32_t> rev_row(n_nodes + 1, 0), rev_edge(n_edges);
  for (uint32_t e = 0; e < n_edges; ++e) rev_row[edge_dst[e] + 1]++;
  for (uint32_t n = 0; n < n_nodes; ++n) rev_row[n + 1] += rev_row[n];
  {
    std::vector<uint32_t> fill(rev_row.begin(), rev_row.end() - 1);
    for (uint32_t e = 0; e < n_edges; ++e) rev_edge[fill[edge_dst[e]]++] = e;
  }
  say("segments done");
  // grid index
  int32_t mnla = INT32_MAX, mnlo = INT32_MAX, mxla = INT32_MIN, mxlo = INT32_MIN;
  for (size_t k = 0; k < shape_ll.size(); k += 2) {
    mnla = std::min(mnla, shape_ll[k]); mxla = std::max(mxla, shape_ll[k]);
    mnlo = std::min(mnlo, shape_ll[k + 1]); mxlo = std::max(mxlo, shape_ll[k + 1]);
  }
  double gmin_lat = std::floor(mnla * 1e-6 / cell_deg) * cell_deg - cell_deg;
  double gmin_lon = std::floor(mnlo * 1e-6 / cell_deg) * cell_deg - cell_deg;
  uint32_t grows = (uint32_t)std::ceil((mxla * 1e-6 - gmin_lat) / cell_deg) + 2;
  uint32_t gcols = (uint32_t)std::ceil((mxlo * 1e-6 - gmin_lon) / cell_deg) + 2;
  if ((uint64_t)grows * gcols >= 0xFFFFFFFFull) return -4;
  uint32_t n_cells = grows * gcols;
  // (cell, edge) entries by a counting sort over cells: every cell lists its edges in
  // ascending order, each once (what sorting the (cell, edge) pairs gives)
  auto edge_cells = [&](uint32_t e, std::vector<uint32_t>& cells) {
    cells.clear();
    for (uint32_t k = edge_shape[e]; k + 1 < edge_shape[e + 1]; ++k) {
      double la0 = shape_ll[2 * (size_t)k] * 1e-6, lo0 = shape_ll[2 * (size_t)k + 1] * 1e-6;
      double la1 = shape_ll[2 * (size_t)k + 2] * 1e-6, lo1 = shape_ll[2 * (size_t)k + 3] * 1e-6;
      double a = std::min(la0, la1) - OTR_GRID_PAD_DEG, b = std::max(la0, la1) + OTR_GRID_PAD_DEG;
      double c = std::min(lo0, lo1) - OTR_GRID_PAD_DEG, d = std::max(lo0, lo1) + OTR_GRID_PAD_DEG;
      int64_t r0 = (int64_t)std::floor((a - gmin_lat) / cell_deg), r1 = (int64_t)std::floor((b - gmin_lat) / cell_deg);
      int64_t c0 = (int64_t)std::floor((c - gmin_lon) / cell_deg), c1 = (int64_t)std::floor((d - gmin_lon) / cell_deg);
      for (int64_t r = std::max<int64_t>(r0, 0); r <= std::min<int64_t>(r1, grows - 1); ++r)
        for (int64_t cc = std::max<int64_t>(c0, 0); cc <= std::min<int64_t>(c1, gcols - 1); ++cc)
          cells.push_back((uint32_t)(r * gcols + cc));
    }
    std::sort(cells.begin(), cells.end());
    cells.erase(std::unique(cells.begin(), cells.end()), cells.end());
  };
  std::vector<uint32_t> cell_row(n_cells + 1, 0), cells;
  for (uint32_t e = 0; e < n_edges; ++e) {
    edge_cells(e, cells);
    for (uint32_t c : cells) cell_row[c + 1]++;
  }
  {
    uint64_t total = 0;
    for (uint32_t c = 0; c < n_cells; ++c) total += cell_row[c + 1];
    if (total >= 0xFFFFFFFFull) return -5;  // u32 cell offsets (include/otr_graph_format.h)
  }
  for (uint32_t c = 0; c < n_cells; ++c) cell_row[c + 1] += cell_row[c];
  std::vector<uint32_t> cell_edge(cell_row[n_cells]);
  {
    std::vector<uint32_t> fill(cell_row.begin(), cell_row.end() - 1);
    for (uint32_t e = 0; e < n_edges; ++e) {
      edge_cells(e, cells);
      for (uint32_t c : cells) cell_edge[fill[c]++] = e;
    }
  }
  say("grid done");

  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  otr_graph_header h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, OTR_GRAPH_MAGIC, 8);
  h.version = OTR_GRAPH_VERSION;
  h.n_nodes = n_nodes; h.n_edges = n_edges; h.n_shape = (uint32_t)(shape_ll.size() / 2);
  h.n_segments = (uint32_t)seg_id.size(); h.n_cells = n_cells; h.n_cell_entries = (uint32_t)cell_edge.size();
  h.grid_rows = grows; h.grid_cols = gcols;
  h.grid_min_lat = gmin_lat; h.grid_min_lon = gmin_lon; h.grid_cell_deg = cell_deg;
  fwrite(&h, sizeof(h), 1, f);
  write_arr(f, node_row, &h.array_offset[OTR_A_NODE_ROW]);
  write_arr(f, node_ll, &h.array_offset[OTR_A_NODE_LL]);
  write_arr(f, rev_row, &h.array_offset[OTR_A_REV_ROW]);
  write_arr(f, rev_edge, &h.array_offset[OTR_A_REV_EDGE]);
  write_arr(f, edge_src, &h.array_offset[OTR_A_EDGE_SRC]);
  write_arr(f, edge_dst, &h.array_offset[OTR_A_EDGE_DST]);
  write_arr(f, edge_len, &h.array_offset[OTR_A_EDGE_LEN]);
  write_arr(f, edge_attr, &h.array_offset[OTR_A_EDGE_ATTR]);
  write_arr(f, edge_shape, &h.array_offset[OTR_A_EDGE_SHAPE]);
  write_arr(f, edge_seg, &h.array_offset[OTR_A_EDGE_SEG]);
  write_arr(f, edge_way, &h.array_offset[OTR_A_EDGE_WAY]);
  write_arr(f, shape_ll, &h.array_offset[OTR_A_SHAPE_LL]);
  write_arr(f, seg_id, &h.array_offset[OTR_A_SEG_ID]);
  write_arr(f, seg_len, &h.array_offset[OTR_A_SEG_LEN]);
  write_arr(f, cell_row, &h.array_offset[OTR_A_CELL_ROW]);
  write_arr(f, cell_edge, &h.array_offset[OTR_A_CELL_EDGE]);
  h.array_offset[OTR_A_END] = (uint64_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  fwrite(&h, sizeof(h), 1, f);
  fclose(f);
  return 0;
}

// Synthesises `n_traces` drives of `n_points` kept probes each on the graph file
// `graph_path`.  Output arrays are caller-allocated with n_traces*n_points entries
// (times are epoch seconds).  mode_mix: fractions of auto/bicycle/pedestrian traces;
// out_mode[t] receives 0/1/2.  point_accuracy < 0 means "no accuracy field".
// ids != NULL: trace t is the drive of vehicle ids[t], drawn from its own generator
// seeded by (seed, ids[t]) — any subset of a fleet (a uuid shard, C3) is generated alone.
static int gen_traces(const char* graph_path, int n_traces, const int64_t* ids, int n_points, int sample_rate,
                      double noise_m, uint64_t seed, double frac_bicycle, double frac_pedestrian, double* out_lat,
                      double* out_lon, int64_t* out_time, uint8_t* out_mode, uint32_t* out_truth_edge,
                      int64_t t_begin, int64_t t_spread) {
  FILE* f = fopen(graph_path, "rb");
  if (!f) return -1;
  otr_graph_header h;
  if (fread(&h, sizeof(h), 1, f) != 1) { fclose(f); return -2; }
  auto rd = [&](int a, size_t bytes) {
    std::vector<char> v(bytes);
    fseek(f, (long)h.array_offset[a], SEEK_SET);
    if (bytes && fread(v.data(), 1, bytes, f) != bytes) v.clear();
    return v;
  };
  auto vnode_row = rd(OTR_A_NODE_ROW, 4ull * (h.n_nodes + 1));
  auto vedge_dst = rd(OTR_A_EDGE_DST, 4ull * h.n_edges);
  auto vedge_src = rd(OTR_A_EDGE_SRC, 4ull * h.n_edges);
  auto vedge_attr = rd(OTR_A_EDGE_ATTR, 4ull * h.n_edges);
  auto vedge_shape = rd(OTR_A_EDGE_SHAPE, 4ull * (h.n_edges + 1));
  auto vshape = rd(OTR_A_SHAPE_LL, 8ull * h.n_shape);
  fclose(f);
  const uint32_t* node_row = (const uint32_t*)vnode_row.data();
  const uint32_t* edge_dst = (const uint32_t*)vedge_dst.data();
  const uint32_t* edge_src = (const uint32_t*)vedge_src.data();
  const uint32_t* edge_attr = (const uint32_t*)vedge_attr.data();
  const uint32_t* edge_shape = (const uint32_t*)vedge_shape.data();
  const int32_t* shape = (const int32_t*)vshape.data();
  const int lookback = (int)std::ceil((double)(30 / (sample_rate + 2)));  // py2 int division
  Rng rng(seed);
  for (int t = 0; t < n_traces; ++t) {
    if (ids) rng = Rng(seed * 0x100000001B3ull ^ (uint64_t)ids[t]);
    double um = rng.uni();
    int mode = um < frac_pedestrian ? 2 : (um < frac_pedestrian + frac_bicycle ? 1 : 0);
    uint32_t mbit = 1u << mode;
    out_mode[t] = (uint8_t)mode;
    double speed_cap = mode == 0 ? 1e9 : (mode == 1 ? 18.0 : 5.0);
    uint32_t e;
    do { e = rng.below(h.n_edges); } while (!(edge_attr[e] & mbit));
    // shape polyline of the current edge in metres along
    std::vector<double> cum;
    auto load_edge = [&](uint32_t ed) {
      cum.assign(1, 0.0);
      for (uint32_t k = edge_shape[ed]; k + 1 < edge_shape[ed + 1]; ++k)
        cum.push_back(cum.back() + seg_len_m(shape[2 * k], shape[2 * k + 1], shape[2 * k + 2], shape[2 * k + 3]));
    };
    load_edge(e);
    double along = rng.uni() * cum.back();
    int64_t t0 = t_begin + (t_spread > 0 ? (int64_t)rng.below((uint32_t)t_spread) : 0);
    std::vector<double> adj_lon, adj_lat;
    int qlon = 0, qlat = 0;
    int kept = 0;
    int64_t sec = 0;
    while (kept < n_points) {
      if (sec % sample_rate == 0) {
        // position on the current edge
        size_t k = 1;
        while (k + 1 < cum.size() && cum[k] < along) ++k;
        uint32_t s0 = edge_shape[e] + (uint32_t)k - 1;
        double seg = cum[k] - cum[k - 1];
        double fr = seg > 0 ? std::min(1.0, std::max(0.0, (along - cum[k - 1]) / seg)) : 0.0;
        double lat = (shape[2 * s0] + fr * (shape[2 * s0 + 2] - shape[2 * s0])) * 1e-6;
        double lon = (shape[2 * s0 + 1] + fr * (shape[2 * s0 + 3] - shape[2 * s0 + 1])) * 1e-6;
        if (noise_m > 0) {
          double a, b;
          for (;;) {  // quadrant rejection (generate_test_trace.py:79-86)
            a = rng.normal() * noise_m;
            b = rng.normal() * noise_m;
            int sa = (a > 0) - (a < 0), sb = (b > 0) - (b < 0);
            if (kept == 0) { qlon = sa; qlat = sb; break; }
            if (sa == qlon && sb == qlat) break;
          }
          adj_lon.push_back(a);
          adj_lat.push_back(b);
          size_t n = adj_lon.size(), from = lookback == 0 ? 0 : (n > (size_t)lookback ? n - lookback : 0);
          double ml = 0, mb = 0;
          for (size_t q = from; q < n; ++q) { ml += adj_lon[q]; mb += adj_lat[q]; }
          ml /= (double)(n - from);
          mb /= (double)(n - from);
          lat += mb / kMetersPerDeg;
          lon += ml / (kMetersPerDeg * std::cos(lat * M_PI / 180.0));
        }
        size_t o = (size_t)t * n_points + kept;
        out_lat[o] = std::nearbyint(lat * 1e6) / 1e6;
        out_lon[o] = std::nearbyint(lon * 1e6) / 1e6;
        out_time[o] = t0 + sec;
        if (out_truth_edge) out_truth_edge[o] = e;
        ++kept;
      }
      // advance one second
      double v = std::min((double)OTR_ATTR_SPEED(edge_attr[e]) / 3.6, speed_cap);
      double rem = v;
      while (rem > 0) {
        if (along + rem <= cum.back()) { along += rem; rem = 0; break; }
        rem -= cum.back() - along;
        uint32_t node = edge_dst[e];
        uint32_t opts[16];
        int no = 0;
        for (uint32_t x = node_row[node]; x < node_row[node + 1] && no < 16; ++x)
          if ((edge_attr[x] & mbit) && edge_dst[x] != edge_src[e]) opts[no++] = x;
        if (no == 0)
          for (uint32_t x = node_row[node]; x < node_row[node + 1] && no < 16; ++x)
            if (edge_attr[x] & mbit) opts[no++] = x;
        if (no == 0) { rem = 0; break; }  // dead end: stop moving
        // drivers mostly keep straight: pick the best-aligned continuation 70% of the time
        uint32_t pick = opts[rng.below((uint32_t)no)];
        if (rng.uni() < 0.7) {
          const int32_t* ns = shape + 2 * (size_t)edge_shape[e];
          double hx = (double)(shape[2 * (size_t)(edge_shape[e + 1] - 1) + 1] - ns[1]);
          double hy = (double)(shape[2 * (size_t)(edge_shape[e + 1] - 1)] - ns[0]);
          double best = -1e300;
          for (int q = 0; q < no; ++q) {
            const int32_t* a = shape + 2 * (size_t)edge_shape[opts[q]];
            const int32_t* z = shape + 2 * (size_t)(edge_shape[opts[q] + 1] - 1);
            double vx = (double)(z[1] - a[1]), vy = (double)(z[0] - a[0]);
            double nv = std::sqrt(vx * vx + vy * vy) + 1e-9;
            double dot = (hx * vx + hy * vy) / nv;
            if (dot > best) { best = dot; pick = opts[q]; }
          }
        }
        e = pick;
        load_edge(e);
        along = 0;
      }
      ++sec;
    }
  }
  return 0;
}

int otrgen_traces(const char* graph_path, int n_traces, int n_points, int sample_rate, double noise_m,
                  uint64_t seed, double frac_bicycle, double frac_pedestrian, double* out_lat,
                  double* out_lon, int64_t* out_time, uint8_t* out_mode, uint32_t* out_truth_edge,
                  int64_t t_begin, int64_t t_spread) {
  return gen_traces(graph_path, n_traces, nullptr, n_points, sample_rate, noise_m, seed, frac_bicycle,
                    frac_pedestrian, out_lat, out_lon, out_time, out_mode, out_truth_edge, t_begin, t_spread);
}

int otrgen_traces_ids(const char* graph_path, int n_traces, const int64_t* ids, int n_points, int sample_rate,
                      double noise_m, uint64_t seed, double frac_bicycle, double frac_pedestrian, double* out_lat,
                      double* out_lon, int64_t* out_time, uint8_t* out_mode, uint32_t* out_truth_edge,
                      int64_t t_begin, int64_t t_spread) {
  return gen_traces(graph_path, n_traces, ids, n_points, sample_rate, noise_m, seed, frac_bicycle,
                    frac_pedestrian, out_lat, out_lon, out_time, out_mode, out_truth_edge, t_begin, t_spread);
}

}  // extern "C"
