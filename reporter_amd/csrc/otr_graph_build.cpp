// otr_graph_build.cpp — host-side graph building (§8f rank 1): the Valhalla tile
// hierarchy of the reference's py/get_tiles.py and the flattener that turns decoded
// road-graph arrays (nodes, directed edges with their shapes and OSMLR associations)
// into the .otrg file otr_configure() uploads (include/otr_graph_format.h).
//
// Tile hierarchy (get_tiles.py:30-102, itself after Valhalla baldr tilehierarchy.cc /
// graphtile.cc): levels 0/1/2 tile the world bbox (-180,-90,180,90) with 4 / 1 / 0.25
// degree tiles, tile id = row * ncolumns + col; GetFile spells level * 10^d + id with
// thousands separators turned into '/', d = the digit count of the level's largest id
// rounded up to a multiple of 3 (level 0 writes its leading digit as '0').  The script's
// main loop (:132-171) lists, per bbox (split at the antimeridian), every tile of every
// level in the order Python 2 iterates {2:.., 1:.., 0:..} — levels 0, 1, 2.
//
// Flattener: edges shorter than 5 cm are contracted (their end nodes merged into the
// smallest node id of the cluster): the route search's exact rounds settle a node once
// its label is below the smallest pending length + its shortest in-edge,
// so millimetre edges would only make the rounds narrow; edges whose ends merged vanish, the
// others keep their shapes with the end points moved onto the surviving nodes, and a
// vanished edge's segment-begin / segment-end flag moves to the neighbouring edge of
// the same OSMLR segment.  Lengths are the shapes' equirectangular lengths (metres per
// degree 20037581.187 / 180, Batch.java:36) — the same rule the synthetic generator
// uses, so a generated graph flattened from its own arrays comes back byte-identical.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/otr.h"
#include "../../include/otr_graph_format.h"

namespace {

constexpr double kMetersPerDeg = 20037581.187 / 180.0;  // Batch.java:36
constexpr double kMinEdgeM = 0.05;

// ---- tile hierarchy (get_tiles.py:30-102) -------------------------------------------
struct TileLevel {
  double size;
  int64_t ncolumns, nrows, max_tile_id;
};

TileLevel tile_level(int level) {
  const double size = level == 0 ? 4.0 : (level == 1 ? 1.0 : 0.25);  // :36-40
  TileLevel t;
  t.size = size;
  t.ncolumns = (int64_t)std::ceil((180.0 - -180.0) / size);  // :48
  t.nrows = (int64_t)std::ceil((90.0 - -90.0) / size);       // :49
  t.max_tile_id = t.ncolumns * t.nrows - 1;                  // :50
  return t;
}

// Tiles.Row (:51-60): -1 outside; the max edge maps to the last row; else truncation
int64_t tile_row(const TileLevel& t, double y) {
  if (y < -90.0 || y > 90.0) return -1;
  if (y == 90.0) return t.nrows - 1;
  return (int64_t)((y - -90.0) / t.size);
}

// Tiles.Col (:62-72)
int64_t tile_col(const TileLevel& t, double x) {
  if (x < -180.0 || x > 180.0) return -1;
  if (x == 180.0) return t.ncolumns - 1;
  const double col = (x - -180.0) / t.size;
  return col >= 0.0 ? (int64_t)col : (int64_t)(col - 1);
}

// Tiles.Digits (:74-79) over a non-negative id: decimal digits (0 has none)
int64_t digits(int64_t n) {
  int64_t d = n < 0 ? 1 : 0;
  while (n) {
    n /= 10;  // Python 2 long division of a non-negative number
    ++d;
  }
  return d;
}

// '{:,}'.format(v): thousands separators on the decimal digits, sign kept in front
std::string with_commas(int64_t v) {
  const bool neg = v < 0;
  const unsigned long long mag = neg ? (unsigned long long)(-(v + 1)) + 1ull : (unsigned long long)v;
  const std::string s = std::to_string(mag);
  std::string out;
  const int n = (int)s.size();
  for (int i = 0; i < n; ++i) {
    out.push_back(s[i]);
    if ((n - 1 - i) % 3 == 0 && i + 1 < n) out.push_back(',');
  }
  return neg ? "-" + out : out;
}

// Tiles.GetFile (:81-102)
std::string tile_file(int level, int64_t tile_id, const char* suffix) {
  const TileLevel t = tile_level(level);
  int64_t max_length = digits(t.max_tile_id);
  const int64_t rem = max_length % 3;
  if (rem) max_length += 3 - rem;
  int64_t p = 1;
  for (int64_t k = 0; k < max_length; ++k) p *= 10;
  std::string f = with_commas((level == 0 ? p : (int64_t)level * p) + tile_id);
  std::replace(f.begin(), f.end(), ',', '/');
  f += ".";
  f += suffix;
  if (level == 0) f = "0" + f.substr(1);  // :93-95
  return f;
}

// ---- flattener ------------------------------------------------------------------------
double seg_len_m(int32_t la, int32_t lo, int32_t lb, int32_t lob) {
  const double lat1 = la * 1e-6, lon1 = lo * 1e-6, lat2 = lb * 1e-6, lon2 = lob * 1e-6;
  const double x = (lon1 - lon2) * kMetersPerDeg * std::cos(0.5 * (lat1 + lat2) * M_PI / 180.0);
  const double y = (lat1 - lat2) * kMetersPerDeg;
  return std::sqrt(x * x + y * y);
}

struct Dsu {
  std::vector<uint32_t> p;
  explicit Dsu(uint32_t n) : p(n) { std::iota(p.begin(), p.end(), 0u); }
  uint32_t find(uint32_t x) {
    while (p[x] != x) x = p[x] = p[p[x]];
    return x;
  }
  void unite(uint32_t a, uint32_t b) {  // the smaller id represents the set
    a = find(a);
    b = find(b);
    if (a == b) return;
    if (a < b) p[b] = a;
    else p[a] = b;
  }
};

template <class T>
bool write_arr(FILE* f, const std::vector<T>& v, uint64_t* off) {
  const long pos = ftell(f);
  const long pad = (64 - pos % 64) % 64;
  static const char zeros[64] = {0};
  if (pad && fwrite(zeros, 1, (size_t)pad, f) != (size_t)pad) return false;
  *off = (uint64_t)(pos + pad);
  return v.empty() || fwrite(v.data(), sizeof(T), v.size(), f) == v.size();
}

thread_local std::string g_err;

}  // namespace

extern "C" {

int32_t otr_tilehier_row(int32_t level, double lat) {
  if (level < 0 || level > 2) return -1;
  return (int32_t)tile_row(tile_level(level), lat);
}

int32_t otr_tilehier_col(int32_t level, double lon) {
  if (level < 0 || level > 2) return -1;
  return (int32_t)tile_col(tile_level(level), lon);
}

int otr_tilehier_file(int32_t level, int64_t tile_id, const char* suffix, char* out, size_t cap) {
  if (level < 0 || level > 2 || !suffix || !out) return OTR_BAD_REQUEST;
  const std::string f = tile_file(level, tile_id, suffix);
  if (f.size() + 1 > cap) return OTR_BAD_REQUEST;
  memcpy(out, f.c_str(), f.size() + 1);
  return OTR_OK;
}

int otr_tilehier_files(double min_lon, double min_lat, double max_lon, double max_lat, const char* suffix, char** out,
                   size_t* out_len) {
  if (!suffix || !out || !out_len) return OTR_BAD_REQUEST;
  // get_tiles.py:143-159: one bbox, or two when it crosses the antimeridian
  double b[4] = {min_lon, min_lat, max_lon, max_lat};
  if (b[0] >= b[2]) b[0] -= 360.0;
  std::vector<std::array<double, 4>> boxes;
  const double range = 180.0 - -180.0;
  if (b[0] < -180.0 && b[2] > -180.0) {
    boxes.push_back({-180.0, b[1], b[2], b[3]});
    boxes.push_back({b[0] + range, b[1], 180.0, b[3]});
  } else if (b[0] < 180.0 && b[2] > 180.0) {
    boxes.push_back({b[0], b[1], 180.0, b[3]});
    boxes.push_back({-180.0, b[1], b[2] - range, b[3]});
  } else {
    boxes.push_back({b[0], b[1], b[2], b[3]});
  }
  std::string text;
  for (const auto& bx : boxes)  // :161-171, levels in Python 2 dict order 0, 1, 2
    for (int level = 0; level <= 2; ++level) {
      const TileLevel t = tile_level(level);
      const int64_t mincol = tile_col(t, bx[0]);
      for (int64_t i = tile_row(t, bx[1]); i <= tile_row(t, bx[3]); ++i) {
        int64_t tile_id = i * t.ncolumns + mincol;
        for (int64_t j = mincol; j <= tile_col(t, bx[2]); ++j, ++tile_id) {
          text += tile_file(level, tile_id, suffix);
          text += '\n';
        }
      }
    }
  char* buf = (char*)malloc(text.size() + 1);
  if (!buf) return OTR_DEVICE_ERROR;
  memcpy(buf, text.c_str(), text.size() + 1);
  *out = buf;
  *out_len = text.size();
  return OTR_OK;
}

int otr_flatten(const otr_flat_graph* in, const char* out_path, otr_flat_stats* stats) {
  if (!in || !out_path || (in->n_nodes && !in->node_ll) ||
      (in->n_edges && (!in->edge_src || !in->edge_dst || !in->edge_attr || !in->shape_off || !in->shape_ll)) ||
      (in->n_segments && (!in->seg_id || !in->seg_len)))
    return OTR_BAD_REQUEST;
  const uint32_t N = in->n_nodes, E = in->n_edges;
  for (uint32_t e = 0; e < E; ++e) {
    if (in->edge_src[e] >= N || in->edge_dst[e] >= N) return OTR_BAD_REQUEST;
    if (in->shape_off[e + 1] < in->shape_off[e] + 2) return OTR_BAD_REQUEST;  // both end points at least
    const uint32_t sg = in->edge_seg ? in->edge_seg[e] : OTR_NO_SEGMENT;
    if (sg != OTR_NO_SEGMENT && sg >= in->n_segments) return OTR_BAD_REQUEST;
  }
  const double cell_deg = in->cell_deg > 0 ? in->cell_deg : 0.0005;
  // shapes with their end points on the nodes
  std::vector<std::vector<std::pair<int32_t, int32_t>>> shp(E);
  for (uint32_t e = 0; e < E; ++e) {
    for (uint32_t k = in->shape_off[e]; k < in->shape_off[e + 1]; ++k)
      shp[e].push_back({in->shape_ll[2 * (size_t)k], in->shape_ll[2 * (size_t)k + 1]});
  }
  auto shape_len = [](const std::vector<std::pair<int32_t, int32_t>>& s) {
    double len = 0;
    for (size_t k = 1; k < s.size(); ++k) len += seg_len_m(s[k - 1].first, s[k - 1].second, s[k].first, s[k].second);
    return len;
  };
  // contract edges < 5 cm until none is left (moving end points can shorten others)
  Dsu dsu(N);
  std::vector<uint32_t> src(in->edge_src, in->edge_src + E), dst(in->edge_dst, in->edge_dst + E);
  std::vector<uint32_t> attr(in->edge_attr, in->edge_attr + E);
  std::vector<char> alive(E, 1);
  std::vector<int32_t> nll(in->node_ll, in->node_ll + 2 * (size_t)N);
  uint32_t n_contracted = 0;
  std::vector<std::vector<uint32_t>> seg_edges;  // built on the first flag transfer
  for (int pass = 0; pass < 64; ++pass) {
    bool any = false;
    for (uint32_t e = 0; e < E; ++e)
      if (alive[e] && dsu.find(src[e]) != dsu.find(dst[e]) && shape_len(shp[e]) < kMinEdgeM) {
        dsu.unite(src[e], dst[e]);
        any = true;
      }
    // edges inside one cluster vanish (short ones, and those whose distinct end nodes
    // merged); their segment flags move to the same segment's neighbouring edge; the
    // others — a true self-loop (a loop road) of 5 cm or more included — are re-attached
    // to the clusters' representatives
    for (uint32_t e = 0; e < E; ++e) {
      if (!alive[e]) continue;
      const uint32_t s = dsu.find(src[e]), d = dsu.find(dst[e]);
      if (s == d && (in->edge_src[e] != in->edge_dst[e] || shape_len(shp[e]) < kMinEdgeM)) {
        alive[e] = 0;
        ++n_contracted;
        const uint32_t sg = in->edge_seg ? in->edge_seg[e] : OTR_NO_SEGMENT;
        if (sg != OTR_NO_SEGMENT && (attr[e] & (OTR_ATTR_SEG_BEGIN | OTR_ATTR_SEG_END))) {
          if (seg_edges.empty()) {
            seg_edges.resize(in->n_segments);
            for (uint32_t f = 0; f < E; ++f)
              if (in->edge_seg[f] != OTR_NO_SEGMENT) seg_edges[in->edge_seg[f]].push_back(f);
          }
          for (const uint32_t f : seg_edges[sg]) {
            if (!alive[f] || f == e) continue;
            if ((attr[e] & OTR_ATTR_SEG_BEGIN) && dsu.find(src[f]) == s) attr[f] |= OTR_ATTR_SEG_BEGIN;
            if ((attr[e] & OTR_ATTR_SEG_END) && dsu.find(dst[f]) == s) attr[f] |= OTR_ATTR_SEG_END;
          }
        }
        continue;
      }
      if (s != src[e] || d != dst[e]) {
        src[e] = s;
        dst[e] = d;
        shp[e].front() = {nll[2 * (size_t)s], nll[2 * (size_t)s + 1]};
        shp[e].back() = {nll[2 * (size_t)d], nll[2 * (size_t)d + 1]};
      }
    }
    if (!any) break;
  }
  // surviving nodes renumbered in id order
  std::vector<uint32_t> new_id(N, OTR_NO_SEGMENT);
  uint32_t n_nodes = 0;
  for (uint32_t v = 0; v < N; ++v)
    if (dsu.find(v) == v) new_id[v] = n_nodes++;
  std::vector<uint32_t> order;
  for (uint32_t e = 0; e < E; ++e)
    if (alive[e]) order.push_back(e);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    const uint32_t sa = new_id[src[a]], sb = new_id[src[b]];
    return sa != sb ? sa < sb : new_id[dst[a]] < new_id[dst[b]];
  });
  const uint32_t n_edges = (uint32_t)order.size();
  std::vector<int32_t> node_ll(2 * (size_t)n_nodes);
  for (uint32_t v = 0; v < N; ++v)
    if (new_id[v] != OTR_NO_SEGMENT) {
      node_ll[2 * (size_t)new_id[v]] = nll[2 * (size_t)v];
      node_ll[2 * (size_t)new_id[v] + 1] = nll[2 * (size_t)v + 1];
    }
  std::vector<uint32_t> node_row(n_nodes + 1, 0), edge_src(n_edges), edge_dst(n_edges), edge_attr(n_edges),
      edge_shape(n_edges + 1), edge_seg(n_edges), edge_way(n_edges);
  std::vector<float> edge_len(n_edges);
  std::vector<int32_t> shape_ll;
  for (uint32_t k = 0; k < n_edges; ++k) {
    const uint32_t e = order[k];
    edge_src[k] = new_id[src[e]];
    edge_dst[k] = new_id[dst[e]];
    node_row[edge_src[k] + 1]++;
    edge_attr[k] = attr[e];
    edge_seg[k] = in->edge_seg ? in->edge_seg[e] : OTR_NO_SEGMENT;
    edge_way[k] = in->edge_way ? in->edge_way[e] : 0u;
    edge_shape[k] = (uint32_t)(shape_ll.size() / 2);
    for (const auto& pt : shp[e]) {
      shape_ll.push_back(pt.first);
      shape_ll.push_back(pt.second);
    }
    edge_len[k] = (float)shape_len(shp[e]);
  }
  edge_shape[n_edges] = (uint32_t)(shape_ll.size() / 2);
  for (uint32_t v = 0; v < n_nodes; ++v) node_row[v + 1] += node_row[v];
  std::vector<uint32_t> rev_row(n_nodes + 1, 0), rev_edge(n_edges);
  for (uint32_t e = 0; e < n_edges; ++e) rev_row[edge_dst[e] + 1]++;
  for (uint32_t v = 0; v < n_nodes; ++v) rev_row[v + 1] += rev_row[v];
  {
    std::vector<uint32_t> fill(rev_row.begin(), rev_row.end() - 1);
    for (uint32_t e = 0; e < n_edges; ++e) rev_edge[fill[edge_dst[e]]++] = e;
  }
  std::vector<uint64_t> seg_id(in->seg_id, in->seg_id + in->n_segments);
  std::vector<uint32_t> seg_len(in->seg_len, in->seg_len + in->n_segments);
  // grid index (include/otr_graph_format.h): every cell a padded shape-segment box touches
  int32_t mnla = INT32_MAX, mnlo = INT32_MAX, mxla = INT32_MIN, mxlo = INT32_MIN;
  for (size_t k = 0; k < shape_ll.size(); k += 2) {
    mnla = std::min(mnla, shape_ll[k]);
    mxla = std::max(mxla, shape_ll[k]);
    mnlo = std::min(mnlo, shape_ll[k + 1]);
    mxlo = std::max(mxlo, shape_ll[k + 1]);
  }
  if (shape_ll.empty()) mnla = mnlo = mxla = mxlo = 0;
  const double gmin_lat = std::floor(mnla * 1e-6 / cell_deg) * cell_deg - cell_deg;
  const double gmin_lon = std::floor(mnlo * 1e-6 / cell_deg) * cell_deg - cell_deg;
  const uint64_t grows = (uint64_t)std::ceil((mxla * 1e-6 - gmin_lat) / cell_deg) + 2;
  const uint64_t gcols = (uint64_t)std::ceil((mxlo * 1e-6 - gmin_lon) / cell_deg) + 2;
  if (grows * gcols >= 0xFFFFFFFFull) {
    g_err = "grid too large: raise cell_deg";
    return OTR_BAD_REQUEST;
  }
  const uint32_t n_cells = (uint32_t)(grows * gcols);
  std::vector<std::pair<uint32_t, uint32_t>> ce;
  for (uint32_t e = 0; e < n_edges; ++e) {
    const size_t first = ce.size();
    for (uint32_t k = edge_shape[e]; k + 1 < edge_shape[e + 1]; ++k) {
      const double la0 = shape_ll[2 * (size_t)k] * 1e-6, lo0 = shape_ll[2 * (size_t)k + 1] * 1e-6;
      const double la1 = shape_ll[2 * (size_t)k + 2] * 1e-6, lo1 = shape_ll[2 * (size_t)k + 3] * 1e-6;
      const double a = std::min(la0, la1) - OTR_GRID_PAD_DEG, b = std::max(la0, la1) + OTR_GRID_PAD_DEG;
      const double c = std::min(lo0, lo1) - OTR_GRID_PAD_DEG, d = std::max(lo0, lo1) + OTR_GRID_PAD_DEG;
      const int64_t r0 = (int64_t)std::floor((a - gmin_lat) / cell_deg), r1 = (int64_t)std::floor((b - gmin_lat) / cell_deg);
      const int64_t c0 = (int64_t)std::floor((c - gmin_lon) / cell_deg), c1 = (int64_t)std::floor((d - gmin_lon) / cell_deg);
      for (int64_t r = std::max<int64_t>(r0, 0); r <= std::min<int64_t>(r1, (int64_t)grows - 1); ++r)
        for (int64_t cc = std::max<int64_t>(c0, 0); cc <= std::min<int64_t>(c1, (int64_t)gcols - 1); ++cc)
          ce.push_back({(uint32_t)(r * (int64_t)gcols + cc), e});
    }
    std::sort(ce.begin() + first, ce.end());
    ce.erase(std::unique(ce.begin() + first, ce.end()), ce.end());
  }
  std::sort(ce.begin(), ce.end());
  std::vector<uint32_t> cell_row((size_t)n_cells + 1, 0), cell_edge(ce.size());
  for (size_t k = 0; k < ce.size(); ++k) {
    cell_row[ce[k].first + 1]++;
    cell_edge[k] = ce[k].second;
  }
  for (uint32_t c = 0; c < n_cells; ++c) cell_row[c + 1] += cell_row[c];

  FILE* f = fopen(out_path, "wb");
  if (!f) {
    g_err = "cannot open output";
    return OTR_BAD_REQUEST;
  }
  otr_graph_header h;
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, OTR_GRAPH_MAGIC, 8);
  h.version = OTR_GRAPH_VERSION;
  h.n_nodes = n_nodes;
  h.n_edges = n_edges;
  h.n_shape = (uint32_t)(shape_ll.size() / 2);
  h.n_segments = (uint32_t)seg_id.size();
  h.n_cells = n_cells;
  h.n_cell_entries = (uint32_t)cell_edge.size();
  h.grid_rows = (uint32_t)grows;
  h.grid_cols = (uint32_t)gcols;
  h.grid_min_lat = gmin_lat;
  h.grid_min_lon = gmin_lon;
  h.grid_cell_deg = cell_deg;
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
  ok = ok && write_arr(f, node_row, &h.array_offset[OTR_A_NODE_ROW]);
  ok = ok && write_arr(f, node_ll, &h.array_offset[OTR_A_NODE_LL]);
  ok = ok && write_arr(f, rev_row, &h.array_offset[OTR_A_REV_ROW]);
  ok = ok && write_arr(f, rev_edge, &h.array_offset[OTR_A_REV_EDGE]);
  ok = ok && write_arr(f, edge_src, &h.array_offset[OTR_A_EDGE_SRC]);
  ok = ok && write_arr(f, edge_dst, &h.array_offset[OTR_A_EDGE_DST]);
  ok = ok && write_arr(f, edge_len, &h.array_offset[OTR_A_EDGE_LEN]);
  ok = ok && write_arr(f, edge_attr, &h.array_offset[OTR_A_EDGE_ATTR]);
  ok = ok && write_arr(f, edge_shape, &h.array_offset[OTR_A_EDGE_SHAPE]);
  ok = ok && write_arr(f, edge_seg, &h.array_offset[OTR_A_EDGE_SEG]);
  ok = ok && write_arr(f, edge_way, &h.array_offset[OTR_A_EDGE_WAY]);
  ok = ok && write_arr(f, shape_ll, &h.array_offset[OTR_A_SHAPE_LL]);
  ok = ok && write_arr(f, seg_id, &h.array_offset[OTR_A_SEG_ID]);
  ok = ok && write_arr(f, seg_len, &h.array_offset[OTR_A_SEG_LEN]);
  ok = ok && write_arr(f, cell_row, &h.array_offset[OTR_A_CELL_ROW]);
  ok = ok && write_arr(f, cell_edge, &h.array_offset[OTR_A_CELL_EDGE]);
  h.array_offset[OTR_A_END] = (uint64_t)ftell(f);
  ok = ok && fseek(f, 0, SEEK_SET) == 0 && fwrite(&h, sizeof(h), 1, f) == 1;
  ok = (fclose(f) == 0) && ok;
  if (!ok) {
    g_err = "write failed";
    return OTR_DEVICE_ERROR;
  }
  if (stats) {
    stats->n_nodes = n_nodes;
    stats->n_edges = n_edges;
    stats->n_contracted_edges = n_contracted;
    stats->n_merged_nodes = N - n_nodes;
  }
  return OTR_OK;
}

}  // extern "C"
