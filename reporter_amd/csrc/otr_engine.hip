// otr_engine.hip — graph upload (flattened CSR + grid → HBM) and the batched
// matching pipeline on one HIP stream.  Kernels: otr_kernels.h.
#include <hipcub/hipcub.hpp>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "otr_engine.h"
#include "otr_kernels.h"
#include "otr_edge.h"
#include "otr_edge1.h"
#include "otr_ingest.h"
#include "otr_launch.h"

namespace otr {
static_assert(kTraceWaves == 4, "grid_trace_rows (otr_launch.h) assumes 4 traces per block");

#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      if (err) *err = std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x;    \
      return OTR_DEVICE_ERROR;                                                           \
    }                                                                                    \
  } while (0)

void finalize_params(MatchParams* p) {
  p->inv2s2 = 1.0 / (p->sigma_z * p->sigma_z * 2.0);
  p->inv_beta = 1.0 / p->beta;
  if (p->kmax > OTR_KMAX) p->kmax = OTR_KMAX;
  if (p->kmax < 1) p->kmax = 1;
}

// values the engine cannot honour are refused by name (400), never silently changed
const char* check_params(const MatchParams& p) {
  if (!(p.breakage_distance >= 0.0 && p.breakage_distance <= kMaxBreakage))
    return "breakage_distance must be within [0, 30000] m";
  if (!(p.max_route_distance_factor >= 0.0) || !(p.max_route_distance_factor < 1e6))
    return "max_route_distance_factor must be >= 0";
  if (!(p.max_route_time_factor >= 0.0) || !(p.max_route_time_factor < 1e6)) return "max_route_time_factor must be >= 0";
  if (!(p.turn_penalty_factor >= 0.0) || !(p.turn_penalty_factor <= 1e6)) return "turn_penalty_factor must be within [0, 1e6]";
  if (!(p.sigma_z > 0.0)) return "sigma_z must be > 0";
  if (!(p.beta > 0.0)) return "beta must be > 0";
  if (!(p.search_radius >= 0.0) || !(p.max_search_radius >= 0.0)) return "search_radius must be >= 0";
  if (!(p.interpolation_distance >= 0.0)) return "interpolation_distance must be >= 0";
  if (!(p.speed_kph >= 0.0) || !(p.queue_kph >= 0.0)) return "speed_kph and queue_kph must be >= 0";
  return nullptr;
}

ModeParams default_mode_params() {
  ModeParams mp{};
  for (int m = 0; m < OTR_MODES; ++m) {
    MatchParams& p = mp.m[m];
    p.sigma_z = 4.07;                   // Dockerfile:14
    p.beta = 3.0;                       // Dockerfile:15
    p.max_route_distance_factor = 5.0;  // Dockerfile:16
    p.max_route_time_factor = 2.0;      // Dockerfile:17,48 (MATCHER_TIME_FACTOR)
    p.breakage_distance = 2000.0;
    p.interpolation_distance = 10.0;
    p.search_radius = 50.0;
    p.max_search_radius = 100.0;
    p.gps_accuracy = 5.0;
    p.kmax = 32;
    p.queue_kph = 10.0;
  }
  // valhalla_build_config per-mode meili sections; mode speeds and queue
  // thresholds of DESIGN.md §3.5/3.8
  mp.m[0].turn_penalty_factor = 200.0;
  mp.m[1].turn_penalty_factor = 140.0;
  mp.m[1].speed_kph = 18.0;
  mp.m[1].queue_kph = 5.0;
  mp.m[2].turn_penalty_factor = 100.0;
  mp.m[2].speed_kph = 5.1;
  mp.m[2].queue_kph = 2.0;
  for (int m = 0; m < OTR_MODES; ++m) finalize_params(&mp.m[m]);
  mp.delta = 60.0;  // round width (m): search order only; C2 39.3M -> 39.7M, C4 4.35M -> ~4.4M single stream vs 100
  return mp;
}

// route time of an edge at the mode's speed, 0.1 s (oracle edge_time_ds)
static uint32_t edge_time_ds(uint32_t attr, uint32_t len_mm, double speed_cap) {
  double kph = (double)OTR_ATTR_SPEED(attr);
  if (!(kph > 0.0)) kph = 30.0;  // unknown speed
  if (speed_cap > 0.0 && speed_cap < kph) kph = speed_cap;
  const double v = (double)len_mm * 0.036 / kph;
  return v < 2.0e9 ? (uint32_t)llround(v) : 2000000000u;
}

// heading of the shape segment a -> b, integer degrees clockwise from north, -1 when
// degenerate (oracle seg_heading)
static int seg_heading(const int32_t* a, const int32_t* b) {
  const double la1 = (double)a[0] * 1e-6, lo1 = (double)a[1] * 1e-6;
  const double la2 = (double)b[0] * 1e-6, lo2 = (double)b[1] * 1e-6;
  const double m = 20037581.187 / 180.0;  // metres per degree, Batch.java:36
  const double x = (lo2 - lo1) * m * cos_deg(0.5 * (la1 + la2));
  const double y = (la2 - la1) * m;
  if (x == 0.0 && y == 0.0) return -1;
  double deg = atan2(x, y) * (180.0 / 3.14159265358979323846);
  if (deg < 0.0) deg = deg + 360.0;
  return (int)(llround(deg) % 360);
}

void turn_table(double factor, int32_t* tab) {
  const double x = -1.0 / 45.0;  // e^(-1/45) by its Taylor series, then powers
  double r = 1.0, term = 1.0;
  for (int k = 1; k <= 20; ++k) {
    term = term * x / (double)k;
    r = r + term;
  }
  double f = 1.0;
  for (int i = 0; i <= 180; ++i) {
    const double v = 1000.0 * factor * f;
    tab[i] = factor > 0.0 ? (int32_t)llround(v) : 0;
    f = f * r;
  }
}

GraphState& graph_state() {
  static GraphState gs;
  return gs;
}

namespace {
struct Mapped {
  void* p = MAP_FAILED;
  size_t n = 0;
  ~Mapped() {
    if (p != MAP_FAILED) munmap(p, n);
  }
};
struct Staged {  // a graph replica being built; freed unless adopted
  std::vector<void*> allocs;
  bool adopted = false;
  ~Staged() {
    if (!adopted)
      for (void* q : allocs) (void)hipFree(q);
  }
};
}  // namespace

int engine_configure(const Config& cfg, std::string* err) {
  for (int m = 0; m < OTR_MODES; ++m)
    if (const char* bad = check_params(cfg.mp.m[m])) {
      if (err) *err = std::string("config: ") + bad;
      return OTR_BAD_REQUEST;
    }
  int fd = open(cfg.graph_path.c_str(), O_RDONLY);
  if (fd < 0) {
    if (err) *err = "cannot open graph file " + cfg.graph_path + ": " + strerror(errno);
    return OTR_BAD_REQUEST;
  }
  struct stat st;
  fstat(fd, &st);
  Mapped mf;
  mf.n = (size_t)st.st_size;
  mf.p = mf.n >= sizeof(otr_graph_header) ? mmap(nullptr, mf.n, PROT_READ, MAP_PRIVATE, fd, 0) : MAP_FAILED;
  close(fd);
  if (mf.p == MAP_FAILED) {
    if (err) *err = "cannot map graph file " + cfg.graph_path;
    return OTR_BAD_REQUEST;
  }
  const char* base = (const char*)mf.p;
  otr_graph_header h;
  memcpy(&h, base, sizeof(h));
  if (memcmp(h.magic, OTR_GRAPH_MAGIC, 8) != 0 || h.version != OTR_GRAPH_VERSION ||
      h.array_offset[OTR_A_END] > (uint64_t)st.st_size) {
    if (err) *err = "not an OTR graph file: " + cfg.graph_path;
    return OTR_BAD_REQUEST;
  }
  if (h.n_nodes >= (1u << 28)) {  // adj packs dst in 28 bits
    if (err) *err = "graph has more than 2^28 nodes";
    return OTR_BAD_REQUEST;
  }
  if (h.n_edges >= (1u << 28)) {  // the edge-state records pack the out-edge id in 28 bits (erec)
    if (err) *err = "graph has more than 2^28 directed edges";
    return OTR_BAD_REQUEST;
  }
  const uint32_t* dst = (const uint32_t*)(base + h.array_offset[OTR_A_EDGE_DST]);
  const float* lenf = (const float*)(base + h.array_offset[OTR_A_EDGE_LEN]);
  const uint32_t* attr = (const uint32_t*)(base + h.array_offset[OTR_A_EDGE_ATTR]);
  const uint32_t* row = (const uint32_t*)(base + h.array_offset[OTR_A_NODE_ROW]);
  const int32_t* nll = (const int32_t*)(base + h.array_offset[OTR_A_NODE_LL]);
  const uint32_t* eshape = (const uint32_t*)(base + h.array_offset[OTR_A_EDGE_SHAPE]);
  const int32_t* sll = (const int32_t*)(base + h.array_offset[OTR_A_SHAPE_LL]);
  // ---- host-side validation and derived views (nothing on the device is touched yet)
  // len_mm = round(len * 1000), >= 1 mm: the integer routing length the oracle derives
  // the same way
  std::vector<uint32_t> len(h.n_edges + 1, 0u);
  for (uint32_t e = 0; e < h.n_edges; ++e) {
    const double mm = (double)lenf[e] * 1000.0;
    if (!(mm >= 0.0 && mm < 2.0e9)) {  // uint32 label arithmetic
      if (err) *err = "graph edge length outside [0, 2000 km)";
      return OTR_BAD_REQUEST;
    }
    len[e] = (uint32_t)std::max(1LL, (long long)llround(mm));
  }
  for (uint32_t u = 0; u < h.n_nodes; ++u)
    if (row[u + 1] < row[u] || row[u + 1] > h.n_edges) {
      if (err) *err = "graph CSR rows are not monotone";
      return OTR_BAD_REQUEST;
    }
  for (uint32_t e = 0; e < h.n_edges; ++e)
    if (dst[e] >= h.n_nodes || eshape[e + 1] < eshape[e] + 2 || eshape[e + 1] > h.n_shape) {
      if (err) *err = "graph edge " + std::to_string(e) + " has a bad end node or shape range";
      return OTR_BAD_REQUEST;
    }
  // minin(v): the shortest in-edge of every node (mm, any mode: a lower bound for each),
  // the IN criterion of the exact search rounds; 0xFFFFFFFF: no in-edge
  std::vector<uint32_t> minin(h.n_nodes + 1, 0xFFFFFFFFu);
  for (uint32_t e = 0; e < h.n_edges; ++e) minin[dst[e]] = std::min(minin[dst[e]], len[e]);
  std::vector<uint4> pack(h.n_edges + 1);
  for (uint32_t e = 0; e < h.n_edges; ++e) pack[e] = make_uint4(dst[e], len[e], attr[e], minin[dst[e]]);
  // per edge what k_prep needs of a candidate's edge in one 16-B gather: {len_mm, src,
  // minin(src), dst} (no dependent minin load; C5's country graph misses the L2 there)
  std::vector<uint4> eprep(h.n_edges + 1, make_uint4(0u, 0u, 0u, 0u));
  {
    const uint32_t* srcv = (const uint32_t*)(base + h.array_offset[OTR_A_EDGE_SRC]);
    for (uint32_t e = 0; e < h.n_edges; ++e) eprep[e] = make_uint4(len[e], srcv[e], minin[srcv[e]], dst[e]);
  }
  // per-node adjacency records: the first 4 out-edges of a node in one 64-B record,
  // {dst | access<<28 | more<<31, len_mm, minin(dst), 0} per edge
  std::vector<uint4> adj(4ull * h.n_nodes + 4, make_uint4(kAdjDstMask, 0u, 0u, 0u));
  for (uint32_t u = 0; u < h.n_nodes; ++u) {
    const uint32_t deg = row[u + 1] - row[u];
    for (uint32_t k = 0; k < deg && k < 4; ++k) {
      const uint32_t e = row[u] + k;
      adj[4ull * u + k] = make_uint4(dst[e] | ((attr[e] & OTR_ATTR_ACCESS_MASK) << 28), len[e], minin[dst[e]], 0u);
    }
    if (deg > 4) adj[4ull * u + 3].x |= kAdjMore;
  }
  // route times per mode (0.1 s) per edge and per adjacency slot
  std::vector<uint32_t> et[OTR_MODES], at[OTR_MODES];
  for (int m = 0; m < OTR_MODES; ++m) {
    et[m].assign(h.n_edges + 1, 0u);
    for (uint32_t e = 0; e < h.n_edges; ++e) et[m][e] = edge_time_ds(attr[e], len[e], cfg.mp.m[m].speed_kph);
    at[m].assign(4ull * h.n_nodes + 4, 0u);
    for (uint32_t u = 0; u < h.n_nodes; ++u)
      for (uint32_t k = 0; k < 4 && row[u] + k < row[u + 1]; ++k) at[m][4ull * u + k] = et[m][row[u] + k];
  }
  // edge headings: first / last non-degenerate shape segment (oracle orc_graph_load)
  std::vector<short2> head(h.n_edges + 1, make_short2(0, 0));
  for (uint32_t e = 0; e < h.n_edges; ++e) {
    const uint32_t k0 = eshape[e], k1 = eshape[e + 1];
    int hb = -1, he = -1;
    for (uint32_t k = k0; k + 1 < k1 && hb < 0; ++k) hb = seg_heading(sll + 2ull * k, sll + 2ull * k + 2);
    for (uint32_t k = k1 - 1; k > k0 && he < 0; --k) he = seg_heading(sll + 2ull * k - 2, sll + 2ull * k);
    head[e] = make_short2((short)(hb < 0 ? 0 : hb), (short)(he < 0 ? 0 : he));
  }
  // edge-state view of the adjacency slots (turn-cost searches, otr_edge.h): the slot's
  // edge id and its begin / end headings
  std::vector<uint2> adje(4ull * h.n_nodes + 4, make_uint2(0u, 0u));
  for (uint32_t u = 0; u < h.n_nodes; ++u)
    for (uint32_t k = 0; k < 4 && row[u] + k < row[u + 1]; ++k) {
      const uint32_t e = row[u] + k;
      adje[4ull * u + k] = make_uint2(e, (uint32_t)(uint16_t)head[e].x | ((uint32_t)(uint16_t)head[e].y << 16));
    }
  // edge-state view (otr_edge1.h): per edge state b (arrived at v = dst(b)) one 16-B record
  // per out-edge slot k < 4 of v: {e | access(e) << 28 | more << 31, len_mm(e), the turn
  // degree b -> e | b's end heading << 8, v}, and per mode the slot's route time in a
  // parallel array: a relaxation is one record load and one time load at the same index,
  // with the turn already resolved
  const size_t es = 4ull * h.n_edges + 4;
  std::vector<uint4> erec(es, make_uint4(kAdjDstMask, 0u, 0u, 0u));
  std::vector<uint32_t> erec_t(es * OTR_MODES, 0u);
  for (uint32_t b = 0; b < h.n_edges; ++b) {
    const uint32_t v = dst[b], deg = row[v + 1] - row[v];
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t hend = (uint32_t)(uint16_t)head[b].y << 8;  // b's end heading (target offers)
      if (k >= deg) {
        erec[4ull * b + k] = make_uint4(kAdjDstMask, 0u, hend, v);  // (access 0: never relaxed)
        continue;
      }
      const uint32_t e = row[v] + k;
      const uint32_t x = e | ((attr[e] & OTR_ATTR_ACCESS_MASK) << 28) | ((k == 3 && deg > 4) ? kAdjMore : 0u);
      erec[4ull * b + k] =
          make_uint4(x, len[e], (uint32_t)turn_degree((int)head[b].y, (int)head[e].x) | hend, v);
      for (int m = 0; m < OTR_MODES; ++m) erec_t[es * m + 4ull * b + k] = std::min(et[m][e], 0x1FFFFu);
    }
  }
  // candidate-search view: each grid-cell entry carries its edge's shape range and
  // attributes, 48 B per entry: {edge, shape begin, shape end, attr} + the first four shape points
  const uint32_t* cedge = (const uint32_t*)(base + h.array_offset[OTR_A_CELL_EDGE]);
  std::vector<uint4> crec(3 * ((size_t)h.n_cell_entries + 1), make_uint4(0u, 0u, 0u, 0u));
  for (uint64_t q = 0; q < h.n_cell_entries; ++q) {
    const uint32_t e = cedge[q];
    if (e >= h.n_edges) {
      if (err) *err = "graph cell index names a missing edge";
      return OTR_BAD_REQUEST;
    }
    const uint32_t k0 = eshape[e], k1 = eshape[e + 1];
    crec[3 * q] = make_uint4(e, k0, k1, attr[e]);
    uint32_t pt[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < 4 && k0 + i < k1; ++i) {
      pt[2 * i] = (uint32_t)sll[2ull * (k0 + i)];
      pt[2 * i + 1] = (uint32_t)sll[2ull * (k0 + i) + 1];
    }
    crec[3 * q + 1] = make_uint4(pt[0], pt[1], pt[2], pt[3]);
    crec[3 * q + 2] = make_uint4(pt[4], pt[5], pt[6], pt[7]);
  }
  // ---- upload into a staged replica
  HIPCHK(hipSetDevice(cfg.device));
  Staged sg;
  bool alloc_ok = true;
  auto upv = [&](const void* src, size_t bytes) -> void* {
    void* d = nullptr;
    if (hipMalloc(&d, bytes ? bytes : 16) != hipSuccess) {
      alloc_ok = false;
      return nullptr;
    }
    sg.allocs.push_back(d);
    if (bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) alloc_ok = false;
    return d;
  };
  auto up = [&](int a, size_t bytes) -> void* { return upv(base + h.array_offset[a], bytes); };
  DevGraph g{};
  g.node_row = (const uint32_t*)up(OTR_A_NODE_ROW, 4ull * (h.n_nodes + 1));
  g.rev_row = (const uint32_t*)up(OTR_A_REV_ROW, 4ull * (h.n_nodes + 1));
  g.node_ll = (const int2*)up(OTR_A_NODE_LL, 8ull * h.n_nodes);
  g.rev_edge = (const uint32_t*)up(OTR_A_REV_EDGE, 4ull * h.n_edges);
  g.edge_src = (const uint32_t*)up(OTR_A_EDGE_SRC, 4ull * h.n_edges);
  g.edge_dst = (const uint32_t*)up(OTR_A_EDGE_DST, 4ull * h.n_edges);
  g.edge_len = (const float*)up(OTR_A_EDGE_LEN, 4ull * h.n_edges);
  g.edge_attr = (const uint32_t*)up(OTR_A_EDGE_ATTR, 4ull * h.n_edges);
  g.edge_shape = (const uint32_t*)up(OTR_A_EDGE_SHAPE, 4ull * (h.n_edges + 1));
  g.edge_seg = (const uint32_t*)up(OTR_A_EDGE_SEG, 4ull * h.n_edges);
  g.edge_way = (const uint32_t*)up(OTR_A_EDGE_WAY, 4ull * h.n_edges);
  g.shape_ll = (const int2*)up(OTR_A_SHAPE_LL, 8ull * h.n_shape);
  g.seg_id = (const unsigned long long*)up(OTR_A_SEG_ID, 8ull * h.n_segments);
  g.seg_len = (const uint32_t*)up(OTR_A_SEG_LEN, 4ull * h.n_segments);
  g.cell_row = (const uint32_t*)up(OTR_A_CELL_ROW, 4ull * (h.n_cells + 1));
  g.cell_edge = (const uint32_t*)up(OTR_A_CELL_EDGE, 4ull * h.n_cell_entries);
  g.len_mm = (const uint32_t*)upv(len.data(), 4ull * len.size());
  g.edge_pack = (const uint4*)upv(pack.data(), sizeof(uint4) * pack.size());
  g.eprep = (const uint4*)upv(eprep.data(), sizeof(uint4) * eprep.size());
  g.adj = (const uint4*)upv(adj.data(), sizeof(uint4) * adj.size());
  g.node_minin = (const uint32_t*)upv(minin.data(), 4ull * minin.size());
  {
    std::vector<uint32_t> all_et, all_at;
    for (int m = 0; m < OTR_MODES; ++m) {
      all_et.insert(all_et.end(), et[m].begin(), et[m].end());
      all_at.insert(all_at.end(), at[m].begin(), at[m].end());
    }
    g.edge_t = (const uint32_t*)upv(all_et.data(), 4ull * all_et.size());
    g.adj_t = (const uint32_t*)upv(all_at.data(), 4ull * all_at.size());
    g.edge_t_stride = (uint32_t)et[0].size();
    g.adj_t_stride = (uint32_t)at[0].size();
  }
  g.edge_head = (const short2*)upv(head.data(), sizeof(short2) * head.size());
  g.adj_e = (const uint2*)upv(adje.data(), sizeof(uint2) * adje.size());
  g.erec = (const uint4*)upv(erec.data(), sizeof(uint4) * erec.size());
  g.erec_t = (const uint32_t*)upv(erec_t.data(), 4ull * erec_t.size());
  g.erec_stride = es;
  g.cell_rec = (const uint4*)upv(crec.data(), sizeof(uint4) * crec.size());
  if (!alloc_ok) {
    if (err) *err = "device allocation for the graph failed";
    return OTR_DEVICE_ERROR;  // the previous graph (if any) stays configured
  }
  g.n_nodes = h.n_nodes;
  g.n_edges = h.n_edges;
  g.n_segments = h.n_segments;
  g.grid_rows = h.grid_rows;
  g.grid_cols = h.grid_cols;
  g.grid_min_lat = h.grid_min_lat;
  g.grid_min_lon = h.grid_min_lon;
  g.grid_cell_deg = h.grid_cell_deg;
  std::vector<unsigned long long> sid((const unsigned long long*)(base + h.array_offset[OTR_A_SEG_ID]),
                                      (const unsigned long long*)(base + h.array_offset[OTR_A_SEG_ID]) + h.n_segments);
  // ---- swap in: batches in flight hold the shared lock, so the old arrays are unused
  GraphState& gs = graph_state();
  std::vector<void*> old;
  {
    std::unique_lock<std::shared_mutex> lk(gs.mu);
    old.swap(gs.allocs);
    gs.allocs = sg.allocs;
    sg.adopted = true;
    gs.dg = g;
    gs.n_nodes = h.n_nodes;
    gs.n_edges = h.n_edges;
    gs.n_segments = h.n_segments;
    gs.seg_id.swap(sid);
    gs.defaults = cfg.mp;
    gs.device = cfg.device;
    gs.ready = true;
  }
  for (void* q : old) (void)hipFree(q);
  return OTR_OK;
}

// ---------------------------------------------------------------------------------
// workspace slots
// ---------------------------------------------------------------------------------

enum Slot {
  S_TRACE_OFF, S_LAT, S_LON, S_TIME, S_ACC, S_MODE,
  S_STATE_CNT, S_TRACE_STATE_OFF, S_STATE_PROBE, S_STATE_TRACE,
  S_CAND_EDGE, S_CAND_P, S_CAND_SQD, S_CAND_COUNT, S_CAND_RADIUS,
  S_PREV, S_G, S_BOUND, S_FORCED, S_NTASK, S_NTRANS, S_TASK_OFF, S_TRANS_OFF, S_NTASK4, S_TASK4_OFF, S_NTASK8, S_TASK8_OFF, S_UNIT,
  S_TASK_STATE, S_TASK_MASK, S_TASK_OVF, S_TRANS,
  S_BP, S_BRK, S_END_WIN, S_WINNER, S_SUBPATH,
  S_PATH_OFF, S_PATH_LEN, S_PATH, S_STEP_OVF,
  S_CAP, S_CAP_OFF, S_POS, S_ACT, S_ENT, S_SUBA, S_SUBB, S_POR_E, S_POR_S0, S_POR_S1, S_POR_SA, S_GSTART,
  S_ROUTE, S_ROUTE_N, S_SEG_ID, S_SEG_START, S_SEG_END, S_SEG_LEN, S_SEG_QUEUE, S_SEG_INTERNAL,
  S_SEG_BSHAPE, S_SEG_ESHAPE, S_SEG_INDEX, S_SEG_N, S_SEG_WAY_N, S_SEG_WAY, S_WAY_N,
  S_REP_ID, S_REP_NEXT, S_REP_T0, S_REP_T1, S_REP_LEN, S_REP_QUEUE, S_REP_SEG, S_REP_N,
  S_SHAPE_USED, S_STATS, S_STATS_LEN, S_HIST, S_COUNTERS, S_SCAN_TMP, S_LIST, S_MISC,
  S_HEUR, S_CPREP, S_ROW_CNT, S_ROW_OFF, S_ROWS, S_ROWS_IN, S_ROWS_OUT, S_ROWS_KEPT, S_IDX_A, S_IDX_B, S_KEY_A, S_KEY_B, S_POS_SCAN, S_RUN_KEEP, S_KEEP, S_FILE_HEAD, S_FILE_START, S_NFILES, S_SORT_TMP,
  S_C_ROUTE_OFF, S_C_SEG_OFF, S_C_WAY_OFF, S_C_REP_OFF, S_C_ARGS, S_C_ROUTE, S_C_SEG_ID, S_C_SEG_START,
  S_C_SEG_END, S_C_SEG_LEN, S_C_SEG_QUEUE, S_C_SEG_INTERNAL, S_C_SEG_BSHAPE, S_C_SEG_ESHAPE, S_C_SEG_WAY_N,
  S_C_SEG_WAY, S_C_SEG_WAY_OFF, S_C_REP_ID, S_C_REP_NEXT, S_C_REP_T0, S_C_REP_T1, S_C_REP_LEN, S_C_REP_QUEUE,
  S_TASK_REC, S_BT, S_CPREP_T, S_TRANS_TC, S_TURN, S_LIST2, S_GFLAG, S_HE_IN, S_HE_SORTED, S_HE_RED, S_HE_OUT, S_HE_RANGE, S_IN_TEXT, S_IN_CNT, S_IN_CSCAN, S_IN_NL, S_IN_HASH, S_IN_UOFF, S_IN_ULEN, S_IN_TIME, S_IN_LAT, S_IN_LON,
  S_IN_ACC, S_IN_KEEP, S_IN_KPOS, S_IN_KIDX, S_IN_KEY_A, S_IN_KEY_B, S_IN_VAL_A, S_IN_VAL_B, S_IN_HEAD, S_IN_GID,
  S_IN_GFIRST, S_IN_GKEY, S_IN_WS, S_IN_KLEN, S_IN_KFLAG, S_IN_POFF, S_IN_TPOS, S_IN_BAD, S_IN_TMP,
  S_IN_T_OFF, S_IN_T_LAT, S_IN_T_LON, S_IN_T_TIME, S_IN_T_ACC, S_IN_T_MODE, S_IN_T_UOFF, S_IN_T_ULEN,
  S_CLEN, S_CAND_NROOT, S_FLAGGED, S_HE_FIDX, S_HE_FHEAD, S_HE_PFILE, S_HE_FFIRST, S_HE_PKEY, S_QUEUE, S_PQUEUE,
  S_E1DUMP0, S_E1DUMP1, S_TASK_DUMP, S_NDUMP0, S_NDUMP1, S_SORT_LIST, S_SORT_HIST,
  S_NUM
};

// A device buffer that cannot be allocated ends the call: need() throws, the entry
// points (run, tiles_cull, hist_reduce, ingest) catch it after draining the stream and
// return OTR_DEVICE_ERROR naming the buffer — no kernel ever runs on a missing buffer.
struct DeviceOom {
  int slot;
  size_t bytes;
};

static bool optional_slot(int s) {
  return s == S_E1DUMP0 || s == S_E1DUMP1 || s == S_TASK_DUMP || s == S_NDUMP0 || s == S_NDUMP1 ||
         s == S_SORT_LIST || s == S_SORT_HIST;
}

template <class T>
T* Matcher::need(int slot, size_t n) {
  if ((int)bufs.size() < S_NUM) bufs.resize(S_NUM);
  DevBuf& b = bufs[slot];
  size_t bytes = (n ? n : 1) * sizeof(T);
  if (b.bytes < bytes) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t nb = bytes + bytes / 4;
    bool ok = hipMalloc(&b.p, nb) == hipSuccess || hipMalloc(&b.p, bytes) == hipSuccess;
    if (!ok && !optional_slot(slot) && release_optional()) {
      (void)hipGetLastError();  // the optional workspace is gone: once more
      nb = bytes;
      ok = hipMalloc(&b.p, bytes) == hipSuccess;
    }
    if (!ok) {
      (void)hipGetLastError();  // clear the sticky allocation error
      b.p = nullptr;
      throw DeviceOom{slot, bytes};
    }
    b.bytes = b.p ? nb : 0;
  }
  return (T*)b.p;
}

// the free device memory an optional buffer must leave (OTR_OPT_RESERVE_GB, default 8 GB or
// an eighth of the device, whichever is more): the later stages' mandatory buffers
static size_t opt_reserve() {
  static const double gb = getenv("OTR_OPT_RESERVE_GB") ? atof(getenv("OTR_OPT_RESERVE_GB")) : -1.0;
  if (gb >= 0) return (size_t)std::min(gb * (double)(1ll << 30), 1e18);
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  return std::max<size_t>(8ull << 30, tot / 8);
}

template <class T>
T* Matcher::want(int slot, size_t n) {
  if ((int)bufs.size() < S_NUM) bufs.resize(S_NUM);
  DevBuf& b = bufs[slot];
  const size_t bytes = (n ? n : 1) * sizeof(T);
  if (b.bytes >= bytes) return (T*)b.p;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < bytes || fr - bytes < opt_reserve()) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (hipMalloc(&b.p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    b.p = nullptr;
    return nullptr;
  }
  b.bytes = bytes;
  return (T*)b.p;
}

bool Matcher::release_optional() {
  if (opt_busy) return false;
  bool any = false;
  for (int s = 0; s < (int)bufs.size(); ++s)
    if (optional_slot(s) && bufs[s].p) {
      if (!any && stream) (void)hipStreamSynchronize(stream);  // (no queued kernel still reads it)
      any = true;
      (void)hipFree(bufs[s].p);
      bufs[s].p = nullptr;
      bufs[s].bytes = 0;
    }
  return any;
}

static int oom_error(hipStream_t stream, const DeviceOom& o, std::string* err) {
  if (stream) (void)hipStreamSynchronize(stream);  // nothing of this call still running
  (void)hipGetLastError();
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  if (err)
    *err = "out of device memory: buffer " + std::to_string(o.slot) + " needs " + std::to_string(o.bytes >> 20) +
           " MiB (" + std::to_string(fr >> 20) + " of " + std::to_string(tot >> 20) +
           " MiB free): split the batch";
  return OTR_DEVICE_ERROR;
}

Matcher::~Matcher() {
  for (auto& b : bufs)
    if (b.p) (void)hipFree(b.p);
  for (auto& sl : gslab)
    for (void* q : {(void*)sl.key, (void*)sl.lab, (void*)sl.qmark, (void*)sl.fr, (void*)sl.touched})
      if (q) (void)hipFree(q);
  if (ev_init)
    for (auto& e : ev) (void)hipEventDestroy(e);
  if (stream) (void)hipStreamDestroy(stream);
}

// per-trace output capacity: route/segment/way/report slots
__global__ void k_capacity(int32_t n_traces, const int64_t* trace_state_off, const int32_t* cand_count,
                           const int32_t* path_len, int64_t* cap) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_traces) return;
  int64_t c = 2;
  for (int64_t s = trace_state_off[t]; s < trace_state_off[t + 1]; ++s) {
    if (cand_count[s] <= 0) continue;
    c += 3;
    if (path_len[s] > 0) c += path_len[s];
  }
  cap[t] = c;
}

__global__ void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// Append `value` to an unordered list, one global atomic per block (a single counter
// takes ~3 ns per same-address atomic: per-wave appends of ~1M items cost ~0.5 ms).
__device__ inline void block_append(bool hit, int64_t value, int64_t* list, unsigned long long* count) {
  __shared__ unsigned int s_n;
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  unsigned int my = 0;
  if (hit) my = atomicAdd(&s_n, 1u);
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_n ? atomicAdd(count, (unsigned long long)s_n) : 0ull;
  __syncthreads();
  if (hit) list[s_base + my] = value;
}

__global__ void k_collect(int64_t n, const int32_t* flag, int64_t* list, unsigned long long* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  block_append(i < n && flag[i], i, list, count);
}

// retry tiers: take the tasks whose flag is in the bit set `want` (bit f = flag value f)
// and clear their flags; tasks flagged for a later tier keep theirs.  The list length
// stays on the device: the next kernel reads it there.
__global__ void k_collect_tier(int64_t n, int32_t* flag, uint32_t want, int64_t* list, unsigned long long* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int f = i < n ? flag[i] : 0;
  const bool sel = f != 0 && ((want >> f) & 1u);
  if (sel) flag[i] = 0;
  block_append(sel, i, list, count);
}

// every task the first route tier flagged (overflow or general): the superset of what the
// later tiers collect, so their collects scan this short list instead of every task
__global__ void k_collect_flagged(int64_t n, const int32_t* flag, int64_t* list, unsigned long long* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  block_append(i < n && flag[i] != 0, i, list, count);
}

// k_collect_tier over the device-counted task list cand[0..*n_cand): a fixed grid
// strides over it (block-uniform trip count: block_append synchronises the block)
__global__ void k_collect_tier_from(const int64_t* cand, const unsigned long long* n_cand, int32_t* flag,
                                    uint32_t want, int64_t* list, unsigned long long* count) {
  const int64_t n = (int64_t)*n_cand;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const int64_t task = i < n ? cand[i] : 0;
    const int f = i < n ? flag[task] : 0;
    const bool sel = f != 0 && ((want >> f) & 1u);
    if (sel) flag[task] = 0;
    block_append(sel, task, list, count);
  }
}

// Spatial order of a retry list (the edge-state tier's 15.7M tasks at C2, deployed): a
// counting sort by the root's id >> shift (4,096 buckets; graph ids are spatially ordered,
// so a bucket is a small patch of the map).  The list tiers split their list into 8
// contiguous ranges, one per XCD (XcdQueue): sorted, each XCD's waves search one band of
// the map and its 4 MB L2 holds that band's records instead of the whole graph's.  Pass 1
// counts (LDS histogram per block, then one global add per non-empty bucket), pass 2 scans
// the 4,096 counts, pass 3 places each task (local rank by LDS atomic + the block's range
// reserved per bucket).  Order inside a bucket is arbitrary: tasks are independent.
constexpr int kSortBuckets = 4096;
__global__ __launch_bounds__(1024) void k_sort_hist(const int64_t* list, const unsigned long long* n_in,
                                                    const uint4* rec, int shift, uint32_t* hist) {
  __shared__ uint32_t h[kSortBuckets];
  const int64_t n = (int64_t)*n_in, i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((int64_t)blockIdx.x * blockDim.x >= n) return;  // (block-uniform)
  for (int b = threadIdx.x; b < kSortBuckets; b += blockDim.x) h[b] = 0;
  __syncthreads();
  if (i < n) atomicAdd(&h[min(rec[3 * list[i]].z >> shift, (uint32_t)kSortBuckets - 1u)], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < kSortBuckets; b += blockDim.x)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}
__global__ __launch_bounds__(1024) void k_sort_scan(uint32_t* hist) {  // one block: exclusive scan in place
  __shared__ uint32_t part[1024];
  constexpr int per = kSortBuckets / 1024;
  uint32_t v[per], t = 0;
  for (int q = 0; q < per; ++q) t += (v[q] = hist[threadIdx.x * per + q]);
  part[threadIdx.x] = t;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan of the block sums
    const uint32_t x = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t base = part[threadIdx.x] - t;
  for (int q = 0; q < per; ++q) {
    hist[threadIdx.x * per + q] = base;
    base += v[q];
  }
}
__global__ __launch_bounds__(1024) void k_sort_place(const int64_t* list, const unsigned long long* n_in,
                                                     const uint4* rec, int shift, uint32_t* cursor, int64_t* out) {
  __shared__ uint32_t h[kSortBuckets];
  const int64_t n = (int64_t)*n_in, i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((int64_t)blockIdx.x * blockDim.x >= n) return;
  for (int b = threadIdx.x; b < kSortBuckets; b += blockDim.x) h[b] = 0;
  __syncthreads();
  int64_t task = 0;
  uint32_t key = 0, r = 0;
  if (i < n) {
    task = list[i];
    key = min(rec[3 * task].z >> shift, (uint32_t)kSortBuckets - 1u);
    r = atomicAdd(&h[key], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kSortBuckets; b += blockDim.x)
    if (h[b]) h[b] = atomicAdd(&cursor[b], h[b]);  // this block's range of bucket b
  __syncthreads();
  if (i < n) out[h[key] + r] = task;
}

// the same over a device-counted list (steps of the path stage): entries list_in[0..*n_in)
__global__ void k_collect_tier_list(const unsigned long long* n_in, int32_t* flag, uint32_t want, int64_t* list,
                                    unsigned long long* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int f = i < (int64_t)*n_in ? flag[i] : 0;
  const bool sel = f != 0 && ((want >> f) & 1u);
  if (sel) flag[i] = 0;
  block_append(sel, i, list, count);
}

// states that need a path: a step inside a sub-path
__global__ void k_step_list(int64_t n_states, const int64_t* prev, const uint8_t* brk, const int32_t* cand_count,
                            int64_t* list, unsigned long long* count) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  block_append(s < n_states && cand_count[s] > 0 && prev[s] >= 0 && !brk[s], s, list, count);
}

// the same steps in two lists within list[0, n_states): the small-search path tier's from
// the front (count_front), the rest from the back (count_back); *n_all = n_states (the
// retry collects scan the whole index range, whose gap keeps its zero flags)
__global__ void k_step_lists(int64_t n_states, const int64_t* prev, const uint8_t* brk, const int32_t* cand_count,
                             PathClass pc, int64_t* list, unsigned long long* count_front,
                             unsigned long long* count_back, unsigned long long* n_all) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s == 0) *n_all = (unsigned long long)n_states;
  const bool hit = s < n_states && cand_count[s] > 0 && prev[s] >= 0 && !brk[s];
  bool small = false;
  if (hit) {
    const int64_t sp = prev[s];
    const int md = pc.mode[pc.state_trace[s]] < OTR_MODES ? pc.mode[pc.state_trace[s]] : 0;
    const uint32_t r = pc.trans[pc.trans_off[s] + (int64_t)pc.winner[sp] * cand_count[s] + pc.winner[s]];
    const double b = fmin(floor(pc.bound[s] * 1000.0), (double)r) * 1e-3;  // (k_paths' bound, m)
    small = !((pc.turn_modes >> md) & 1u) && pc.est4 * (float)(b * b) <= pc.small_keys;
  }
  // one atomic per wave and list
  const unsigned long long mf = __ballot(hit && small), mb = __ballot(hit && !small);
  const int lane = (int)(threadIdx.x % OTR_WAVE);
  unsigned long long bf = 0, bb = 0;
  if (lane == 0) {
    if (mf) bf = atomicAdd(count_front, (unsigned long long)__popcll(mf));
    if (mb) bb = atomicAdd(count_back, (unsigned long long)__popcll(mb));
  }
  bf = __shfl(bf, 0);
  bb = __shfl(bb, 0);
  const unsigned long long below = (1ull << lane) - 1ull;
  if (hit && small) list[bf + __popcll(mf & below)] = s;
  if (hit && !small) list[n_states - 1 - (int64_t)(bb + __popcll(mb & below))] = s;
}

// work counters: fold the kCShards shards of every (bank, kind) into one value before the
// copy-out (one block of kCShards threads per pair)
__global__ __launch_bounds__(kCShards) void k_ctr_fold(const unsigned long long* in, unsigned long long* out) {
  __shared__ unsigned long long part[kCShards / OTR_WAVE];
  unsigned long long v = in[(size_t)blockIdx.x * kCShards + threadIdx.x];
  for (int o = OTR_WAVE / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane_id() == 0) part[threadIdx.x / OTR_WAVE] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kCShards / OTR_WAVE; ++w) t += part[w];
    out[blockIdx.x] = t;
  }
}

static inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

// Retry tiers of the route search after the first (160-slot, 2 per wave) tier, as
// capacity * 10 + searches per wave.  512x2 (two 512-slot searches per wave) takes the
// long-bound overflows: C4 route 117 -> 112 ms against a 1024-slot G = 1 tier; a 2048-slot
// tier before the 4096 one (2.5x its occupancy): C4 4.57M -> 4.79M probes/s.  The last tier is always the 4096-slot one (its
// overflows are per-trace errors).  OTR_TIERS overrides the list for A/B runs, e.g.
// "256,512x2,1024,4096".
// the small-search tier's default size limit (keys of k_ntask's estimate; OTR_SMALL_KEYS)
constexpr double kSmallKeys = 24.0;
// the tiny-search tier's (eight searches per wave, at most 8 targets; OTR_TINY_KEYS)
constexpr double kTinyKeys = 12.0;
// the small-search path tier's (keys of k_step_lists' estimate; OTR_SMALL_PATH_KEYS)
constexpr double kSmallPathKeys = 16.0;

static std::vector<int> route_tiers() {
  std::vector<int> t;
  const char* env = getenv("OTR_TIERS");
  std::string spec = env ? env : "256,448x2,1024,2048";
  size_t i = 0;
  while (i < spec.size()) {
    size_t j = spec.find(',', i);
    if (j == std::string::npos) j = spec.size();
    const std::string item = spec.substr(i, j - i);
    const int cap = atoi(item.c_str());
    const int gw = item.find('x') != std::string::npos ? atoi(item.c_str() + item.find('x') + 1) : 1;
    const int code = cap * 10 + gw;
    if (code == 2561 || code == 5121 || code == 7681 || code == 10241 || code == 20481 || code == 3842 || code == 4482 ||
        code == 5122)
      t.push_back(code);
    i = j + 1;
  }
  if (t.size() > 4) t.resize(4);  // at most 5 retry tiers (otr_batch_result route_tier_*)
  t.push_back(40961);
  return t;
}

int Matcher::run(const otr_trace_batch* in, const ModeParams& mp, otr_batch_result* out, std::string* err) {
  try {
    const int rc = run_impl(in, mp, out, err);
    opt_busy = false;
    return rc;
  } catch (const DeviceOom& o) {
    opt_busy = false;
    return oom_error(stream, o, err);
  }
}

// a persistent grid (work queues or a grid stride over a device-side list) of at most
// `full` blocks, but never more than the list can hold (`units`, known on the host: tasks
// or steps): a small batch does not launch thousands of workgroups that find nothing
static unsigned pgrid(unsigned full, int64_t units) {
  const int64_t u = std::max<int64_t>(8, (units + 7) / 8 * 8);
  return (unsigned)std::min<int64_t>((int64_t)full, u);
}

int Matcher::run_impl(const otr_trace_batch* in, const ModeParams& mp, otr_batch_result* out, std::string* err) {
  GraphState& gs = graph_state();
  std::shared_lock<std::shared_mutex> graph_lock(gs.mu);  // a reconfigure waits for this batch
  if (!gs.ready) {
    if (err) *err = "otr_configure has not been called";
    return OTR_NOT_CONFIGURED;
  }
  HIPCHK(hipSetDevice(gs.device));
  if (!stream) HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  if (!ev_init) {
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    ev_init = true;
  }
  const bool timing = (in->flags & OTR_BATCH_TIMING) != 0;
  bool used[10] = {false};
  auto tb = [&](int k) {
    if (timing) (void)hipEventRecord(ev[2 * k], stream);
  };
  auto te = [&](int k) {
    if (timing) {
      (void)hipEventRecord(ev[2 * k + 1], stream);
      used[k] = true;
    }
  };
  memset(out, 0, sizeof(*out));
  const int32_t T = in->n_traces;
  out->n_traces = T;
  if (T <= 0) return OTR_OK;
  const DevGraph& g = gs.dg;
  BatchDev b{};
  b.n_traces = T;
  int64_t N = 0;
  if (in->memory == OTR_MEM_HOST) {
    N = in->trace_offsets[T];
    int64_t* d_off = need<int64_t>(S_TRACE_OFF, T + 1);
    double* d_lat = need<double>(S_LAT, N);
    double* d_lon = need<double>(S_LON, N);
    int64_t* d_time = need<int64_t>(S_TIME, N);
    uint8_t* d_mode = need<uint8_t>(S_MODE, T);
    float* d_acc = in->accuracy ? need<float>(S_ACC, N) : nullptr;
    if (!d_off || !d_lat || !d_lon || !d_time || !d_mode || (in->accuracy && !d_acc)) {
      if (err) *err = "device allocation failed";
      return OTR_DEVICE_ERROR;
    }
    HIPCHK(hipMemcpyAsync(d_off, in->trace_offsets, 8 * (T + 1), hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_lat, in->lat, 8 * N, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_lon, in->lon, 8 * N, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_time, in->time, 8 * N, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_mode, in->mode, T, hipMemcpyHostToDevice, stream));
    if (d_acc) HIPCHK(hipMemcpyAsync(d_acc, in->accuracy, 4 * N, hipMemcpyHostToDevice, stream));
    b.trace_off = d_off;
    b.lat = d_lat;
    b.lon = d_lon;
    b.time = d_time;
    b.mode = d_mode;
    b.acc = d_acc;
  } else {
    HIPCHK(hipMemcpyAsync(&N, in->trace_offsets + T, 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    b.trace_off = in->trace_offsets;
    b.lat = in->lat;
    b.lon = in->lon;
    b.time = in->time;
    b.mode = in->mode;
    b.acc = in->accuracy;
  }
  out->n_probes = N;
  // one wave per state / trace in the per-state and per-trace kernels: a dispatch counts
  // its work-items in 32 bits, so a batch holds at most kMaxBatchProbes = 2^26 - 64 probes
  // (otr_launch.h: the widest launch of such a batch, k_candidates at states = probes,
  // stays below 2^32; callers split larger inputs, the JSON service batches at 16M)
  if (N > kMaxBatchProbes || max_launch_items(N, N, 1) > kMaxDispatchItems) {
    if (err)
      *err = "batch of " + std::to_string(N) + " probes: at most " + std::to_string(kMaxBatchProbes) +
             " per otr_match_batch call";
    return OTR_BAD_REQUEST;
  }
  h_trace_status.assign(T, OTR_OK);
  // counter banks of OTR_COUNTERS kinds x kCShards: 0 the batch (and the first route
  // tier), 1 the 512-state edge tier, 2..6 the LDS retry tiers, 7 the 64-bit tier, 8..9 the
  // global-memory tiers, 10 the first edge tier, 11 the 1024-state edge tier, 12 the
  // small-search first tier, 13 the tiny-search one; folded at
  // the end into n_ctr values behind them
  constexpr int kBanks = 14;
  const size_t bank = (size_t)OTR_COUNTERS * kCShards;
  const size_t n_ctr = kBanks * (size_t)OTR_COUNTERS;
  unsigned long long* d_counters = need<unsigned long long>(S_COUNTERS, kBanks * bank + n_ctr);
  HIPCHK(hipMemsetAsync(d_counters, 0, kBanks * bank * 8, stream));
  size_t scan_bytes = 0;
  auto scan = [&](const int64_t* src, int64_t* dst_np1, int64_t n) -> int {
    // dst[0] = 0, dst[1..n] = inclusive prefix sums
    HIPCHK(hipMemsetAsync(dst_np1, 0, 8, stream));
    if (n == 0) return OTR_OK;
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb, src, dst_np1 + 1, (int)n, stream));
    void* tmp = need<char>(S_SCAN_TMP, tb > scan_bytes ? tb : scan_bytes);
    scan_bytes = scan_bytes > tb ? scan_bytes : tb;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, src, dst_np1 + 1, (int)n, stream));
    return OTR_OK;
  };
  auto read_i64 = [&](const int64_t* p, int64_t* v) -> int {
    HIPCHK(hipMemcpyAsync(v, p, 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    return OTR_OK;
  };
  int rc;
  // ---- K0: states
  int64_t* state_cnt = need<int64_t>(S_STATE_CNT, T);
  int64_t* trace_state_off = need<int64_t>(S_TRACE_STATE_OFF, T + 1);
  tb(OTR_STAGE_STATES);
  k_select_states<<<grid_for(T, 256), 256, 0, stream>>>(b, mp, state_cnt, nullptr, nullptr, nullptr);
  te(OTR_STAGE_STATES);
  if ((rc = scan(state_cnt, trace_state_off, T))) return rc;
  int64_t S = 0;
  if ((rc = read_i64(trace_state_off + T, &S))) return rc;
  out->n_states = S;
  int64_t* state_probe = need<int64_t>(S_STATE_PROBE, S);
  int32_t* state_trace = need<int32_t>(S_STATE_TRACE, S);
  k_select_states<<<grid_for(T, 256), 256, 0, stream>>>(b, mp, state_cnt, trace_state_off, state_probe,
                                                        state_trace);
  // ---- K1: candidates
  CandBuf cb;
  cb.edge = need<uint32_t>(S_CAND_EDGE, (size_t)S * OTR_KMAX);
  cb.p = need<double>(S_CAND_P, (size_t)S * OTR_KMAX);
  cb.sqd = need<double>(S_CAND_SQD, (size_t)S * OTR_KMAX);
  cb.count = need<int32_t>(S_CAND_COUNT, S);
  cb.radius = need<double>(S_CAND_RADIUS, S);
  if (!cb.edge || !cb.p || !cb.sqd || !cb.count) {
    if (err) *err = "device allocation failed (candidates)";
    return OTR_DEVICE_ERROR;
  }
  if (S > 0) {
    tb(OTR_STAGE_CANDIDATES);
    // two states per wave when no mode keeps more than 32 candidates (lane groups of 32) and
    // no search radius can exceed 100 m (windows of a few cells: C2 1.86 -> 1.72 ms, C5 16.1
    // -> 11.8 ms; C4's 200 m windows take 15.9 -> 22.1 ms with half the lanes each, so they
    // keep a wave per state).  A probe's radius is min(max_search_radius, max(search_radius,
    // accuracy)): without per-probe accuracies the mode's gps_accuracy stands for it.
    bool kc32 = true;
    for (int m = 0; m < OTR_MODES; ++m) {
      const MatchParams& q = mp.m[m];
      const double rmax = b.acc ? q.max_search_radius
                                : std::min(q.max_search_radius, std::max(q.search_radius, q.gps_accuracy));
      kc32 = kc32 && q.kmax <= 32 && rmax <= 100.0;
    }
    static const int cand_g = getenv("OTR_CAND_G") ? atoi(getenv("OTR_CAND_G")) : 2;  // A/B knob
    if (kc32 && cand_g == 2)
      k_candidates<2><<<(unsigned)grid_candidates((S + 1) / 2).blocks, 64, 0, stream>>>(g, b, mp, S, state_probe,
                                                                                       state_trace, cb, d_counters);
    else
      k_candidates<1><<<(unsigned)grid_candidates(S).blocks, 64, 0, stream>>>(g, b, mp, S, state_probe, state_trace, cb,
                                                                        d_counters);
    te(OTR_STAGE_CANDIDATES);
  }
  // ---- K_link + task map
  uint32_t turn_modes = 0;  // modes whose searches carry turn costs (edge-based, k_general)
  for (int m = 0; m < OTR_MODES; ++m)
    if (mp.m[m].turn_penalty_factor > 0.0) turn_modes |= 1u << m;
  StepBuf sb;
  sb.prev = need<int64_t>(S_PREV, S);
  sb.g = need<double>(S_G, S);
  sb.bound = need<double>(S_BOUND, S);
  sb.forced = need<uint8_t>(S_FORCED, S);
  sb.bt = need<int32_t>(S_BT, S);
  sb.ntask = need<int64_t>(S_NTASK, S);
  sb.ntrans = need<int64_t>(S_NTRANS, S);
  int64_t* task_off = need<int64_t>(S_TASK_OFF, S + 1);
  int64_t* trans_off = need<int64_t>(S_TRANS_OFF, S + 1);
  tb(OTR_STAGE_LINK);  // (K_link, the search inputs and the task records: through k_tasks)
  k_link<<<(unsigned)grid_link(T).blocks, 256, 0, stream>>>(b, mp, trace_state_off, state_probe, cb.count, sb);
  // K2b: per-state search inputs
  PrepArgs pr{};
  pr.n_states = S;
  pr.prev = sb.prev;
  pr.bound = sb.bound;
  pr.cand_count = cb.count;
  pr.cand_edge = cb.edge;
  pr.cand_p = cb.p;
  pr.state_trace = state_trace;
  pr.mode = b.mode;
  pr.cprep = need<uint4>(S_CPREP, (size_t)S * OTR_KMAX);
  pr.cprep_t = need<uint2>(S_CPREP_T, (size_t)S * OTR_KMAX);
  pr.clen = need<uint2>(S_CLEN, (size_t)S * OTR_KMAX);
  pr.nroot = need<int32_t>(S_CAND_NROOT, S);
  pr.turn_modes = turn_modes;
  if (!pr.cprep || !pr.cprep_t || !pr.clen || !pr.nroot) {
    if (err) *err = "device allocation failed (prep)";
    return OTR_DEVICE_ERROR;
  }
  // two states per wave when no mode keeps more than 32 candidates (K <= 32 lanes)
  bool k32 = true;
  for (int m = 0; m < OTR_MODES; ++m) k32 = k32 && mp.m[m].kmax <= 32;
  if (S > 0) {
    if (k32) k_prep<2><<<(unsigned)grid_per_state_waves(S, 2).blocks, 256, 0, stream>>>(g, pr);
    else k_prep<1><<<(unsigned)grid_per_state_waves(S, 1).blocks, 256, 0, stream>>>(g, pr);
  }
  // the first tier's size estimate (k_ntask, k_tasks, for route_unit): an exact search runs
  // to its bounds unless its targets resolve first, so its keys grow with the area it can
  // reach, est = c * density * reach^2, reach = min(length bound, time bound x 50 km/h
  // capped by the mode's speed).  A search whose estimate exceeds the first tier's table
  // starts in the retry tier that holds it: k_tasks flags it and the first tier passes it
  // on without loading its step.  c = 0.5 (C4's 60 s steps reach ~1.7 km and start in the
  // 1024-slot tier: C4 1.69M -> 2.47M probes/s; c = 1.7, the full-exhaustion fit of C2,
  // sent them to the 4096 tier, 1.07M; C2's 15 s steps stay in the first tier either way,
  // profiles/r03_est_*).  OTR_EST_K scales c (A/B knob; 0 = every search starts in the
  // first tier).  A step whose estimate is at most OTR_SMALL_KEYS keys (and has at most
  // 16 targets) goes to the small-search tier, four searches per wave (k_ntask).
  static const int route_g = getenv("OTR_ROUTE_G") ? atoi(getenv("OTR_ROUTE_G")) : 2;  // A/B knob
  float est_k = 0.f, est_v[OTR_MODES];
  uint32_t est_tier_keys[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  int n_est_tiers = 0;
  {
    static const double est_scale = getenv("OTR_EST_K") ? atof(getenv("OTR_EST_K")) : 1.0;
    const double mlat = g.grid_min_lat + 0.5 * g.grid_rows * g.grid_cell_deg;
    const double area = (g.grid_rows * g.grid_cell_deg * kMetersPerDeg) *
                        (g.grid_cols * g.grid_cell_deg * kMetersPerDeg * cos_deg(fmin(fabs(mlat), 89.0)));
    est_k = (float)(est_scale * 0.5 * (area > 0.0 ? (double)g.n_nodes / area : 0.0));
    for (int m = 0; m < OTR_MODES; ++m) {
      const double kph = mp.m[m].speed_kph > 0.0 && mp.m[m].speed_kph < 50.0 ? mp.m[m].speed_kph : 50.0;
      est_v[m] = (float)(kph / 3.6);
    }
    static const std::vector<int> tl = route_tiers();
    n_est_tiers = (int)std::min<size_t>(tl.size(), 8);
    for (int t = 0; t < n_est_tiers; ++t) est_tier_keys[t] = (uint32_t)((tl[t] / 10) * 7 / 8);
  }
  static const double small_keys = getenv("OTR_SMALL_KEYS") ? atof(getenv("OTR_SMALL_KEYS")) : kSmallKeys;  // A/B knob
  static const double tiny_keys = getenv("OTR_TINY_KEYS") ? atof(getenv("OTR_TINY_KEYS")) : kTinyKeys;  // A/B knob
  const bool small_tier = route_g == 2 && k32 && small_keys > 0.0 && est_k > 0.f;
  const bool tiny_tier = small_tier && tiny_keys > 0.0;
  int64_t* ntask4 = small_tier ? need<int64_t>(S_NTASK4, S) : nullptr;
  int64_t* task4_off = small_tier ? need<int64_t>(S_TASK4_OFF, S + 1) : nullptr;
  int64_t* ntask8 = tiny_tier ? need<int64_t>(S_NTASK8, S) : nullptr;
  int64_t* task8_off = tiny_tier ? need<int64_t>(S_TASK8_OFF, S + 1) : nullptr;
  if ((small_tier && (!ntask4 || !task4_off)) || (tiny_tier && (!ntask8 || !task8_off))) {
    if (err) *err = "device allocation failed (task map)";
    return OTR_DEVICE_ERROR;
  }
  // the step's task count: the distinct roots (k_prep) of the previous state's candidates
  if (S > 0) {
    SmallArgs sa{};
    sa.ntask4 = ntask4;
    sa.ntask8 = ntask8;
    sa.tiny_keys = (float)tiny_keys;
    sa.bound = sb.bound;
    sa.bt = sb.bt;
    sa.forced = sb.forced;
    sa.cand_count = cb.count;
    sa.state_trace = state_trace;
    sa.mode = b.mode;
    sa.turn_modes = turn_modes;
    sa.est_k = est_k;
    for (int m = 0; m < OTR_MODES; ++m) sa.est_v[m] = est_v[m];
    sa.small_keys = (float)small_keys;
    k_ntask<<<grid_for(S, 256), 256, 0, stream>>>(S, sb.prev, pr.nroot, sb.ntask, sa);
  }
  if ((rc = scan(sb.ntask, task_off, S))) return rc;
  if (small_tier && (rc = scan(ntask4, task4_off, S))) return rc;
  if (tiny_tier && (rc = scan(ntask8, task8_off, S))) return rc;
  if ((rc = scan(sb.ntrans, trans_off, S))) return rc;
  // NT: every task; [0, NT8) the tiny tier's, [NT8, NT8 + NT4) the small tier's
  int64_t NT = 0, NTR = 0, NT4 = 0, NT8 = 0;
  HIPCHK(hipMemcpyAsync(&NT, task_off + S, 8, hipMemcpyDeviceToHost, stream));
  if (small_tier) HIPCHK(hipMemcpyAsync(&NT4, task4_off + S, 8, hipMemcpyDeviceToHost, stream));
  if (tiny_tier) HIPCHK(hipMemcpyAsync(&NT8, task8_off + S, 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&NTR, trans_off + S, 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  NT += NT4 + NT8;
  int32_t* task_ovf = need<int32_t>(S_TASK_OVF, NT);
  uint32_t* trans = need<uint32_t>(S_TRANS, NTR);
  uint32_t* trans_tc = need<uint32_t>(S_TRANS_TC, turn_modes ? NTR : 1);  // read for turn modes only
  uint4* task_rec = need<uint4>(S_TASK_REC, 3 * (size_t)std::max<int64_t>(NT, 1));
  if (!task_ovf || !trans || !trans_tc || !task_rec) {
    if (err) *err = "device allocation failed (transitions)";
    return OTR_DEVICE_ERROR;
  }
  if (S > 0) {  // tasks and their records (K2 + K2c)
    TaskArgs ta{};
    ta.n_states = S;
    ta.prev = sb.prev;
    ta.cand_count = cb.count;
    ta.cand_edge = cb.edge;
    ta.edge_dst = g.edge_dst;
    ta.task_off = task_off;
    ta.bound = sb.bound;
    ta.forced = sb.forced;
    ta.bt = sb.bt;
    ta.state_trace = state_trace;
    ta.mode = b.mode;
    ta.cprep = pr.cprep;
    ta.cprep_t = pr.cprep_t;
    ta.trans_off = trans_off;
    ta.turn_modes = turn_modes;
    ta.rec = task_rec;
    ta.ntask4 = ntask4;
    ta.task4_off = task4_off;
    ta.nt4 = NT4;
    ta.ntask8 = ntask8;
    ta.task8_off = task8_off;
    ta.nt8 = NT8;
    ta.flag_turn = task_ovf;  // turn-mode tasks start in the first edge-state tier (flag 5)
    // the two-search first tier's table: a step expected beyond it is flagged here
    ta.est_first_keys = route_g == 2 ? (OTR_CAP1 * OTR_LOAD1) / 8 : 0;
    ta.est_k = est_k;
    for (int m = 0; m < OTR_MODES; ++m) ta.est_v[m] = est_v[m];
    ta.n_tiers = n_est_tiers;
    for (int t = 0; t < n_est_tiers; ++t) ta.tier_keys[t] = est_tier_keys[t];
    if (NT > 0) HIPCHK(hipMemsetAsync(task_ovf, 0, 4 * NT, stream));
    if (k32) k_tasks<2><<<(unsigned)grid_per_state_waves(S, 2).blocks, 256, 0, stream>>>(ta);
    else k_tasks<1><<<(unsigned)grid_per_state_waves(S, 1).blocks, 256, 0, stream>>>(ta);
  }
  te(OTR_STAGE_LINK);
  // turn cost tables of this batch's parameters (oracle orc_turn_table)
  int32_t* d_turn = need<int32_t>(S_TURN, 181 * OTR_MODES);
  h_turn.resize(181 * OTR_MODES);
  for (int m = 0; m < OTR_MODES; ++m) turn_table(mp.m[m].turn_penalty_factor, h_turn.data() + 181 * m);
  HIPCHK(hipMemcpyAsync(d_turn, h_turn.data(), 4 * 181 * OTR_MODES, hipMemcpyHostToDevice, stream));
  // ---- K3/K4: routing + transition costs
  RouteArgs ra{};
  ra.task_list = nullptr;
  ra.n_tasks = NT;
  ra.prev = sb.prev;
  ra.g = sb.g;
  ra.bound = sb.bound;
  ra.forced = sb.forced;
  ra.trans_off = trans_off;
  ra.trans = trans;
  ra.cand_count = cb.count;
  ra.cand_edge = cb.edge;
  ra.cand_p = cb.p;
  ra.state_trace = state_trace;
  ra.mode = b.mode;
  ra.bt = sb.bt;
  ra.turn = d_turn;
  ra.trans_tc = trans_tc;
  ra.cprep = pr.cprep;
  ra.cprep_t = pr.cprep_t;
  ra.clen = pr.clen;
  ra.rec = task_rec;
  for (int m = 0; m < OTR_MODES; ++m) ra.inv_beta[m] = mp.m[m].inv_beta;
  ra.overflow_flag = task_ovf;
  ra.stamps = d_counters;
  ra.est_k = est_k;
  for (int m = 0; m < OTR_MODES; ++m) ra.est_v[m] = est_v[m];
  ra.n_tiers = n_est_tiers;
  for (int t = 0; t < n_est_tiers; ++t) ra.tier_keys[t] = est_tier_keys[t];
  // device-side counters of the retry lists: [0..7] route tiers, [8] general tier 1,
  // [9] general tier 2, [10] route tasks left unrouted, [11] steps, [12..15] path tiers,
  // [16] path general 1, [17] path general 2, [18] paths left, [19] general overflow
  // count, [20] cap flag, [21] exact node path tier, [23] first edge-state tier, [24] tasks
  // the first route tier
  // flagged, [25..26] edge-state route tiers, [27..28] edge-state path tiers, [29] exact
  // edge route tier, [30] exact node route tier, [31] exact edge path tier, [32..96) path
  // bump cursors
  unsigned long long* cnt = need<unsigned long long>(S_MISC, 32 + kShards);
  HIPCHK(hipMemsetAsync(cnt, 0, 8 * (32 + kShards), stream));
  int64_t* list = need<int64_t>(S_LIST, std::max<int64_t>(NT, S));
  int64_t* fail_tasks = need<int64_t>(S_GFLAG, std::max<int64_t>(NT, 1));
  int64_t* flagged = need<int64_t>(S_FLAGGED, std::max<int64_t>(NT, 1));
  if (!list || !fail_tasks || !flagged) {
    if (err) *err = "device allocation failed (retry lists)";
    return OTR_DEVICE_ERROR;
  }
  // general (global-memory) search slabs: allocated on first use, cleared once
  auto slabs = [&](int tier, GSlabs* out) -> int {
    GSlab& sl = gslab[tier];
    const uint32_t cap = tier == 0 ? (1u << 15) : (1u << 20);
    const uint32_t n = tier == 0 ? 1024u : 8u;
    if (!sl.key) {
      // all five arrays or none: a partial set is freed and the batch fails with
      // OTR_DEVICE_ERROR (a later batch never sees a half-allocated slab)
      const size_t c = (size_t)cap * n;
      void* p[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
      const size_t bytes[5] = {4 * c, 8 * c, 4 * c, 8 * c, 4 * c};
      bool good = true;
      for (int attempt = 0; attempt < 2; ++attempt) {
        good = true;
        for (int q = 0; q < 5 && good; ++q) good = hipMalloc(&p[q], bytes[q]) == hipSuccess;
        if (good) break;
        (void)hipGetLastError();
        for (void*& q : p)
          if (q) (void)hipFree(q), q = nullptr;
        if (attempt > 0 || !release_optional()) break;  // (the optional workspace gone: once more)
      }
      if (good)
        good = hipMemsetAsync(p[0], 0xFF, 4 * c, stream) == hipSuccess &&
               hipMemsetAsync(p[1], 0xFF, 8 * c, stream) == hipSuccess &&
               hipMemsetAsync(p[2], 0, 4 * c, stream) == hipSuccess;
      if (!good) {
        (void)hipGetLastError();
        for (void* q : p)
          if (q) (void)hipFree(q);
        throw DeviceOom{S_NUM + tier, 28 * c};  // (the global-search slabs of this tier)
      }
      sl.key = (uint32_t*)p[0];
      sl.lab = (unsigned long long*)p[1];
      sl.qmark = (uint32_t*)p[2];
      sl.fr = (uint32_t*)p[3];
      sl.touched = (uint32_t*)p[4];
    }
    out->key = sl.key;
    out->lab = sl.lab;
    out->qmark = sl.qmark;
    out->fr = sl.fr;
    out->touched = sl.touched;
    out->cap = cap;
    out->n = n;
    return OTR_OK;
  };
  GenArgs ga{};
  ga.prev = sb.prev;
  ga.g = sb.g;
  ga.bt = sb.bt;
  ga.bound = sb.bound;
  ga.cand_count = cb.count;
  ga.cand_edge = cb.edge;
  ga.cand_p = cb.p;
  ga.cprep = pr.cprep;
  ga.cprep_t = pr.cprep_t;
  ga.state_trace = state_trace;
  ga.mode_of_trace = b.mode;
  ga.turn_modes = turn_modes;
  ga.turn = d_turn;
  ga.rec = task_rec;
  ga.trans_off = trans_off;
  ga.trans = trans;
  ga.trans_tc = trans_tc;
  ga.counters = d_counters;
  ga.n_overflow = cnt + 19;
  if (NT > 0) {
    // two searches per wave (CAP 160 tables); wider steps and overflows retry below
    // the LDS tiers count their work only when asked (OTR_BATCH_ROUTE_WORK): the end-of-
    // wave counter atomics cost ~7% of the first tier (tools/ab_libs.sh)
    unsigned long long* rwork = (in->flags & OTR_BATCH_ROUTE_WORK) ? d_counters : nullptr;
    // the LDS route kernels: with the work counters (CNT) only when counting was asked for
#define OTR_ROUTE_LAUNCH(C, G_, LIST_, GRID, ARGS, CTR)                                       \
  do {                                                                                      \
    if (CTR) k_route<C, G_, LIST_, false, true><<<GRID, 64, 0, stream>>>(g, ARGS, CTR);      \
    else k_route<C, G_, LIST_, false, false><<<GRID, 64, 0, stream>>>(g, ARGS, nullptr);     \
  } while (0)
    // turn-mode (edge-state) tasks belong to the edge-state tiers below: the node
    // tiers pass them on unflagged, and when every mode has turn costs (the deployed
    // configuration) no node task exists and the first node tier is not launched at all
    const bool turns = turn_modes != 0u;
#ifdef OTR_FORCE_GENERAL
    const bool node_tasks = true;  // (test build: the first tier flags every task for k_general)
#else
    const bool node_tasks = turn_modes != (1u << OTR_MODES) - 1u;
#endif
#ifdef OTR_FORCE_RETRY
    {  // test build: OTR_FORCE_EDGE bits force the edge-state tiers to fail (tests/test_gpu_tiers.py)
      const char* fe = getenv("OTR_FORCE_EDGE");
      ra.force_edge = fe ? atoi(fe) : 0;
    }
#endif
    // the list tiers' work queues (XcdQueue): 8 counters per launch, 128 B apart
    constexpr int kQueueWords = 16 * 8;
    unsigned long long* queues = need<unsigned long long>(S_QUEUE, 16 * kQueueWords);
    HIPCHK(hipMemsetAsync(queues, 0, 8 * 16 * kQueueWords, stream));
    // retry-tier dumps (search_run NDump, otr_edge1.h): per task, the dump slot its search
    // left for the next tier; every tier that fails a task writes it (-1: restart), so the
    // first node tier, which flags every task a retry tier will see, initialises it
    static const bool nresume = !getenv("OTR_NRESUME") || atoi(getenv("OTR_NRESUME")) != 0;  // A/B knob
    static const bool eresume = !getenv("OTR_E1RESUME") || atoi(getenv("OTR_E1RESUME")) != 0;  // A/B knob
    int32_t* task_dump = nullptr;  // (optional: without it outgrown searches restart, same results)
    if ((nresume && node_tasks) || (eresume && turns)) task_dump = want<int32_t>(S_TASK_DUMP, NT);
    opt_busy = true;  // the optional workspace stays until the route stage's kernels are queued
    ra.task_dump = task_dump;
    tb(OTR_STAGE_ROUTE);
    if (node_tasks) {
      // one unit (G searches) per block, in launches of at most 2^25 blocks: a dispatch's
      // grid size counts work-items in 32 bits (178M tasks at 12.5M probes would wrap).
      // The small tier (four searches per wave, tasks [0, NT4)) first, then the two-search
      // tier over the rest
      constexpr int64_t kMaxUnits = 1ll << 25;
      // the tiny tier (eight searches per wave, tasks [0, NT8)) only in batches that are
      // mostly tiny steps (C5); elsewhere its few tasks join the small tier's range (they are
      // adjacent), which saves a launch (C1: 18k tiny tasks cost 2 %)
      const bool tiny_run = NT8 > 0 && (2 * NT8 >= NT || tiny_keys >= 1e8);  // (1e8: tests force it)
      const int64_t small_lo = tiny_run ? NT8 : 0;
      if (tiny_run) {
        unsigned long long* rc8 = rwork ? d_counters + 13 * bank : nullptr;
        if (timing) (void)hipEventRecord(ev[24 + 2 * 13], stream);
        const int64_t units = (NT8 + 7) / 8;
        for (int64_t base = 0; base < units; base += kMaxUnits) {
          RouteArgs rf = ra;
          rf.n_tasks = NT8;
          rf.unit_base = base;
          const int64_t u = std::min<int64_t>(kMaxUnits, units - base);
          OTR_ROUTE_LAUNCH(OTR_CAP8, 8, false, (unsigned)(8 * ((u + 7) / 8)), rf, rc8);
        }
        if (timing) (void)hipEventRecord(ev[24 + 2 * 13 + 1], stream);
        out->route_tier_code[13] = OTR_CAP8 * 10 + 8;
      }
      if (NT8 + NT4 - small_lo > 0) {
        unsigned long long* rc4 = rwork ? d_counters + 12 * bank : nullptr;
        if (timing) (void)hipEventRecord(ev[24 + 2 * 12], stream);
        const int64_t units = (NT8 + NT4 - small_lo + 3) / 4;
        // (a block per unit: a persistent grid over per-XCD queues was slower, C5 26.5 ->
        // 35.6 ms)
        for (int64_t base = 0; base < units; base += kMaxUnits) {
          RouteArgs rf = ra;
          rf.n_tasks = NT8 + NT4;
          rf.task_base = small_lo;
          rf.unit_base = base;
          const int64_t u = std::min<int64_t>(kMaxUnits, units - base);
          OTR_ROUTE_LAUNCH(OTR_CAP4, 4, false, (unsigned)(8 * ((u + 7) / 8)), rf, rc4);
        }
        if (timing) (void)hipEventRecord(ev[24 + 2 * 12 + 1], stream);
        out->route_tier_code[12] = OTR_CAP4 * 10 + 4;
      }
      const int64_t units = route_g == 2 ? (NT - NT8 - NT4 + 1) / 2 : NT;
      for (int64_t base = 0; base < units; base += kMaxUnits) {
        RouteArgs rf = ra;
        rf.unit_base = base;
        rf.task_base = NT8 + NT4;
        const int64_t u = std::min<int64_t>(kMaxUnits, units - base);
        const unsigned grid = (unsigned)(8 * ((u + 7) / 8));
        if (route_g == 2) OTR_ROUTE_LAUNCH(OTR_CAP1, 2, false, grid, rf, rwork);
        else OTR_ROUTE_LAUNCH(256, 1, false, grid, rf, rwork);
      }
      out->route_tier_code[0] = route_g == 2 ? OTR_CAP1 * 10 + 2 : 2561;
    }
    te(OTR_STAGE_ROUTE);
    // overflow retries with larger LDS tables (same results, fewer resident waves): each
    // tier takes its list on the device and runs a fixed grid over it — no host round
    // trip between tiers.  Tier t takes the previous tier's overflows (flag 1) and the
    // first-tier tasks whose size estimate starts them in a tier <= t (flags 16 + u, u <= t);
    // OTR_TIERS (A/B knob) lists the retry kernels.
    tb(OTR_STAGE_ROUTE_BIG);
    static const std::vector<int> tiers = route_tiers();
    const int ntier = (int)tiers.size();
    // persistent grids over per-XCD queues: about twice a tier's resident waves (256 CUs x
    // 4 SIMDs x 8 waves for the small tables, fewer for the big ones, whose LDS admits
    // fewer); a block that finds its queue drained exits at once
    // the first tier's flagged tasks, once; every later collect scans only them
    k_collect_flagged<<<grid_for(NT, 1024), 1024, 0, stream>>>(NT, task_ovf, flagged, cnt + 24);
    constexpr unsigned kCollectGrid = 512;
    // node dump slots: tier t writes buffer t % 2 and tier t + 1 resumes from it; slots for a
    // quarter of the tasks, at most OTR_NDUMP_GB (4) GB per buffer (C4: 4 % of the 1024-slot
    // searches outgrow it, 10 KB each); beyond them, or without the memory, searches restart
    unsigned long long* ndump[2] = {nullptr, nullptr};
    uint32_t nslots[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    // (tables compiled with the resume / dump code, otr_kernels.h OTR_ND_IN_MIN / OTR_ND_OUT_MIN)
    auto nd_in = [&](int t) { return t > 0 && t < ntier && tiers[t] / 10 >= OTR_ND_IN_MIN; };
    auto nd_out = [&](int t) { return t + 1 < ntier && tiers[t] / 10 >= OTR_ND_OUT_MIN && nd_in(t + 1); };
    if (nresume && node_tasks && task_dump && ntier > 1) {
      static const double gb = getenv("OTR_NDUMP_GB") ? atof(getenv("OTR_NDUMP_GB")) : 4.0;
      const int64_t cap_bytes = (int64_t)(gb * (double)(1ll << 30));
      size_t words[2] = {0, 0};
      for (int t = 0; t + 1 < ntier && t < 8; ++t) {
        if (!nd_out(t)) continue;
        const uint32_t w = nd_words(tiers[t] / 10);
        nslots[t] = (uint32_t)std::min<int64_t>(std::max<int64_t>(NT / 4, 1024), cap_bytes / (8 * (int64_t)w));
        words[t & 1] = std::max<size_t>(words[t & 1], (size_t)nslots[t] * w);
      }
      for (int q = 0; q < 2; ++q)
        if (words[q]) ndump[q] = want<unsigned long long>(q == 0 ? S_NDUMP0 : S_NDUMP1, words[q]);
      if ((words[0] && !ndump[0]) || (words[1] && !ndump[1])) ndump[0] = ndump[1] = nullptr;
    }
    for (int tier = 0; tier < (node_tasks ? ntier : 0); ++tier) {  // (no node task: no node tier)
      unsigned long long* c = cnt + tier;
      k_collect_tier_from<<<kCollectGrid, 1024, 0, stream>>>(flagged, cnt + 24, task_ovf,
                                                            0x2u | (((2u << tier) - 1u) << 16), list + 0, c);
      RouteArgs rb = ra;
      rb.task_list = list;
      rb.list_count = c;
      rb.queue = queues + tier * kQueueWords;
      const bool din = nd_in(tier) && nd_out(tier - 1) && ndump[(tier + 1) & 1] != nullptr;
      const bool dout = nd_out(tier) && ndump[tier & 1] != nullptr;
      rb.dump_in = din ? ndump[(tier + 1) & 1] : nullptr;
      rb.dump_in_words = din ? nd_words(tiers[tier - 1] / 10) : 0u;
      rb.dump_out = dout ? ndump[tier & 1] : nullptr;
      rb.dump_ctr = queues + 15 * kQueueWords + 16 * tier;  // (queue 15: zeroed above; one line per tier)
      rb.dump_out_words = dout ? nd_words(tiers[tier] / 10) : 0u;
      rb.dump_out_slots = dout ? nslots[tier] : 0u;
      unsigned long long* rcn = rwork ? d_counters + (2 + tier) * bank : nullptr;
      out->route_tier_code[1 + tier] = tiers[tier];
      if (timing) (void)hipEventRecord(ev[24 + 2 * (1 + tier)], stream);
#define OTR_TIER(C, G_) \
  OTR_ROUTE_LAUNCH(C, G_, true, pgrid((C) <= 512 ? 16384u : 16384u * 512u / (C), (NT + (G_) - 1) / (G_)), rb, rcn)
      switch (tiers[tier]) {
        case 2561: OTR_TIER(256, 1); break;
        case 5121: OTR_TIER(512, 1); break;
        case 7681: OTR_TIER(768, 1); break;
        case 10241: OTR_TIER(1024, 1); break;
        case 20481: OTR_TIER(2048, 1); break;
        case 3842: OTR_TIER(384, 2); break;
        case 4482: OTR_TIER(448, 2); break;
        case 5122: OTR_TIER(512, 2); break;
        default: OTR_TIER(4096, 1); break;
      }
#undef OTR_TIER
      if (timing) (void)hipEventRecord(ev[24 + 2 * (1 + tier) + 1], stream);
    }
#ifndef OTR_FORCE_GENERAL  // (test build: every search in k_general)
    // the node-mode tasks whose (length << sh | time) words need more than 32 bits
    // (flag 3: long gaps between states) run in an LDS table of 64-bit words (same labels,
    // DESIGN.md §3.5); what outgrows it is flagged 3 again
    {
      unsigned long long* c = cnt + 7;
      k_collect_tier_from<<<kCollectGrid, 1024, 0, stream>>>(flagged, cnt + 24, task_ovf, 0x8u, list, c);
      RouteArgs rb = ra;
      rb.task_list = list;
      rb.list_count = c;
      rb.queue = queues + 8 * kQueueWords;
      out->route_tier_code[8] = 900000 + 2048;
      if (timing) (void)hipEventRecord(ev[24 + 2 * 8], stream);
      if (rwork) k_route<2048, 1, true, true, true><<<pgrid(4096, NT), 64, 0, stream>>>(g, rb, d_counters + 7 * bank);
      else k_route<2048, 1, true, true, false><<<pgrid(4096, NT), 64, 0, stream>>>(g, rb, nullptr);
      if (timing) (void)hipEventRecord(ev[24 + 2 * 8 + 1], stream);
    }
#endif
    // edge-state tiers (turn-cost modes, otr_edge1.h): OTR_E1CAP (360) states (flag 5, slot
    // 10), 512 (flag 6, slot 9), 1024 (flag 7, slot 11); what outgrows those (flag 3) goes on below
    if (turns) {
      // dump slots of the first two edge tiers: a search they outgrow between two rounds
      // resumes in the next table (otr_edge1.h e1_dump / e1_restore) instead of starting
      // over; slots for 1/16 of the tasks (C2, deployed: 4.4 % outgrow the first table),
      // at most 4 GB / 1 GB — searches beyond them, or when the memory is not there,
      // restart in the next table (same results)
      unsigned long long* dump[2] = {nullptr, nullptr};
      uint32_t dslots[2] = {0u, 0u};
      const uint32_t dwords[2] = {e1_dump_words(OTR_E1CAP), e1_dump_words(512)};
      if (eresume && task_dump) {
        const int64_t cap_bytes[2] = {4ll << 30, 1ll << 30};
        const int64_t wanted[2] = {std::max<int64_t>(NT / 16, 4096), std::max<int64_t>(NT / 64, 1024)};
        for (int q = 0; q < 2; ++q) {  // (no dumps beyond what was allocated: those searches restart)
          const int64_t n = std::min<int64_t>(wanted[q], cap_bytes[q] / (8 * (int64_t)dwords[q]));
          dump[q] = want<unsigned long long>(q == 0 ? S_E1DUMP0 : S_E1DUMP1, (size_t)n * dwords[q]);
          dslots[q] = dump[q] ? (uint32_t)n : 0u;
        }
        if (!dump[0]) dump[1] = nullptr, dslots[1] = 0u;
      }
      for (int et = 0; et < 3; ++et) {
        const int slot = et == 0 ? 10 : (et == 1 ? 9 : 11);
        out->route_tier_code[slot] = 6000000 + (et == 0 ? OTR_E1CAP : (et == 1 ? 512 : 1024)) * 100 + 32;
        unsigned long long* c = cnt + (et == 0 ? 23 : 24 + et);
        k_collect_tier_from<<<kCollectGrid, 1024, 0, stream>>>(flagged, cnt + 24, task_ovf, 0x20u << et, list, c);
        RouteArgs rb = ra;
        rb.task_list = list;
        // the first edge tier's list in spatial order (k_sort_*: one band of the map per XCD)
        static const bool esort = !getenv("OTR_SORT") || atoi(getenv("OTR_SORT")) != 0;  // A/B knob
        int64_t* list2 = nullptr;
        uint32_t* hist = nullptr;
        if (et == 0 && esort && NT >= 65536) {
          list2 = want<int64_t>(S_SORT_LIST, NT);  // (no memory for the copy: the list stays in task order)
          hist = list2 ? want<uint32_t>(S_SORT_HIST, kSortBuckets) : nullptr;
        }
        if (list2 && hist) {
          int bits = 0;
          while (bits < 32 && (g.n_edges >> bits) > 0u) ++bits;
          const int shift = bits > 12 ? bits - 12 : 0;
          HIPCHK(hipMemsetAsync(hist, 0, 4 * kSortBuckets, stream));
          k_sort_hist<<<grid_for(NT, 1024), 1024, 0, stream>>>(list, c, task_rec, shift, hist);
          k_sort_scan<<<1, 1024, 0, stream>>>(hist);
          k_sort_place<<<grid_for(NT, 1024), 1024, 0, stream>>>(list, c, task_rec, shift, hist, list2);
          rb.task_list = list2;
        }
        rb.list_count = c;
        rb.queue = queues + (9 + et) * kQueueWords;
        rb.dump_in = et > 0 ? dump[et - 1] : nullptr;
        rb.dump_in_words = et > 0 ? dwords[et - 1] : 0u;
        rb.dump_in_cap = et == 1 ? OTR_E1CAP : 512;
        rb.dump_out = et < 2 ? dump[et] : nullptr;
        rb.dump_ctr = queues + (13 + et) * kQueueWords;  // (queues 13, 14: zeroed above)
        rb.dump_out_words = et < 2 ? dwords[et] : 0u;
        rb.dump_out_slots = et < 2 ? dslots[et] : 0u;
        rb.task_dump = task_dump;
        unsigned long long* rcn = rwork ? d_counters + (et == 0 ? 10 : (et == 1 ? 1 : 11)) * bank : nullptr;
        if (timing) (void)hipEventRecord(ev[24 + 2 * slot], stream);
        // persistent grids of at least every resident wave (16 per CU at 384 states, 13 at
        // 512, 6 at 1024) claiming tasks from per-XCD queues; steps with more than 32
        // targets (modes keeping > 32 candidates) pass the lean tiers (their TG = 32) on to
        // k_general
        if (et == 0) k_route_e1<OTR_E1CAP><<<pgrid(8192, NT), 64, 0, stream>>>(g, rb, rcn);
        else if (et == 1) k_route_e1<512><<<pgrid(4096, NT), 64, 0, stream>>>(g, rb, rcn);
        else k_route_e1<1024><<<pgrid(2048, NT), 64, 0, stream>>>(g, rb, rcn);
        if (timing) (void)hipEventRecord(ev[24 + 2 * slot + 1], stream);
      }
    }
    opt_busy = false;  // (every user of the optional workspace is queued)
    // everything left — tasks whose labels need 64 bits, overflows of the largest LDS
    // tables (node and edge-state) — runs in the global-memory search: first on 32K-slot
    // slabs, then what outgrew those on 1M-slot slabs
    for (int gt = 0; gt < 2; ++gt) {
      unsigned long long* c = cnt + 8 + gt;
      k_collect_tier_from<<<kCollectGrid, 1024, 0, stream>>>(flagged, cnt + 24, task_ovf, gt == 0 ? 0x1Eu : 0x2u, list,
                                                            c);
      GSlabs gs2;
      if ((rc = slabs(gt, &gs2))) return rc;
      ga.mode = 0;
      ga.list = list;
      ga.list_count = c;
      ga.flag = task_ovf;
      ga.counters = d_counters + (8 + gt) * bank;
      out->route_tier_code[6 + gt] = -1 - gt;
      if (timing) (void)hipEventRecord(ev[24 + 2 * (6 + gt)], stream);
      k_general<<<pgrid(gs2.n, NT), kGenThreads, 0, stream>>>(g, ga, gs2);
      if (timing) (void)hipEventRecord(ev[24 + 2 * (6 + gt) + 1], stream);
    }
    // tasks still flagged (beyond a 1M-state slab): their traces get OTR_MATCH_ERROR
    k_collect_tier_from<<<kCollectGrid, 1024, 0, stream>>>(flagged, cnt + 24, task_ovf, 0x1Eu, fail_tasks, cnt + 10);
    te(OTR_STAGE_ROUTE_BIG);
  }
  // ---- K5: Viterbi
  ViterbiArgs va{};
  va.n_traces = T;
  va.trace_state_off = trace_state_off;
  va.cand_count = cb.count;
  va.cand_sqd = cb.sqd;
  va.prev = sb.prev;
  va.trans_off = trans_off;
  va.trans = trans;
  va.trans_tc = trans_tc;
  va.turn_modes = turn_modes;
  va.g = sb.g;
  va.mode = b.mode;
  for (int m = 0; m < OTR_MODES; ++m) va.inv2s2[m] = mp.m[m].inv2s2;
  for (int m = 0; m < OTR_MODES; ++m) va.inv_beta[m] = mp.m[m].inv_beta;
  va.bp = need<int8_t>(S_BP, (size_t)S * OTR_KMAX);
  va.brk = need<uint8_t>(S_BRK, S);
  va.end_win = need<int32_t>(S_END_WIN, S);
  va.winner = need<int32_t>(S_WINNER, S);
  va.subpath = need<int32_t>(S_SUBPATH, S);
  tb(OTR_STAGE_VITERBI);
  {
    // two traces per wave when no mode keeps more than 32 candidates (K <= 32 lanes); a
    // batch too small to fill the GPU that way (fewer than 8,192 traces: C1's 1,000) runs
    // one trace per wave with each step's predecessor scan split over the two halves
    static const int64_t split_below = getenv("OTR_VIT_SPLIT") ? atoll(getenv("OTR_VIT_SPLIT")) : 8192;  // A/B knob
    if (k32 && T < split_below) {
      k_viterbi<1, true><<<(unsigned)(T < 1048576 ? T : 1048576), 64, 0, stream>>>(va, d_counters);
    } else if (k32) {
      const int64_t w = (T + 1) / 2;
      k_viterbi<2><<<(unsigned)(w < 1048576 ? w : 1048576), 64, 0, stream>>>(va, d_counters);
    } else {
      k_viterbi<1><<<(unsigned)(T < 1048576 ? T : 1048576), 64, 0, stream>>>(va, d_counters);
    }
  }
  te(OTR_STAGE_VITERBI);
  // ---- K6: winner paths (step list, tiers and general fallback counted on the device)
  int64_t* path_off = need<int64_t>(S_PATH_OFF, S);
  int32_t* path_len = need<int32_t>(S_PATH_LEN, S);
  if (S > 0) k_fill_i32<<<grid_for(S, 256), 256, 0, stream>>>(path_len, S, 0);
  {
    int64_t* steps = need<int64_t>(S_LIST2, std::max<int64_t>(S, 1));
    unsigned long long* nsteps_d = cnt + 11;
    // the small-search path tier (four searches per wave): steps whose winning route
    // bounds a search of at most OTR_SMALL_PATH_KEYS keys (estimate: 4 x the node density
    // x r^2, the diamond of road distance r around the root and its frontier); the
    // two-search tier takes the rest.  Both lists' lengths come back to the host (one
    // synchronisation) so each tier launches the blocks its list needs and no more (a grid
    // sized for every step costs a dispatch per empty block: C5 paths 13.2 -> 18.8 ms
    // instead of 8.3).  Only in batches whose route tasks went mostly to the small route
    // tier (C5, C1): at C2 (3 % small) the synchronisation cost more than the tier saved.
    static const double small_path_keys =
        getenv("OTR_SMALL_PATH_KEYS") ? atof(getenv("OTR_SMALL_PATH_KEYS")) : kSmallPathKeys;  // A/B knob
    const bool small_paths = small_path_keys > 0.0 && est_k > 0.f && (small_path_keys >= 1e8 || 2 * (NT4 + NT8) >= NT);
    unsigned long long* nsteps4_d = cnt + 21;  // (the front list's count)
    unsigned long long* nall_d = cnt + 22;     // (S: the collects' index range)
    unsigned long long h_nsteps[2] = {0ull, 0ull};  // (front, back)
    if (S > 0 && small_paths) {
      PathClass pc{};
      pc.winner = va.winner;
      pc.trans_off = trans_off;
      pc.trans = trans;
      pc.bound = sb.bound;
      pc.state_trace = state_trace;
      pc.mode = b.mode;
      pc.turn_modes = turn_modes;
      pc.est4 = 8.f * est_k;  // (est_k = half the node density)
      pc.small_keys = (float)small_path_keys;
      HIPCHK(hipMemsetAsync(nsteps4_d, 0, 16, stream));
      k_step_lists<<<grid_for(S, 256), 256, 0, stream>>>(S, sb.prev, va.brk, cb.count, pc, steps, nsteps4_d, nsteps_d,
                                                          nall_d);
      HIPCHK(hipMemcpyAsync(&h_nsteps[0], nsteps4_d, 8, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(&h_nsteps[1], nsteps_d, 8, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
    } else if (S > 0) {
      k_step_list<<<grid_for(S, 1024), 1024, 0, stream>>>(S, sb.prev, va.brk, cb.count, steps, nsteps_d);
    }
    // the retry collects' index range: every step index (front and back lists), or the list
    const unsigned long long* nscan_d = small_paths ? nall_d : nsteps_d;
    int32_t* step_ovf = need<int32_t>(S_STEP_OVF, S + 1);
    int64_t capacity = kShards * ((int64_t)S * 24 / kShards + 1024);
    bool paths_fit = S == 0;
    for (int attempt = 0; attempt < 8 && S > 0; ++attempt) {
      uint32_t* path = need<uint32_t>(S_PATH, capacity);
      if (!path || !step_ovf) {
        if (err) *err = "device allocation failed (paths)";
        return OTR_DEVICE_ERROR;
      }
      HIPCHK(hipMemsetAsync(step_ovf, 0, 4 * (S + 1), stream));
      HIPCHK(hipMemsetAsync(cnt + 12, 0, 8 * 9, stream));  // path tier counts, cap flag
      HIPCHK(hipMemsetAsync(cnt + 27, 0, 8 * 2, stream));  // edge-state path tier counts
      HIPCHK(hipMemsetAsync(cnt + 32, 0, 8 * kShards, stream));
      PathArgs pa{};
      pa.steps = steps;
      pa.n_steps = S;
      pa.n_steps_dev = nsteps_d;
      pa.prev = sb.prev;
      pa.bound = sb.bound;
      pa.brk = va.brk;
      pa.winner = va.winner;
      pa.cand_edge = cb.edge;
      pa.cand_p = cb.p;
      pa.state_trace = state_trace;
      pa.mode = b.mode;
      pa.cprep = ra.cprep;
      pa.cprep_t = ra.cprep_t;
      pa.bt = sb.bt;
      pa.turn_modes = turn_modes;
      pa.path_off = path_off;
      pa.path_len = path_len;
      pa.path = path;
      pa.cursor = cnt + 32;
      pa.capacity = capacity;
      pa.overflow_flag = step_ovf;
      pa.cap_flag = (int32_t*)(cnt + 20);
      pa.cand_count = cb.count;
      pa.trans_off = trans_off;
      pa.trans = trans;
      pa.force_edge = ra.force_edge;
      // the path retry tiers' work queues (XcdQueue)
      constexpr int kPQWords = 16 * 8;
      unsigned long long* pq = need<unsigned long long>(S_PQUEUE, 8 * kPQWords);
      HIPCHK(hipMemsetAsync(pq, 0, 8 * 8 * kPQWords, stream));
      tb(OTR_STAGE_PATHS);
      if (small_paths) {
        // the front list four searches per wave, the back list two, each grid sized by its
        // list's length (blocks past a list's end exit at once, but cost a dispatch each)
        if (h_nsteps[0] > 0) {
          PathArgs p4 = pa;
          p4.n_steps_dev = nsteps4_d;
          k_paths<OTR_CAP4, 4><<<(unsigned)grid_paths((int64_t)(h_nsteps[0] + 1) / 2).blocks, 64, 0, stream>>>(
              g, p4, nullptr, nullptr);
        }
        if (h_nsteps[1] > 0) {
          PathArgs p2 = pa;
          p2.from_back = true;
          k_paths<OTR_CAP1, 2><<<(unsigned)grid_paths((int64_t)h_nsteps[1]).blocks, 64, 0, stream>>>(g, p2, nullptr,
                                                                                                     nullptr);
        }
      } else {
        // (steps <= states: two searches per wave)
        k_paths<OTR_CAP1, 2><<<(unsigned)grid_paths(S).blocks, 64, 0, stream>>>(g, pa, nullptr, nullptr);
      }
      te(OTR_STAGE_PATHS);
      tb(OTR_STAGE_PATHS_BIG);
      // large-table retries for table overflows (flag 1), on device-side lists; each
      // launch's waves claim steps from its own per-XCD queue (XcdQueue)
      for (int tier = 0; tier < 3; ++tier) {
        unsigned long long* c = cnt + 12 + tier;
        k_collect_tier_list<<<grid_for(S, 1024), 1024, 0, stream>>>(nscan_d, step_ovf, 0x2u, list, c);
        PathArgs pb = pa;
        pb.queue = pq + tier * kPQWords;
        if (tier == 0) k_paths<512, 1><<<pgrid(16384, S), 64, 0, stream>>>(g, pb, list, c);
        else if (tier == 1) k_paths<1024, 1><<<pgrid(8192, S), 64, 0, stream>>>(g, pb, list, c);
        else k_paths<4096, 1><<<pgrid(4096, S), 64, 0, stream>>>(g, pb, list, c);
      }
      // turn-cost winners (flag 5): the edge-state LDS search, 384 then 2048 states
      if (turn_modes != 0u) {
        for (int et = 0; et < 2; ++et) {
          unsigned long long* c = cnt + 27 + et;
          k_collect_tier_list<<<grid_for(S, 1024), 1024, 0, stream>>>(nscan_d, step_ovf, et == 0 ? 0x20u : 0x40u,
                                                                       list, c);
          PathArgs pb = pa;
          pb.queue = pq + (3 + et) * kPQWords;
          if (et == 0) k_paths_edge<384><<<pgrid(4096, S), 64, 0, stream>>>(g, pb, d_turn, list, c, 6);
          else k_paths_edge<2048><<<pgrid(512, S), 64, 0, stream>>>(g, pb, d_turn, list, c, 3);
        }
      }
      // 64-bit labels, the largest-table overflows and what the edge tiers left: k_general
      ga.steps = steps;
      ga.winner = va.winner;
      ga.path_off = path_off;
      ga.path_len = path_len;
      ga.path = path;
      ga.cursor = cnt + 32;
      ga.capacity = capacity;
      ga.cap_flag = (int32_t*)(cnt + 20);
      for (int gt = 0; gt < 2; ++gt) {
        unsigned long long* c = cnt + 16 + gt;
        k_collect_tier_list<<<grid_for(S, 1024), 1024, 0, stream>>>(nscan_d, step_ovf, gt == 0 ? 0xAu : 0x2u, list,
                                                                     c);
        GSlabs gs2;
        if ((rc = slabs(gt, &gs2))) return rc;
        ga.mode = 1;
        ga.list = list;
        ga.list_count = c;
        ga.flag = step_ovf;
        ga.counters = nullptr;
        k_general<<<pgrid(gs2.n, S), kGenThreads, 0, stream>>>(g, ga, gs2);
      }
      // steps still flagged (beyond a 1M-state slab): named after the final sync
      k_collect_tier_list<<<grid_for(S, 1024), 1024, 0, stream>>>(nscan_d, step_ovf, 0xAu, list, cnt + 18);
      te(OTR_STAGE_PATHS_BIG);
      unsigned long long capflag = 0;
      std::vector<unsigned long long> cur(kShards);
      HIPCHK(hipMemcpyAsync(&capflag, cnt + 20, 8, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(cur.data(), cnt + 32, 8 * kShards, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      if ((capflag & 0xFFFFFFFFu) == 0) {  // every path fitted its region
        paths_fit = true;
        break;
      }
      unsigned long long mx = 0;
      for (auto c : cur) mx = c > mx ? c : mx;
      capacity = kShards * ((int64_t)mx + (int64_t)mx / 2 + 1024);  // grow and redo
    }
    if (!paths_fit) {  // (the capacity grows 1.5x past the largest shard: never seen)
      if (err) *err = "winner paths did not fit the path buffer after 8 attempts";
      return OTR_DEVICE_ERROR;
    }
  }
  // ---- K7: stitching, segments, report()
  int64_t* cap = need<int64_t>(S_CAP, T);
  int64_t* cap_off = need<int64_t>(S_CAP_OFF, T + 1);
  k_capacity<<<grid_for(T, 256), 256, 0, stream>>>(T, trace_state_off, cb.count, path_len, cap);
  if ((rc = scan(cap, cap_off, T))) return rc;
  int64_t C = 0;
  if ((rc = read_i64(cap_off + T, &C))) return rc;
  SegArgs sa{};
  sa.b = b;
  sa.trace_state_off = trace_state_off;
  sa.state_probe = state_probe;
  sa.cand_count = cb.count;
  sa.cand_edge = cb.edge;
  sa.cand_p = cb.p;
  sa.prev = sb.prev;
  sa.brk = va.brk;
  sa.winner = va.winner;
  sa.path_off = path_off;
  sa.path_len = path_len;
  sa.path = (const uint32_t*)need<uint32_t>(S_PATH, 1);
  sa.pos = need<int64_t>(S_POS, S);
  sa.act = need<int64_t>(S_ACT, S);
  sa.ent = need<int64_t>(S_ENT, S);
  sa.suba = need<int32_t>(S_SUBA, S);
  sa.subb = need<int32_t>(S_SUBB, S);
  sa.por_e = need<uint32_t>(S_POR_E, C);
  sa.por_s0 = need<int64_t>(S_POR_S0, C);
  sa.por_s1 = need<int64_t>(S_POR_S1, C);
  sa.por_sa = need<int32_t>(S_POR_SA, C);
  sa.gstart = need<int32_t>(S_GSTART, C);
  sa.cap_off = cap_off;
  sa.route = need<uint32_t>(S_ROUTE, C);
  sa.route_n = need<int64_t>(S_ROUTE_N, T);
  sa.seg_id = need<unsigned long long>(S_SEG_ID, C);
  sa.seg_start = need<double>(S_SEG_START, C);
  sa.seg_end = need<double>(S_SEG_END, C);
  sa.seg_length = need<int32_t>(S_SEG_LEN, C);
  sa.seg_queue = need<int32_t>(S_SEG_QUEUE, C);
  sa.seg_internal = need<uint8_t>(S_SEG_INTERNAL, C);
  sa.seg_bshape = need<int32_t>(S_SEG_BSHAPE, C);
  sa.seg_eshape = need<int32_t>(S_SEG_ESHAPE, C);
  sa.seg_index = need<uint32_t>(S_SEG_INDEX, C);
  sa.seg_n = need<int64_t>(S_SEG_N, T);
  sa.seg_way_n = need<int64_t>(S_SEG_WAY_N, C);
  sa.seg_way = need<uint32_t>(S_SEG_WAY, C);
  sa.way_n = need<int64_t>(S_WAY_N, T);
  sa.rep_id = need<unsigned long long>(S_REP_ID, C);
  sa.rep_next = need<unsigned long long>(S_REP_NEXT, C);
  sa.rep_t0 = need<double>(S_REP_T0, C);
  sa.rep_t1 = need<double>(S_REP_T1, C);
  sa.rep_length = need<int32_t>(S_REP_LEN, C);
  sa.rep_queue = need<int32_t>(S_REP_QUEUE, C);
  sa.rep_seg = need<uint32_t>(S_REP_SEG, C);
  sa.rep_n = need<int64_t>(S_REP_N, T);
  sa.shape_used = need<int32_t>(S_SHAPE_USED, T);
  sa.stats = need<int32_t>(S_STATS, 7 * (size_t)T);
  sa.stats_len = need<double>(S_STATS_LEN, 2 * (size_t)T);
  sa.threshold = (double)(in->threshold_sec >= 0 ? in->threshold_sec : 15);
  sa.report_levels = in->report_levels;
  sa.transition_levels = in->transition_levels;
  for (int m = 0; m < OTR_MODES; ++m) sa.queue_kph[m] = mp.m[m].queue_kph;
  tb(OTR_STAGE_SEGMENTS);
  k_segments<<<(unsigned)grid_segments(T).blocks, 64, 0, stream>>>(g, sa, d_counters);
  te(OTR_STAGE_SEGMENTS);
  // ---- K8: hour buckets → histogram
  HistArgs ha{};
  ha.b = b;
  ha.cap_off = cap_off;
  ha.rep_n = sa.rep_n;
  ha.rep_id = sa.rep_id;
  ha.rep_t0 = sa.rep_t0;
  ha.rep_t1 = sa.rep_t1;
  ha.rep_length = sa.rep_length;
  ha.rep_queue = sa.rep_queue;
  ha.rep_seg = sa.rep_seg;
  ha.quantisation = in->quantisation > 0 ? in->quantisation : 3600;
  ha.base_time = in->hist_base_time;
  ha.hours = in->hist_hours;
  ha.n_segments = g.n_segments;
  ha.n_rows = d_counters + 8 * kCShards;
  size_t hist_len = (size_t)(in->hist_hours > 0 ? in->hist_hours : 0) * g.n_segments * OTR_HIST_BINS;
  ha.hist = hist_len ? (in->hist_device ? in->hist_device : need<uint32_t>(S_HIST, hist_len)) : nullptr;
  if (hist_len) HIPCHK(hipMemsetAsync(ha.hist, 0, hist_len * 4, stream));
  tb(OTR_STAGE_HISTOGRAM);
  // K8 also counts the rows (n_rows) when K9 does not
  if (hist_len || !(in->flags & OTR_BATCH_TILE_ROWS))
    k_histogram<<<(unsigned)grid_trace_rows(T).blocks, 256, 0, stream>>>(ha);
  te(OTR_STAGE_HISTOGRAM);
  // ---- K9: simple_reporter tile rows (optional)
  if (in->flags & OTR_BATCH_TILE_ROWS) {
    TileArgs ta{};
    ta.b = b;
    ta.cap_off = cap_off;
    ta.rep_n = sa.rep_n;
    ta.rep_id = sa.rep_id;
    ta.rep_next = sa.rep_next;
    ta.rep_t0 = sa.rep_t0;
    ta.rep_t1 = sa.rep_t1;
    ta.rep_length = sa.rep_length;
    ta.rep_queue = sa.rep_queue;
    ta.quantisation = ha.quantisation;
    ta.rules = in->tile_rules;
    ta.row_cnt = need<int64_t>(S_ROW_CNT, T);
    k_tile_rows<<<(unsigned)grid_trace_rows(T).blocks, 256, 0, stream>>>(ta);
    int64_t* row_off = need<int64_t>(S_ROW_OFF, T + 1);
    if ((rc = scan(ta.row_cnt, row_off, T))) return rc;
    int64_t R = 0;
    if ((rc = read_i64(row_off + T, &R))) return rc;
    ta.row_off = row_off;
    ta.rows = need<otr_tile_row>(S_ROWS, R > 0 ? R : 1);
    if (R > 0) k_tile_rows<<<(unsigned)grid_trace_rows(T).blocks, 256, 0, stream>>>(ta);
    out->d_rows = ta.rows;
    out->n_rows = R;
  }
  HIPCHK(hipGetLastError());
  std::vector<unsigned long long> hc(n_ctr);
  unsigned long long h_fail[2] = {0ull, 0ull};  // route tasks / paths beyond every search tier
  k_ctr_fold<<<(unsigned)n_ctr, kCShards, 0, stream>>>(d_counters, d_counters + kBanks * bank);
  HIPCHK(hipMemcpyAsync(hc.data(), d_counters + kBanks * bank, n_ctr * 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&h_fail[0], cnt + 10, 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&h_fail[1], cnt + 18, 8, hipMemcpyDeviceToHost, stream));
  // per-trace output counts in the same drain (one host wait per batch for all of them)
  std::vector<int64_t> route_n(T), seg_n(T), way_n(T), rep_n(T);
  HIPCHK(hipMemcpyAsync(route_n.data(), sa.route_n, 8 * T, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(seg_n.data(), sa.seg_n, 8 * T, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(rep_n.data(), sa.rep_n, 8 * T, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(way_n.data(), sa.way_n, 8 * T, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (h_fail[0] + h_fail[1] > 0 && getenv("OTR_DEBUG_FAIL")) {  // diagnostic: which stage, which tiers
    unsigned long long hc2[32];
    HIPCHK(hipMemcpy(hc2, cnt, 8 * 32, hipMemcpyDeviceToHost));
    fprintf(stderr, "otr: %llu route tasks, %llu paths beyond every tier; tier lists:", h_fail[0], h_fail[1]);
    for (int k = 0; k < 32; ++k) fprintf(stderr, " %llu", hc2[k]);
    fprintf(stderr, "\n");
    if (h_fail[1]) {  // the first failing winner paths: state, its step's bound and winning route
      const int64_t* steps_d = need<int64_t>(S_LIST2, 1);
      std::vector<int64_t> ks(std::min<unsigned long long>(h_fail[1], 6));
      HIPCHK(hipMemcpy(ks.data(), list, 8 * ks.size(), hipMemcpyDeviceToHost));
      for (int64_t k : ks) {
        int64_t s = 0, sp = 0, to = 0;
        int32_t wi = 0, wj = 0, K = 0;
        double bd = 0;
        HIPCHK(hipMemcpy(&s, steps_d + k, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&sp, sb.prev + s, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&wj, need<int32_t>(S_WINNER, 1) + s, 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&wi, need<int32_t>(S_WINNER, 1) + sp, 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&K, cb.count + s, 4, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&to, trans_off + s, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&bd, sb.bound + s, 8, hipMemcpyDeviceToHost));
        uint32_t r = 0;
        HIPCHK(hipMemcpy(&r, trans + to + (int64_t)wi * K + wj, 4, hipMemcpyDeviceToHost));
        fprintf(stderr, "otr: step k %lld state %lld prev %lld winners %d/%d K %d trans_off %lld bound %.3f route %u\n",
                (long long)k, (long long)s, (long long)sp, wi, wj, K, (long long)to, bd, r);
      }
    }
  }
  if (h_fail[0] + h_fail[1] > 0) {
    // beyond a 1M-state slab (never seen): name the traces (task/step -> state -> trace)
    for (int which = 0; which < 2; ++which) {
      const unsigned long long nf = h_fail[which];
      if (!nf) continue;
      std::vector<int64_t> idx(nf), st(nf);
      HIPCHK(hipMemcpy(idx.data(), which == 0 ? fail_tasks : list, 8 * nf, hipMemcpyDeviceToHost));
      const int64_t* src = need<int64_t>(S_LIST2, 1);  // (steps: the step list; tasks: their records)
      for (unsigned long long k = 0; k < nf; ++k) {
        int64_t sidx = 0;
        int32_t t = 0;
        if (which == 0) {
          uint32_t s32 = 0;
          HIPCHK(hipMemcpy(&s32, task_rec + 3 * idx[k], 4, hipMemcpyDeviceToHost));
          sidx = s32;
        } else {
          HIPCHK(hipMemcpy(&sidx, src + idx[k], 8, hipMemcpyDeviceToHost));
        }
        HIPCHK(hipMemcpy(&t, state_trace + sidx, 4, hipMemcpyDeviceToHost));
        if (t >= 0 && t < T && h_trace_status[t] == OTR_OK) {
          h_trace_status[t] = OTR_MATCH_ERROR;
          ++out->n_overflow_traces;
        }
      }
    }
  }
  auto ctr = [&](int b, int k) {
    return hc[(size_t)b * OTR_COUNTERS + (size_t)k];
  };
  for (int k = 0; k < OTR_COUNTERS; ++k) out->counters[k] = ctr(0, k);
  for (int k : {3, 4, 13, 14}) out->counters[k] += ctr(12, k) + ctr(13, k);  // (the first tier: every launch)
  // per route kernel: searches, settled, relaxed, transition entries (banks 0, 2..6, 8..9;
  // slot 8, the 64-bit LDS tier: bank 7; the edge-state tiers: slot 10 the first (bank 10),
  // slot 9 the 512-state one (bank 1), slot 11 the 1024-state one (bank 11))
  for (int t = 0; t < 14; ++t) {
    const int b = t == 0 ? 0 : (t < 6 ? 1 + t : (t < 8 ? 2 + t : (t == 8 ? 7 : (t == 9 ? 1 : t))));
    out->route_tier_work[t][0] = ctr(b, 6);
    out->route_tier_work[t][1] = ctr(b, 3);
    out->route_tier_work[t][2] = ctr(b, 4);
    out->route_tier_work[t][3] = ctr(b, 5);
    if ((t >= 1 && t < 6) || t == 8) {  // the LDS retry tiers together (counters 9 / 10)
      out->counters[9] += ctr(b, 3);
      out->counters[10] += ctr(b, 4);
    }
  }
  out->counters[5] = (uint64_t)NT;
  out->counters[6] = (uint64_t)NTR;
  // edge-state searches resumed from a dump (the 512- and 1024-state tiers) and dumped
  // (the first two edge tiers), with OTR_BATCH_ROUTE_WORK
  out->counters[22] = ctr(1, 22) + ctr(11, 22);
  out->counters[23] = ctr(10, 23) + ctr(1, 23);
  // node searches resumed from / dumped to a retry tier's dump (the node retry tiers, banks 2..6)
  out->counters[11] = out->counters[12] = 0;
  for (int b = 2; b < 7; ++b) {
    out->counters[11] += ctr(b, 11);
    out->counters[12] += ctr(b, 12);
  }
  if (!(in->flags & OTR_BATCH_TILE_ROWS)) out->n_rows = (int64_t)out->counters[8];
  else out->counters[8] = (uint64_t)out->n_rows;  // K9 counted them (K8 may not have run)
  out->d_hist = ha.hist;
  out->hist_len = (int64_t)hist_len;
  if (timing) {
    for (int k = 0; k < 10; ++k)
      if (used[k]) (void)hipEventElapsedTime(&out->kernel_ms[k], ev[2 * k], ev[2 * k + 1]);
    for (int t = 1; t < 14; ++t)
      if (out->route_tier_code[t] != 0)
        (void)hipEventElapsedTime(&out->route_tier_ms[t], ev[24 + 2 * t], ev[24 + 2 * t + 1]);
    // (the route stage holds the tiny and small tiers' launches, then the two-search tier's)
    out->route_tier_ms[0] = out->kernel_ms[OTR_STAGE_ROUTE] - out->route_tier_ms[12] - out->route_tier_ms[13];
    (void)hipGetLastError();  // an unrecorded pair must not leave a sticky error for the next call
  }
  // ---- copy-out (tests / JSON path), compacting the capacity layout
  int64_t nroute = 0, nseg = 0, nrep = 0;
  for (int t = 0; t < T; ++t) {
    nroute += route_n[t];
    nseg += seg_n[t];
    nrep += rep_n[t];
  }
  out->n_route = nroute;
  out->n_seg = nseg;
  out->n_rep = nrep;
  out->status = out->n_overflow_traces ? OTR_MATCH_ERROR : OTR_OK;
  const bool full = (in->flags & OTR_BATCH_COPY_OUT) != 0;
  if (!full && !(in->flags & OTR_BATCH_COPY_REPORTS)) return OTR_OK;
  out->trace_status = h_trace_status.data();
  auto dl = [&](auto& vec, const void* src, size_t n) -> int {
    vec.resize(n ? n : 1);
    if (n) HIPCHK(hipMemcpyAsync(vec.data(), src, n * sizeof(vec[0]), hipMemcpyDeviceToHost, stream));
    return OTR_OK;
  };
  if (full) {
    if ((rc = dl(h_trace_state_off, trace_state_off, T + 1))) return rc;
    if ((rc = dl(h_state_probe, state_probe, S))) return rc;
    if ((rc = dl(h_cand_count, cb.count, S))) return rc;
    if ((rc = dl(h_cand_edge, cb.edge, (size_t)S * OTR_KMAX))) return rc;
    if ((rc = dl(h_cand_p, cb.p, (size_t)S * OTR_KMAX))) return rc;
    if ((rc = dl(h_cand_sqd, cb.sqd, (size_t)S * OTR_KMAX))) return rc;
    if ((rc = dl(h_winner, va.winner, S))) return rc;
    if ((rc = dl(h_subpath, va.subpath, S))) return rc;
  }
  if ((rc = dl(h_shape_used, sa.shape_used, T))) return rc;
  if ((rc = dl(h_stats, sa.stats, 7 * (size_t)T))) return rc;
  if ((rc = dl(h_stats_len, sa.stats_len, 2 * (size_t)T))) return rc;
  // dense layout on device (k_compact), then only the used entries cross PCIe
  int64_t nway = 0;
  for (int t = 0; t < T; ++t) nway += way_n[t];
  CompactArgs ca{};
  ca.n_traces = T;
  ca.cap_off = cap_off;
  int64_t* route_off = need<int64_t>(S_C_ROUTE_OFF, T + 1);
  int64_t* seg_off = need<int64_t>(S_C_SEG_OFF, T + 1);
  int64_t* way_off = need<int64_t>(S_C_WAY_OFF, T + 1);
  int64_t* rep_off = need<int64_t>(S_C_REP_OFF, T + 1);
  if ((rc = scan(sa.seg_n, seg_off, T)) || (rc = scan(sa.way_n, way_off, T)) || (rc = scan(sa.rep_n, rep_off, T)))
    return rc;
  if (full && (rc = scan(sa.route_n, route_off, T))) return rc;
  ca.route_off = full ? route_off : nullptr;
  ca.seg_off = seg_off;
  ca.way_off = way_off;
  ca.rep_off = rep_off;
  SegArgs* d_sa = need<SegArgs>(S_C_ARGS, 1);
  HIPCHK(hipMemcpyAsync(d_sa, &sa, sizeof(SegArgs), hipMemcpyHostToDevice, stream));
  ca.s = d_sa;
  auto n1 = [](int64_t n) { return (size_t)(n > 0 ? n : 1); };
  ca.route = need<uint32_t>(S_C_ROUTE, n1(nroute));
  ca.seg_id = need<unsigned long long>(S_C_SEG_ID, n1(nseg));
  ca.seg_start = need<double>(S_C_SEG_START, n1(nseg));
  ca.seg_end = need<double>(S_C_SEG_END, n1(nseg));
  ca.seg_length = need<int32_t>(S_C_SEG_LEN, n1(nseg));
  ca.seg_queue = need<int32_t>(S_C_SEG_QUEUE, n1(nseg));
  ca.seg_internal = need<uint8_t>(S_C_SEG_INTERNAL, n1(nseg));
  ca.seg_bshape = need<int32_t>(S_C_SEG_BSHAPE, n1(nseg));
  ca.seg_eshape = need<int32_t>(S_C_SEG_ESHAPE, n1(nseg));
  ca.seg_way_n = need<int64_t>(S_C_SEG_WAY_N, n1(nseg));
  ca.seg_way = need<uint32_t>(S_C_SEG_WAY, n1(nway));
  ca.rep_id = need<unsigned long long>(S_C_REP_ID, n1(nrep));
  ca.rep_next = need<unsigned long long>(S_C_REP_NEXT, n1(nrep));
  ca.rep_t0 = need<double>(S_C_REP_T0, n1(nrep));
  ca.rep_t1 = need<double>(S_C_REP_T1, n1(nrep));
  ca.rep_length = need<int32_t>(S_C_REP_LEN, n1(nrep));
  ca.rep_queue = need<int32_t>(S_C_REP_QUEUE, n1(nrep));
  k_compact<<<(unsigned)grid_compact(T).blocks, 64, 0, stream>>>(ca);
  int64_t* seg_way_off = need<int64_t>(S_C_SEG_WAY_OFF, (size_t)nseg + 1);
  if ((rc = scan(ca.seg_way_n, seg_way_off, nseg))) return rc;
  HIPCHK(hipGetLastError());
  if (full && (rc = dl(h_route_edge, ca.route, nroute))) return rc;
  if (!full) h_route_edge.clear();
  if ((rc = dl(h_seg_id, ca.seg_id, nseg)) || (rc = dl(h_seg_start, ca.seg_start, nseg)) ||
      (rc = dl(h_seg_end, ca.seg_end, nseg)) || (rc = dl(h_seg_length, ca.seg_length, nseg)) ||
      (rc = dl(h_seg_queue, ca.seg_queue, nseg)) || (rc = dl(h_seg_internal, ca.seg_internal, nseg)) ||
      (rc = dl(h_seg_bshape, ca.seg_bshape, nseg)) || (rc = dl(h_seg_eshape, ca.seg_eshape, nseg)) ||
      (rc = dl(h_seg_way_off, seg_way_off, (size_t)nseg + 1)) || (rc = dl(h_seg_way, ca.seg_way, nway)) ||
      (rc = dl(h_rep_id, ca.rep_id, nrep)) || (rc = dl(h_rep_next, ca.rep_next, nrep)) ||
      (rc = dl(h_rep_t0, ca.rep_t0, nrep)) || (rc = dl(h_rep_t1, ca.rep_t1, nrep)) ||
      (rc = dl(h_rep_length, ca.rep_length, nrep)) || (rc = dl(h_rep_queue, ca.rep_queue, nrep)))
    return rc;
  HIPCHK(hipStreamSynchronize(stream));
  h_trace_route_off.assign(T + 1, 0);
  h_trace_seg_off.assign(T + 1, 0);
  h_trace_rep_off.assign(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    h_trace_route_off[t + 1] = h_trace_route_off[t] + route_n[t];
    h_trace_seg_off[t + 1] = h_trace_seg_off[t] + seg_n[t];
    h_trace_rep_off[t + 1] = h_trace_rep_off[t] + rep_n[t];
  }
  auto P = [](auto& v) { return v.empty() ? nullptr : v.data(); };
  if (full) {
    out->trace_state_off = P(h_trace_state_off);
    out->state_probe = P(h_state_probe);
    out->cand_count = P(h_cand_count);
    out->cand_edge = P(h_cand_edge);
    out->cand_p = P(h_cand_p);
    out->cand_sqd = P(h_cand_sqd);
    out->winner = P(h_winner);
    out->subpath = P(h_subpath);
    out->trace_route_off = P(h_trace_route_off);
    out->route_edge = P(h_route_edge);
  }
  out->trace_seg_off = P(h_trace_seg_off);
  out->seg_id = (uint64_t*)P(h_seg_id);
  out->seg_start = P(h_seg_start);
  out->seg_end = P(h_seg_end);
  out->seg_length = P(h_seg_length);
  out->seg_queue = P(h_seg_queue);
  out->seg_internal = P(h_seg_internal);
  out->seg_begin_shape = P(h_seg_bshape);
  out->seg_end_shape = P(h_seg_eshape);
  out->seg_way_off = P(h_seg_way_off);
  out->seg_way = P(h_seg_way);
  out->trace_rep_off = P(h_trace_rep_off);
  out->rep_id = (uint64_t*)P(h_rep_id);
  out->rep_next = (uint64_t*)P(h_rep_next);
  out->rep_t0 = P(h_rep_t0);
  out->rep_t1 = P(h_rep_t1);
  out->rep_length = P(h_rep_length);
  out->rep_queue = P(h_rep_queue);
  out->shape_used = P(h_shape_used);
  out->stats = P(h_stats);
  out->stats_len = P(h_stats_len);
  return OTR_OK;
}

// report() over many segment lists on the device (include/otr.h otr_report_lists_device):
// one thread per list runs the report_segments K7 runs.
__global__ void k_report_lists(ReportLists a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  const int64_t o = a.seg_off[c];
  ReportStats rs;
  report_segments((int32_t)(a.seg_off[c + 1] - o), a.seg_id + o, a.start + o, a.end + o, a.internal + o, a.queue + o,
                  a.has_length + o, a.length + o, a.begin_shape + o, nullptr, a.end_time[c], a.threshold[c], a.rl[c],
                  a.tl[c], a.rep_id + o, a.rep_next + o, a.rep_t0 + o, a.rep_t1 + o, a.rep_length + o, a.rep_queue + o,
                  nullptr, &rs);
  a.n_rep[c] = rs.n_rep;
  a.shape_used[c] = rs.shape_used;
  for (int k = 0; k < 6; ++k) a.counts[6 * c + k] = rs.counts[k];
  for (int k = 0; k < 2; ++k) {
    a.lengths[2 * c + k] = rs.lengths[k];
    a.length_set[2 * c + k] = rs.length_set[k];
  }
}

int report_lists_device(const ReportLists& h, std::string* err) {
  GraphState& gs = graph_state();
  HIPCHK(hipSetDevice(gs.device));
  const int32_t n = h.n;
  if (n <= 0) return OTR_OK;
  const int64_t S = h.seg_off[n];
  std::vector<void*> mem;
  bool ok = true;
  auto put = [&](const void* src, size_t bytes) -> void* {
    void* d = nullptr;
    if (hipMalloc(&d, bytes ? bytes : 16) != hipSuccess) ok = false;
    mem.push_back(d);
    if (ok && bytes && src && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
    return d;
  };
  ReportLists d = h;
  d.seg_off = (const int64_t*)put(h.seg_off, 8ull * (n + 1));
  d.seg_id = (const unsigned long long*)put(h.seg_id, 8ull * S);
  d.start = (const double*)put(h.start, 8ull * S);
  d.end = (const double*)put(h.end, 8ull * S);
  d.internal = (const uint8_t*)put(h.internal, (size_t)S);
  d.queue = (const int32_t*)put(h.queue, 4ull * S);
  d.has_length = (const uint8_t*)put(h.has_length, (size_t)S);
  d.length = (const int32_t*)put(h.length, 4ull * S);
  d.begin_shape = (const int32_t*)put(h.begin_shape, 4ull * S);
  d.end_time = (const int64_t*)put(h.end_time, 8ull * n);
  d.threshold = (const double*)put(h.threshold, 8ull * n);
  d.rl = (const uint32_t*)put(h.rl, 4ull * n);
  d.tl = (const uint32_t*)put(h.tl, 4ull * n);
  d.rep_id = (unsigned long long*)put(nullptr, 8ull * S);
  d.rep_next = (unsigned long long*)put(nullptr, 8ull * S);
  d.rep_t0 = (double*)put(nullptr, 8ull * S);
  d.rep_t1 = (double*)put(nullptr, 8ull * S);
  d.rep_length = (int32_t*)put(nullptr, 4ull * S);
  d.rep_queue = (int32_t*)put(nullptr, 4ull * S);
  d.n_rep = (int32_t*)put(nullptr, 4ull * n);
  d.shape_used = (int32_t*)put(nullptr, 4ull * n);
  d.counts = (int32_t*)put(nullptr, 24ull * n);
  d.lengths = (double*)put(nullptr, 16ull * n);
  d.length_set = (int32_t*)put(nullptr, 8ull * n);
  auto release = [&] {
    for (void* q : mem)
      if (q) (void)hipFree(q);
  };
  if (!ok) {
    release();
    if (err) *err = "device allocation failed (report lists)";
    return OTR_DEVICE_ERROR;
  }
  k_report_lists<<<grid_for(n, 128), 128>>>(d);
  hipError_t e = hipDeviceSynchronize();
  auto get = [&](void* dst, const void* src, size_t bytes) {
    if (e == hipSuccess && bytes) e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
  };
  get(h.rep_id, d.rep_id, 8ull * S);
  get(h.rep_next, d.rep_next, 8ull * S);
  get(h.rep_t0, d.rep_t0, 8ull * S);
  get(h.rep_t1, d.rep_t1, 8ull * S);
  get(h.rep_length, d.rep_length, 4ull * S);
  get(h.rep_queue, d.rep_queue, 4ull * S);
  get(h.n_rep, d.n_rep, 4ull * n);
  get(h.shape_used, d.shape_used, 4ull * n);
  get(h.counts, d.counts, 24ull * n);
  get(h.lengths, d.lengths, 16ull * n);
  get(h.length_set, d.length_set, 8ull * n);
  release();
  if (e != hipSuccess) {
    if (err) *err = std::string("HIP error: ") + hipGetErrorString(e);
    return OTR_DEVICE_ERROR;
  }
  return OTR_OK;
}

// Tile stage: sort rows into simple_reporter's line order per file, then cull
// (K10).  Result rows are copied to host (matcher-owned).
int Matcher::tiles_cull(const otr_tile_row* rows, int64_t n, int memory, int privacy, int rules,
                        const otr_tile_row** out, int64_t* n_out, std::string* err) {
  try {
    return tiles_cull_impl(rows, n, memory, privacy, rules, out, n_out, err);
  } catch (const DeviceOom& o) {
    return oom_error(stream, o, err);
  }
}

int Matcher::tiles_cull_impl(const otr_tile_row* rows, int64_t n, int memory, int privacy, int rules,
                        const otr_tile_row** out, int64_t* n_out, std::string* err) {
  GraphState& gs = graph_state();
  HIPCHK(hipSetDevice(gs.device));
  if (!stream) HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  *n_out = 0;
  *out = nullptr;
  h_tile_rows.clear();
  if (n <= 0) return OTR_OK;
  if (n >= (int64_t)INT32_MAX) {
    if (err) *err = "too many tile rows for one call";
    return OTR_BAD_REQUEST;
  }
  // staging: in (copy of the caller's rows), sorted, kept; permutation + radix keys
  otr_tile_row* d_in = need<otr_tile_row>(S_ROWS_IN, n);
  otr_tile_row* d = need<otr_tile_row>(S_ROWS_OUT, n);
  otr_tile_row* d_kept = need<otr_tile_row>(S_ROWS_KEPT, n);
  int32_t* perm_a = need<int32_t>(S_IDX_A, n);
  int32_t* perm_b = need<int32_t>(S_IDX_B, n);
  unsigned long long* key_a = need<unsigned long long>(S_KEY_A, n);
  unsigned long long* key_b = need<unsigned long long>(S_KEY_B, n);
  int64_t* head = need<int64_t>(S_FILE_HEAD, n);
  int64_t* keep = need<int64_t>(S_KEEP, n);
  int64_t* pos = need<int64_t>(S_POS_SCAN, n);
  int64_t* fstart = need<int64_t>(S_FILE_START, n);
  if (!d_in || !d || !d_kept || !perm_a || !perm_b || !key_a || !key_b || !head || !keep || !pos || !fstart) {
    if (err) *err = "device allocation failed (tiles)";
    return OTR_DEVICE_ERROR;
  }
  HIPCHK(hipMemcpyAsync(d_in, rows, sizeof(otr_tile_row) * n,
                        memory == OTR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, stream));
  const int ni = (int)n;
  size_t tb_sort = 0, tb_scan = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, key_a, key_b, perm_a, perm_b, ni, 0, 64, stream));
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan, head, pos, ni, stream));
  void* tmp = need<char>(S_SORT_TMP, std::max(tb_sort, tb_scan));
  if (!tmp) {
    if (err) *err = "device allocation failed (tiles)";
    return OTR_DEVICE_ERROR;
  }
  // LSD over the sort fields: stable radix passes, least significant field first (the
  // identity start keeps arrival order within equal keys)
  k_iota_i32<<<grid_for(n, 256), 256, 0, stream>>>(perm_a, n);
  const bool pair_order = rules == OTR_TILE_RULES_STREAM;
  for (int f = pair_order ? TF_NEXT : TF_COUNT - 1; f >= 0; --f) {
    if (pair_order) k_pair_key<<<grid_for(n, 256), 256, 0, stream>>>(d_in, perm_a, n, f, key_a);
    else k_line_key<<<grid_for(n, 256), 256, 0, stream>>>(d_in, perm_a, n, f, key_a);
    size_t tb = tb_sort;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key_a, key_b, perm_a, perm_b, ni, 0,
                                              (f == TF_FILE || pair_order) ? 64 : 63, stream));
    std::swap(perm_a, perm_b);
  }
  k_gather_rows<<<grid_for(n, 256), 256, 0, stream>>>(d_in, perm_a, n, d);
  // runs of equal (file, id, next_id): heads → scan → run starts; per-run decision
  k_run_heads<<<grid_for(n, 256), 256, 0, stream>>>(d, n, head);
  size_t tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, pos, ni, stream));
  k_scatter_index<<<grid_for(n, 256), 256, 0, stream>>>(head, pos, n, fstart);
  int64_t nr = 0;
  HIPCHK(hipMemcpyAsync(&nr, pos + (n - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (nr < 1 || nr > n) {
    if (err) *err = "tile run split failed";
    return OTR_DEVICE_ERROR;
  }
  uint8_t* run_keep = need<uint8_t>(S_RUN_KEEP, nr);
  if (!run_keep) {
    if (err) *err = "device allocation failed (tiles)";
    return OTR_DEVICE_ERROR;
  }
  k_cull_runs<<<grid_for(nr, 256), 256, 0, stream>>>(d, n, fstart, nr, privacy, run_keep);
  k_row_keep<<<grid_for(n, 256), 256, 0, stream>>>(pos, run_keep, n, keep);
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, keep, head, ni, stream));  // head: reused as positions
  std::swap(pos, head);
  k_scatter_flagged<otr_tile_row><<<grid_for(n, 256), 256, 0, stream>>>(d, keep, pos, n, d_kept);
  int64_t nk = 0;
  HIPCHK(hipMemcpyAsync(&nk, pos + (n - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (nk < 0 || nk > n) {
    if (err) *err = "tile cull compaction failed";
    return OTR_DEVICE_ERROR;
  }
  h_tile_rows.resize(nk > 0 ? nk : 1);
  if (nk > 0) HIPCHK(hipMemcpy(h_tile_rows.data(), d_kept, sizeof(otr_tile_row) * nk, hipMemcpyDeviceToHost));
  HIPCHK(hipGetLastError());
  *out = h_tile_rows.data();
  *n_out = nk;
  return OTR_OK;
}

// ---- keyed speed histogram (include/otr.h otr_hist_reduce) -----------------
__global__ void k_rows_to_entries(const otr_tile_row* r, int64_t n, otr_hist_entry* e) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  otr_hist_entry x;
  x.file = r[i].file;
  x.id = r[i].id;
  x.next_id = r[i].next_id;
  x.speed_bin = (uint32_t)r[i].speed_bin;
  x.count = 1u;
  e[i] = x;
}
// key ranges of the entries, for the fewest radix-sort bits: OR of the ids and next ids
// (their widths), min / max hour bucket, and whether every file is the one K9 derives
// from its id (bucket << 25 | level << 22 | tile: then (file, id) order is (bucket,
// level, tile, index) order, one packed key)
struct EntryRange {
  unsigned long long id_or, next_or, file_or, bmin, bmax, foreign;
};
// a fixed grid (kRangeBlocks x 1024) strides over the entries; one set of atomics per
// block (one per wave queued ~23K atomics on a single line: 263 us for 244K entries)
constexpr int kRangeBlocks = 128;
__global__ __launch_bounds__(1024) void k_entry_range(const otr_hist_entry* e, int64_t n, EntryRange* r) {
  unsigned long long v[6] = {0ull, 0ull, 0ull, ~0ull, 0ull, 0ull};  // id, next, file OR; bmin; bmax; foreign
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const otr_hist_entry x = e[i];
    v[0] |= x.id;
    v[1] |= x.next_id;
    v[2] |= x.file;
    const unsigned long long b = x.file >> 25;
    v[3] = b < v[3] ? b : v[3];
    v[4] = b > v[4] ? b : v[4];
    v[5] |= (x.file & 0x1FFFFFFull) != (((x.id & 7ull) << 22) | ((x.id >> 3) & 0x3FFFFFull)) ? 1ull : 0ull;
  }
  for (int o = OTR_WAVE / 2; o > 0; o >>= 1) {
    for (int q : {0, 1, 2, 5}) v[q] |= __shfl_xor(v[q], o);
    const unsigned long long a = __shfl_xor(v[3], o), b = __shfl_xor(v[4], o);
    v[3] = a < v[3] ? a : v[3];
    v[4] = b > v[4] ? b : v[4];
  }
  __shared__ unsigned long long part[1024 / OTR_WAVE][6];
  if (lane_id() == 0)
    for (int q = 0; q < 6; ++q) part[threadIdx.x / OTR_WAVE][q] = v[q];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x / OTR_WAVE); ++w) {
      for (int q : {0, 1, 2, 5}) v[q] |= part[w][q];
      v[3] = part[w][3] < v[3] ? part[w][3] : v[3];
      v[4] = part[w][4] > v[4] ? part[w][4] : v[4];
    }
    atomicOr(&r->id_or, v[0]);
    atomicOr(&r->next_or, v[1]);
    atomicOr(&r->file_or, v[2]);
    atomicMin(&r->bmin, v[3]);
    atomicMax(&r->bmax, v[4]);
    atomicOr(&r->foreign, v[5]);
  }
}
static int bit_width(unsigned long long v) { return v ? 64 - __builtin_clzll(v) : 0; }
// sort key of one LSD pass: 0 file, 1 id, 2 next id, 3 speed bin, 4 next id << 3 | bin,
// 5 (bucket - bmin) << 46 | level << 43 | tile << 21 | index (K9 files, 46-bit ids)
__global__ void k_entry_key(const otr_hist_entry* e, const int32_t* perm, int64_t n, int field,
                            unsigned long long bmin, unsigned long long* key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const otr_hist_entry& x = e[perm[i]];
  unsigned long long k;
  switch (field) {
    case 0: k = x.file; break;
    case 1: k = x.id; break;
    case 2: k = x.next_id; break;
    case 3: k = x.speed_bin; break;
    case 4: k = (x.next_id << 3) | (x.speed_bin & 7u); break;
    default:
      k = (((x.file >> 25) - bmin) << 46) | ((x.id & 7ull) << 43) | (((x.id >> 3) & 0x3FFFFFull) << 21) |
          ((x.id >> 25) & 0x1FFFFFull);
  }
  key[i] = k;
}
__global__ void k_gather_entries(const otr_hist_entry* in, const int32_t* idx, int64_t n, otr_hist_entry* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[idx[i]];
}
// run heads over sorted entries: pair = 0 the full key, 1 the (file, id, next_id) pair
__global__ void k_entry_heads(const otr_hist_entry* e, int64_t n, int pair, int64_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool h = i == 0;
  if (!h) {
    const otr_hist_entry &a = e[i - 1], &b = e[i];
    h = a.file != b.file || a.id != b.id || a.next_id != b.next_id || (!pair && a.speed_bin != b.speed_bin);
  }
  head[i] = h ? 1 : 0;
}
__global__ void k_entry_counts(const otr_hist_entry* e, int64_t n, int64_t* c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = e[i].count;
}
// the last entry of every run carries its run's count sum: csum = inclusive scan of counts,
// run r spans [start_r, next start); out[r] = entry at start_r with count = the sum
__global__ void k_entry_reduce(const otr_hist_entry* e, int64_t n, const int64_t* run_start, int64_t n_runs,
                               const int64_t* csum, otr_hist_entry* out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_runs) return;
  const int64_t s = run_start[r], t = r + 1 < n_runs ? run_start[r + 1] : n;
  otr_hist_entry x = e[s];
  const int64_t tot = csum[t - 1] - (s > 0 ? csum[s - 1] : 0);
  x.count = (uint32_t)(tot < 0xFFFFFFFFll ? tot : 0xFFFFFFFFll);
  out[r] = x;
}
// The owner's privacy cull of simple_reporter.py:218-239 on keyed entries.  A pair's run
// length in its file is its total count over the speed bins (one line per tile row); the
// reference sorts a file's lines as strings, so its runs are in the string order of
// (id, next_id) (dec_key), and the loop judges every run alone (kept iff >= privacy)
// except that a trailing run of ONE line is judged together with the run before it (both
// kept iff that run's length + 1 >= privacy).  Per file (files are
// contiguous in the numeric entry order), one block finds the string-last and the
// string-second pair (a top-2 reduction), then every entry gets its keep flag.
struct PairFile {
  unsigned long long s1, n1, s2, n2;  // dec_key of (id, next id): the string-last pair, the one before it
  int64_t t1, t2;                     // their totals
};
__device__ inline bool pf_after(unsigned long long as, unsigned long long an, unsigned long long bs,
                                unsigned long long bn) {
  return as > bs || (as == bs && an > bn);
}
__device__ inline void pf_add(PairFile& T, unsigned long long s, unsigned long long n, int64_t t) {
  if (pf_after(s, n, T.s1, T.n1)) {
    T.s2 = T.s1;
    T.n2 = T.n1;
    T.t2 = T.t1;
    T.s1 = s;
    T.n1 = n;
    T.t1 = t;
  } else if (pf_after(s, n, T.s2, T.n2)) {
    T.s2 = s;
    T.n2 = n;
    T.t2 = t;
  }
}
__global__ void k_pair_file_heads(const otr_hist_entry* e, const int64_t* pair_start, int64_t n_pairs, int64_t* head) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_pairs) head[p] = p == 0 || e[pair_start[p]].file != e[pair_start[p - 1]].file ? 1 : 0;
}
// every pair's string-order keys (dec_key of id and next id) and total, one thread per
// pair: the per-file reduction below then only compares
struct PairKey {
  unsigned long long s, n;
  int64_t t;
};
__global__ void k_pair_keys(const otr_hist_entry* e, const int64_t* pair_start, int64_t n_pairs, int64_t n,
                            const int64_t* csum, PairKey* K) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const int64_t s = pair_start[p], t = p + 1 < n_pairs ? pair_start[p + 1] : n;
  const otr_hist_entry& x = e[s];
  K[p] = PairKey{dec_key(x.id), dec_key(x.next_id), csum[t - 1] - (s > 0 ? csum[s - 1] : 0)};
}
// one 1024-thread block per file over its pairs [ffirst[f], ffirst[f + 1]): the top two pairs
// by (dec_key(id), dec_key(next_id)) and their totals (dec_key > 0: 0 marks "none")
__global__ __launch_bounds__(1024) void k_pair_file_top2(const PairKey* K, int64_t n_pairs, const int64_t* ffirst,
                                                        int64_t nf, PairFile* F) {
  const int64_t f = blockIdx.x;
  const int64_t p0 = ffirst[f], p1 = f + 1 < nf ? ffirst[f + 1] : n_pairs;
  PairFile T{0ull, 0ull, 0ull, 0ull, 0, 0};
  for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const PairKey k = K[p];
    pf_add(T, k.s, k.n, k.t);
  }
  __shared__ PairFile sh[1024];
  sh[threadIdx.x] = T;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      const PairFile U = sh[threadIdx.x + w];
      if (U.s1) pf_add(T, U.s1, U.n1, U.t1);
      if (U.s2) pf_add(T, U.s2, U.n2, U.t2);
      sh[threadIdx.x] = T;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) F[f] = T;
}
__global__ void k_entry_keep(const int64_t* pair_pos, int64_t n, const PairKey* K, const int64_t* fidx,
                             const PairFile* F, int32_t privacy, int64_t* keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t p = pair_pos[i] - 1;
  const PairKey pk = K[p];
  bool k = pk.t >= (int64_t)privacy;
  const PairFile& f = F[fidx[p] - 1];
  if (f.s2 != 0ull && f.t1 == 1) {  // the file's string-last run is one line: judged with the run before it
    if ((pk.s == f.s1 && pk.n == f.n1) || (pk.s == f.s2 && pk.n == f.n2)) k = f.t2 + 1 >= (int64_t)privacy;
  }
  keep[i] = k ? 1 : 0;
}

int Matcher::copy_out(void* dst, const void* src, size_t bytes, int dst_memory, std::string* err) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, dst_memory == OTR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                        stream));
  HIPCHK(hipStreamSynchronize(stream));
  return OTR_OK;
}

int Matcher::hist_reduce(const void* in, int64_t n, int memory, int rows_in, int privacy, const otr_hist_entry** out,
                         int64_t* n_out, std::string* err) {
  try {
    return hist_reduce_impl(in, n, memory, rows_in, privacy, out, n_out, err);
  } catch (const DeviceOom& o) {
    return oom_error(stream, o, err);
  }
}

int Matcher::hist_reduce_impl(const void* in, int64_t n, int memory, int rows_in, int privacy, const otr_hist_entry** out,
                         int64_t* n_out, std::string* err) {
  GraphState& gs = graph_state();
  HIPCHK(hipSetDevice(gs.device));
  if (!stream) HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  *out = nullptr;
  *n_out = 0;
  if (n <= 0) return OTR_OK;
  if (n >= (int64_t)INT32_MAX) {
    if (err) *err = "too many histogram entries for one call";
    return OTR_BAD_REQUEST;
  }
  auto fail = [&](const char* what) {
    if (err) *err = what;
    return OTR_DEVICE_ERROR;
  };
  otr_hist_entry* e_in = need<otr_hist_entry>(S_HE_IN, n);
  otr_hist_entry* e_sorted = need<otr_hist_entry>(S_HE_SORTED, n);
  otr_hist_entry* e_red = need<otr_hist_entry>(S_HE_RED, n);
  otr_hist_entry* e_out = need<otr_hist_entry>(S_HE_OUT, n);
  int32_t* perm_a = need<int32_t>(S_IDX_A, n);
  int32_t* perm_b = need<int32_t>(S_IDX_B, n);
  unsigned long long* key_a = need<unsigned long long>(S_KEY_A, n);
  unsigned long long* key_b = need<unsigned long long>(S_KEY_B, n);
  int64_t* head = need<int64_t>(S_FILE_HEAD, n);
  int64_t* pos = need<int64_t>(S_POS_SCAN, n);
  int64_t* rstart = need<int64_t>(S_FILE_START, n);
  int64_t* csum = need<int64_t>(S_KEEP, n);
  if (!e_in || !e_sorted || !e_red || !e_out || !perm_a || !perm_b || !key_a || !key_b || !head || !pos || !rstart ||
      !csum)
    return fail("device allocation failed (histogram)");
  const hipMemcpyKind kind = memory == OTR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (rows_in) {
    otr_tile_row* rows = need<otr_tile_row>(S_ROWS_IN, n);
    if (!rows) return fail("device allocation failed (histogram)");
    HIPCHK(hipMemcpyAsync(rows, in, sizeof(otr_tile_row) * n, kind, stream));
    k_rows_to_entries<<<grid_for(n, 256), 256, 0, stream>>>(rows, n, e_in);
  } else {
    HIPCHK(hipMemcpyAsync(e_in, in, sizeof(otr_hist_entry) * n, kind, stream));
  }
  const int ni = (int)n;
  size_t tb_sort = 0, tb_scan = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, key_a, key_b, perm_a, perm_b, ni, 0, 64, stream));
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan, head, pos, ni, stream));
  void* tmp = need<char>(S_SORT_TMP, std::max(tb_sort, tb_scan));
  if (!tmp) return fail("device allocation failed (histogram)");
  // LSD over (file, id, next_id, speed_bin), stable passes over a permutation, each only
  // as wide as the keys' range: typically two passes of ~49 bits (next id and bin) and
  // ~47 bits (hour offset and the id in file order), instead of 3 + 3 x 64 bits
  EntryRange* rng = need<EntryRange>(S_HE_RANGE, 1);
  if (!rng) return fail("device allocation failed (histogram)");
  EntryRange hr{0ull, 0ull, 0ull, ~0ull, 0ull, 0ull};
  HIPCHK(hipMemcpyAsync(rng, &hr, sizeof(hr), hipMemcpyHostToDevice, stream));
  k_entry_range<<<(unsigned)std::min<int64_t>(kRangeBlocks, (n + 1023) / 1024), 1024, 0, stream>>>(e_in, n, rng);
  HIPCHK(hipMemcpyAsync(&hr, rng, sizeof(hr), hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  std::vector<std::pair<int, int>> passes;  // (field, end bit), least significant first
  const int wn = bit_width(hr.next_or), wi = bit_width(hr.id_or), ws = bit_width(hr.bmax - hr.bmin);
  if (wn + 3 <= 64) passes.push_back({4, wn + 3});
  else passes.insert(passes.end(), {{3, 3}, {2, wn}});
  if (!hr.foreign && wi <= 46 && ws + 46 <= 64) passes.push_back({5, std::max(46 + ws, 1)});
  else passes.insert(passes.end(), {{1, std::max(wi, 1)}, {0, std::max(bit_width(hr.file_or), 1)}});
  k_iota_i32<<<grid_for(n, 256), 256, 0, stream>>>(perm_a, n);
  for (const auto& ps : passes) {
    k_entry_key<<<grid_for(n, 256), 256, 0, stream>>>(e_in, perm_a, n, ps.first, hr.bmin, key_a);
    size_t tb = tb_sort;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key_a, key_b, perm_a, perm_b, ni, 0, ps.second, stream));
    std::swap(perm_a, perm_b);
  }
  k_gather_entries<<<grid_for(n, 256), 256, 0, stream>>>(e_in, perm_a, n, e_sorted);
  // runs of equal keys -> one entry each, counts summed
  k_entry_heads<<<grid_for(n, 256), 256, 0, stream>>>(e_sorted, n, 0, head);
  size_t tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, pos, ni, stream));
  k_scatter_index<<<grid_for(n, 256), 256, 0, stream>>>(head, pos, n, rstart);
  k_entry_counts<<<grid_for(n, 256), 256, 0, stream>>>(e_sorted, n, head);  // head reused: counts
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, csum, ni, stream));
  int64_t nr = 0;
  HIPCHK(hipMemcpyAsync(&nr, pos + (n - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (nr < 1 || nr > n) return fail("histogram run split failed");
  k_entry_reduce<<<grid_for(nr, 256), 256, 0, stream>>>(e_sorted, n, rstart, nr, csum, e_red);
  otr_hist_entry* result = e_red;
  int64_t nres = nr;
  if (privacy > 1) {
    // pairs over the reduced entries: heads, totals, keep flags, compaction
    const int nri = (int)nr;
    k_entry_heads<<<grid_for(nr, 256), 256, 0, stream>>>(e_red, nr, 1, head);
    tb = tb_scan;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, pos, nri, stream));
    k_scatter_index<<<grid_for(nr, 256), 256, 0, stream>>>(head, pos, nr, rstart);
    int64_t np = 0;
    HIPCHK(hipMemcpyAsync(&np, pos + (nr - 1), 8, hipMemcpyDeviceToHost, stream));
    k_entry_counts<<<grid_for(nr, 256), 256, 0, stream>>>(e_red, nr, head);
    tb = tb_scan;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, csum, nri, stream));
    HIPCHK(hipStreamSynchronize(stream));
    // per file: the string-last and string-second pairs (the reference loop's trailing run)
    int64_t* fidx = need<int64_t>(S_HE_FIDX, std::max<int64_t>(np, 1));
    int64_t* fhead = need<int64_t>(S_HE_FHEAD, std::max<int64_t>(np, 1));
    if (!fidx || !fhead) return fail("device allocation failed (histogram)");
    k_pair_file_heads<<<grid_for(np, 256), 256, 0, stream>>>(e_red, rstart, np, fhead);
    tb = tb_scan;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, fhead, fidx, (int)np, stream));
    int64_t nf = 0;
    HIPCHK(hipMemcpyAsync(&nf, fidx + (np - 1), 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    PairFile* pf = need<PairFile>(S_HE_PFILE, std::max<int64_t>(nf, 1));
    int64_t* ffirst = need<int64_t>(S_HE_FFIRST, std::max<int64_t>(nf, 1));
    if (!pf || !ffirst) return fail("device allocation failed (histogram)");
    PairKey* pkey = need<PairKey>(S_HE_PKEY, std::max<int64_t>(np, 1));
    if (!pkey) return fail("device allocation failed (histogram)");
    k_scatter_index<<<grid_for(np, 256), 256, 0, stream>>>(fhead, fidx, np, ffirst);
    k_pair_keys<<<grid_for(np, 256), 256, 0, stream>>>(e_red, rstart, np, nr, csum, pkey);
    k_pair_file_top2<<<(unsigned)nf, 1024, 0, stream>>>(pkey, np, ffirst, nf, pf);
    int64_t* keep = head;  // counts no longer needed
    k_entry_keep<<<grid_for(nr, 256), 256, 0, stream>>>(pos, nr, pkey, fidx, pf, privacy, keep);
    int64_t* kpos = rstart;  // pair starts no longer needed after k_entry_keep
    tb = tb_scan;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, keep, kpos, nri, stream));
    k_scatter_flagged<otr_hist_entry><<<grid_for(nr, 256), 256, 0, stream>>>(e_red, keep, kpos, nr, e_out);
    HIPCHK(hipMemcpyAsync(&nres, kpos + (nr - 1), 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    result = e_out;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(stream));
  *out = result;
  *n_out = nres;
  return OTR_OK;
}

// ---- K11 ingest (include/otr.h otr_ingest) ----------------------------------------------
int Matcher::ingest(const char* text, int64_t len, int memory, const otr_ingest_format* fmt, otr_ingest_result* out,
                    std::string* err) {
  try {
    return ingest_impl(text, len, memory, fmt, out, err);
  } catch (const DeviceOom& o) {
    return oom_error(stream, o, err);
  }
}

int Matcher::ingest_impl(const char* text, int64_t len, int memory, const otr_ingest_format* fmt, otr_ingest_result* out,
                    std::string* err) {
  GraphState& gs = graph_state();
  HIPCHK(hipSetDevice(gs.device));
  if (!stream) HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  memset(out, 0, sizeof(*out));
  out->bad_line = -1;
  if (fmt->rules < OTR_INGEST_SHARD || fmt->rules > OTR_INGEST_JAVA_SV || fmt->mode < 0 || fmt->mode > 2 ||
      fmt->inactivity < 0 || (fmt->rules != OTR_INGEST_SHARD && (fmt->separator < 1 || fmt->separator > 255))) {
    if (err) *err = "bad ingest format";
    return OTR_BAD_REQUEST;
  }
  for (int k : {fmt->uuid_index, fmt->time_index, fmt->lat_index, fmt->lon_index, fmt->accuracy_index})
    if (fmt->rules != OTR_INGEST_SHARD && (k < 0 || k > 4096)) {
      if (err) *err = "bad ingest field index";
      return OTR_BAD_REQUEST;
    }
  out->batch.memory = OTR_MEM_DEVICE;
  if (len <= 0) return OTR_OK;
  if (len >= ((int64_t)1 << 40)) {
    if (err) *err = "ingest text too large";
    return OTR_BAD_REQUEST;
  }
  auto fail = [&](const char* what) {
    if (err) *err = what;
    return OTR_DEVICE_ERROR;
  };
  // text in HBM, zero-padded to whole 16-byte chunks
  const int64_t n_chunks = (len + 15) / 16;
  uint8_t* d_text = need<uint8_t>(S_IN_TEXT, 16 * n_chunks);
  int64_t* cnt = need<int64_t>(S_IN_CNT, n_chunks);
  int64_t* cscan = need<int64_t>(S_IN_CSCAN, n_chunks);
  unsigned long long* bad = need<unsigned long long>(S_IN_BAD, 1);
  if (!d_text || !cnt || !cscan || !bad) return fail("device allocation failed (ingest)");
  HIPCHK(hipMemsetAsync(d_text + 16 * (n_chunks - 1), 0, 16, stream));
  HIPCHK(hipMemcpyAsync(d_text, text, len, memory == OTR_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                        stream));
  HIPCHK(hipMemsetAsync(bad, 0xFF, 8, stream));
  if (!ev_init) {
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    ev_init = true;
  }
  HIPCHK(hipEventRecord(ev[20], stream));
  size_t tb_scan = 0;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan, cnt, cscan, (int)std::min<int64_t>(n_chunks, INT32_MAX),
                                          stream));
  if (n_chunks >= INT32_MAX) return fail("ingest text too large");
  void* tmp = need<char>(S_IN_TMP, tb_scan);
  if (!tmp) return fail("device allocation failed (ingest)");
  k_nl_count<<<grid_for(n_chunks, 256), 256, 0, stream>>>(reinterpret_cast<const uint4*>(d_text), n_chunks, cnt);
  size_t tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, cnt, cscan, (int)n_chunks, stream));
  int64_t n_nl = 0;
  uint8_t last = 0;
  HIPCHK(hipMemcpyAsync(&n_nl, cscan + (n_chunks - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&last, d_text + (len - 1), 1, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  // Python's file iteration: a final fragment without '\n' is a line too
  const int64_t n_lines = n_nl + (last != '\n' ? 1 : 0);
  out->n_lines = n_lines;
  if (n_lines >= INT32_MAX) {
    if (err) *err = "too many lines for one ingest";
    return OTR_BAD_REQUEST;
  }
  const int64_t nL = std::max<int64_t>(n_lines, 1);
  int64_t* nl = need<int64_t>(S_IN_NL, std::max<int64_t>(n_nl, 1));
  IngestLines L{};
  L.text = d_text;
  L.len = len;
  L.nl = nl;
  L.n_nl = n_nl;
  L.n_lines = n_lines;
  L.hash = need<uint64_t>(S_IN_HASH, nL);
  L.uoff = need<int64_t>(S_IN_UOFF, nL);
  L.ulen = need<int32_t>(S_IN_ULEN, nL);
  L.time = need<int64_t>(S_IN_TIME, nL);
  L.lat = need<double>(S_IN_LAT, nL);
  L.lon = need<double>(S_IN_LON, nL);
  L.acc = need<float>(S_IN_ACC, nL);
  L.keep = need<int64_t>(S_IN_KEEP, nL);
  L.bad = bad;
  int64_t* kpos = need<int64_t>(S_IN_KPOS, nL);
  int32_t* kidx = need<int32_t>(S_IN_KIDX, nL);
  if (!nl || !L.hash || !L.uoff || !L.ulen || !L.time || !L.lat || !L.lon || !L.acc || !L.keep || !kpos || !kidx)
    return fail("device allocation failed (ingest)");
  if (n_nl) k_nl_write<<<grid_for(n_chunks, 256), 256, 0, stream>>>(reinterpret_cast<const uint4*>(d_text), n_chunks,
                                                                    cscan, nl);
  IngestFmt f{};
  f.rules = fmt->rules;
  f.sep = fmt->separator;
  f.tfmt = fmt->time_format;
  f.use_bbox = fmt->use_bbox;
  f.idx[0] = fmt->uuid_index;
  f.idx[1] = fmt->time_index;
  f.idx[2] = fmt->lat_index;
  f.idx[3] = fmt->lon_index;
  f.idx[4] = fmt->accuracy_index;
  for (int k = 0; k < 4; ++k) f.bbox[k] = fmt->bbox[k];
  HIPCHK(hipEventRecord(ev[21], stream));
  k_ingest_parse<<<grid_for(n_lines, 256), 256, 0, stream>>>(L, f);
  HIPCHK(hipEventRecord(ev[22], stream));
  unsigned long long hbad = ~0ull;
  HIPCHK(hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (hbad != ~0ull) {
    out->bad_line = (int64_t)(hbad >> 8);
    out->bad_reason = (int32_t)(hbad & 0xFF);
    if (err) *err = "malformed probe line " + std::to_string(out->bad_line);
    return OTR_BAD_REQUEST;
  }
  // kept lines (bbox), in line order
  const int nI = (int)n_lines;
  size_t tb_sort = 0;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan, L.keep, kpos, nI, stream));
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                            (const int32_t*)nullptr, (int32_t*)nullptr, nI, 0, 64, stream));
  tmp = need<char>(S_IN_TMP, std::max(tb_scan, tb_sort));
  if (!tmp) return fail("device allocation failed (ingest)");
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, L.keep, kpos, nI, stream));
  k_scatter_index32<<<grid_for(n_lines, 256), 256, 0, stream>>>(L.keep, kpos, n_lines, kidx);
  int64_t M = 0;
  HIPCHK(hipMemcpyAsync(&M, kpos + (n_lines - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  out->n_kept = M;
  if (M == 0) return OTR_OK;
  const int nM = (int)M;
  uint64_t* key_a = need<uint64_t>(S_IN_KEY_A, M);
  uint64_t* key_b = need<uint64_t>(S_IN_KEY_B, M);
  int32_t* val_a = need<int32_t>(S_IN_VAL_A, M);
  int32_t* val_b = need<int32_t>(S_IN_VAL_B, M);
  int64_t* head = need<int64_t>(S_IN_HEAD, M);
  int64_t* gid = need<int64_t>(S_IN_GID, M);
  int32_t* gfirst = need<int32_t>(S_IN_GFIRST, M);
  uint32_t* gkey = need<uint32_t>(S_IN_GKEY, nL);
  if (!key_a || !key_b || !val_a || !val_b || !head || !gid || !gfirst || !gkey)
    return fail("device allocation failed (ingest)");
  // 1. group by uuid: sort (hash, line) — the stable sort keeps line order within a hash
  k_gather_by<uint64_t><<<grid_for(M, 256), 256, 0, stream>>>(L.hash, kidx, M, key_a);
  tb = tb_sort;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key_a, key_b, kidx, val_b, nM, 0, 64, stream));
  k_group_heads<<<grid_for(M, 256), 256, 0, stream>>>(key_b, val_b, M, L.uoff, L.ulen, d_text, head, bad);
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, gid, nM, stream));
  k_group_first<<<grid_for(M, 256), 256, 0, stream>>>(head, gid, val_b, M, gfirst);
  k_group_key<<<grid_for(M, 256), 256, 0, stream>>>(gid, val_b, M, gfirst, gkey);
  int64_t n_uuid = 0;
  HIPCHK(hipMemcpyAsync(&n_uuid, gid + (M - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, stream));
  // 2. final order (first appearance of the uuid, time, line): stable LSD passes
  int64_t* tkey_a = reinterpret_cast<int64_t*>(key_a);
  int64_t* tkey_b = reinterpret_cast<int64_t*>(key_b);
  k_gather_by<int64_t><<<grid_for(M, 256), 256, 0, stream>>>(L.time, kidx, M, tkey_a);
  tb = tb_sort;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, tkey_a, tkey_b, kidx, val_a, nM, 0, 64, stream));
  uint32_t* gk_a = reinterpret_cast<uint32_t*>(key_a);
  uint32_t* gk_b = reinterpret_cast<uint32_t*>(key_b);
  k_gather_by<uint32_t><<<grid_for(M, 256), 256, 0, stream>>>(gkey, val_a, M, gk_a);
  int end_bit = 1;
  while (end_bit < 32 && ((int64_t)1 << end_bit) < n_lines) ++end_bit;
  tb = tb_sort;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, gk_a, gk_b, val_a, val_b, nM, 0, end_bit, stream));
  const int32_t* perm = val_b;
  // 3. windows
  k_win_heads<<<grid_for(M, 256), 256, 0, stream>>>(perm, M, gkey, L.time, fmt->inactivity, head);
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, head, gid, nM, stream));  // gid: window ids now
  int64_t n_win = 0;
  HIPCHK(hipMemcpyAsync(&n_win, gid + (M - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  if (hbad != ~0ull) {
    out->bad_line = (int64_t)(hbad >> 8);
    out->bad_reason = (int32_t)(hbad & 0xFF);
    if (err) *err = "uuid hash collision at line " + std::to_string(out->bad_line);
    return OTR_BAD_REQUEST;
  }
  out->n_uuids = (int32_t)n_uuid;
  int64_t* ws = need<int64_t>(S_IN_WS, n_win);
  int64_t* klen = need<int64_t>(S_IN_KLEN, n_win);
  int64_t* kflag = need<int64_t>(S_IN_KFLAG, n_win);
  int64_t* poff = need<int64_t>(S_IN_POFF, n_win);
  int64_t* tpos = need<int64_t>(S_IN_TPOS, n_win);
  if (!ws || !klen || !kflag || !poff || !tpos) return fail("device allocation failed (ingest)");
  k_scatter_index<<<grid_for(M, 256), 256, 0, stream>>>(head, gid, M, ws);
  k_win_len<<<grid_for(n_win, 256), 256, 0, stream>>>(ws, n_win, M, klen, kflag);
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, klen, poff, (int)n_win, stream));
  tb = tb_scan;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, kflag, tpos, (int)n_win, stream));
  int64_t n_tr = 0, n_pr = 0;
  HIPCHK(hipMemcpyAsync(&n_tr, tpos + (n_win - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipMemcpyAsync(&n_pr, poff + (n_win - 1), 8, hipMemcpyDeviceToHost, stream));
  HIPCHK(hipStreamSynchronize(stream));
  out->n_traces = (int32_t)n_tr;
  out->n_probes = n_pr;
  if (n_tr == 0) return OTR_OK;
  IngestOut o{};
  o.trace_off = need<int64_t>(S_IN_T_OFF, n_tr + 1);
  o.lat = need<double>(S_IN_T_LAT, n_pr);
  o.lon = need<double>(S_IN_T_LON, n_pr);
  o.time = need<int64_t>(S_IN_T_TIME, n_pr);
  o.acc = need<float>(S_IN_T_ACC, n_pr);
  o.mode = need<uint8_t>(S_IN_T_MODE, n_tr);
  o.uoff = need<int64_t>(S_IN_T_UOFF, n_tr);
  o.ulen = need<int32_t>(S_IN_T_ULEN, n_tr);
  if (!o.trace_off || !o.lat || !o.lon || !o.time || !o.acc || !o.mode || !o.uoff || !o.ulen)
    return fail("device allocation failed (ingest)");
  k_win_emit<<<grid_for(M, 256), 256, 0, stream>>>(perm, M, gid, ws, klen, poff, tpos, (int32_t)n_tr, L,
                                                   (uint8_t)fmt->mode, o);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ev[23], stream));
  HIPCHK(hipStreamSynchronize(stream));
  HIPCHK(hipEventElapsedTime(&out->parse_ms, ev[21], ev[22]));
  HIPCHK(hipEventElapsedTime(&out->total_ms, ev[20], ev[23]));
  otr_trace_batch& b = out->batch;
  b.n_traces = (int32_t)n_tr;
  b.memory = OTR_MEM_DEVICE;
  b.trace_offsets = o.trace_off;
  b.lat = o.lat;
  b.lon = o.lon;
  b.time = o.time;
  b.accuracy = o.acc;
  b.mode = o.mode;
  out->d_trace_uuid_off = o.uoff;
  out->d_trace_uuid_len = o.ulen;
  return OTR_OK;
}

}  // namespace otr
