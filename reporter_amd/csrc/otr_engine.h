// otr_engine.h — host-side engine: HBM graph replica, per-matcher workspace and the
// batched pipeline (K0..K8).  Internal C++ interface between otr_engine.hip and the
// C-ABI in otr_api.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/otr.h"
#include "otr_device.h"

namespace otr {

struct Config {
  ModeParams mp;
  std::string graph_path;
  int device = 0;
};

ModeParams default_mode_params();
void finalize_params(MatchParams* p);
const char* check_params(const MatchParams& p);  // nullptr when the engine can honour p

// The configured graph, resident in HBM (one replica per process/GPU).  A reconfigure
// builds the new replica aside and swaps it in under the exclusive lock; batches hold
// the shared lock for their whole run, so no kernel ever sees a freed array.
struct GraphState {
  bool ready = false;
  int device = 0;
  DevGraph dg{};
  ModeParams defaults{};
  std::vector<void*> allocs;
  uint64_t n_nodes = 0, n_edges = 0, n_segments = 0;
  // host copy of the few arrays the JSON path needs
  std::vector<unsigned long long> seg_id;
  std::shared_mutex mu;
};

GraphState& graph_state();
int engine_configure(const Config& cfg, std::string* err);

struct ReportLists {
  int32_t n;
  const int64_t* seg_off;
  const unsigned long long* seg_id;
  const double *start, *end;
  const uint8_t* internal;
  const int32_t* queue;
  const uint8_t* has_length;
  const int32_t *length, *begin_shape;
  const int64_t* end_time;
  const double* threshold;
  const uint32_t *rl, *tl;
  unsigned long long *rep_id, *rep_next;
  double *rep_t0, *rep_t1;
  int32_t *rep_length, *rep_queue, *n_rep, *shape_used, *counts;
  double* lengths;
  int32_t* length_set;
};

int report_lists_device(const ReportLists& h, std::string* err);

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// one tier of global-memory search slabs (otr_general.h), owned by a matcher
struct GSlab {
  uint32_t* key = nullptr;
  unsigned long long* lab = nullptr;
  uint32_t* qmark = nullptr;
  uint32_t* fr = nullptr;
  uint32_t* touched = nullptr;
};

// turn cost table (mm) of a turn_penalty_factor: factor * exp(-deg / 45) for deg 0..180
// (oracle orc_turn_table: the same operations)
void turn_table(double factor, int32_t* tab181);

struct Matcher {
  hipStream_t stream = nullptr;
  std::vector<DevBuf> bufs;
  GSlab gslab[2];
  std::vector<int32_t> h_turn;
  // host result storage (OTR_BATCH_COPY_OUT)
  std::vector<int64_t> h_trace_state_off, h_state_probe, h_trace_route_off, h_trace_seg_off, h_seg_way_off,
      h_trace_rep_off;
  std::vector<int32_t> h_cand_count, h_winner, h_subpath, h_seg_length, h_seg_queue, h_seg_bshape, h_seg_eshape,
      h_rep_length, h_rep_queue, h_shape_used, h_stats, h_trace_status;
  std::vector<uint32_t> h_cand_edge, h_route_edge, h_seg_way;
  std::vector<double> h_cand_p, h_cand_sqd, h_seg_start, h_seg_end, h_rep_t0, h_rep_t1, h_stats_len;
  std::vector<unsigned long long> h_seg_id, h_rep_id, h_rep_next;
  std::vector<uint8_t> h_seg_internal;
  std::vector<otr_tile_row> h_tile_rows;
  hipEvent_t ev[56];  // 0..19 batch stages, 20..23 ingest, 24..49 route tiers
  bool ev_init = false;

  template <class T>
  T* need(int slot, size_t n);
  // optional workspace (the retry tiers' resume dumps, the spatial sort's copy): taken
  // only while the device keeps a reserve free for the mandatory buffers of later stages,
  // nullptr otherwise (the searches then restart: same results)
  template <class T>
  T* want(int slot, size_t n);
  // frees the optional workspace after the stream drains (a mandatory need() that cannot
  // allocate retries once after it); not while the route stage's kernels hold it
  bool release_optional();
  bool opt_busy = false;
  // entry points: a device allocation failure inside returns OTR_DEVICE_ERROR (no kernel
  // runs on a missing buffer); the *_impl bodies do the work
  int run(const otr_trace_batch* in, const ModeParams& mp, otr_batch_result* out, std::string* err);
  int tiles_cull(const otr_tile_row* rows, int64_t n, int memory, int privacy, int rules, const otr_tile_row** out,
                 int64_t* n_out, std::string* err);
  int hist_reduce(const void* in, int64_t n, int memory, int rows_in, int privacy, const otr_hist_entry** out,
                  int64_t* n_out, std::string* err);
  int run_impl(const otr_trace_batch* in, const ModeParams& mp, otr_batch_result* out, std::string* err);
  int tiles_cull_impl(const otr_tile_row* rows, int64_t n, int memory, int privacy, int rules,
                      const otr_tile_row** out, int64_t* n_out, std::string* err);
  int hist_reduce_impl(const void* in, int64_t n, int memory, int rows_in, int privacy, const otr_hist_entry** out,
                       int64_t* n_out, std::string* err);
  int ingest_impl(const char* text, int64_t len, int memory, const otr_ingest_format* fmt, otr_ingest_result* out,
                  std::string* err);
  int copy_out(void* dst, const void* src, size_t bytes, int dst_memory, std::string* err);
  int ingest(const char* text, int64_t len, int memory, const otr_ingest_format* fmt, otr_ingest_result* out,
             std::string* err);
  ~Matcher();
};

}  // namespace otr
