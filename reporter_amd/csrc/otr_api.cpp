// otr_api.cpp — the C-ABI of include/otr.h: configuration, the JSON drop-in entry
// points (valhalla.Configure / SegmentMatcher.Match / POST /report) and the batched
// throughput API.  Each function cites the reference interface it replaces.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/otr.h"
#include "otr_engine.h"
#include "otr_launch.h"
#include "otr_json.h"
#include "otr_format.h"
#include "otr_report.h"
#include "otr_service.h"

using otrjson::Value;

static thread_local std::string g_last_error;

struct otr_matcher {
  otr::Matcher m;
};

namespace {

char* dup_out(const std::string& s, char** out, size_t* out_len) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size());
  p[s.size()] = '\0';
  if (out) *out = p;
  if (out_len) *out_len = s.size();
  return p;
}

int fail(int code, const std::string& msg, char** out, size_t* out_len) {
  g_last_error = msg;
  std::string body = "{\"error\":\"" + msg + "\"}";  // reporter_service.py:214-245 builds it the same way
  if (out) dup_out(body, out, out_len);
  return code;
}

void apply_options(otr::MatchParams* p, const Value* o) {
  if (!o || o->kind != Value::Object) return;
  auto num = [&](const char* k, double* dst) {
    const Value* v = o->get(k);
    if (v && v->kind == Value::Number) *dst = v->as_double();
  };
  num("sigma_z", &p->sigma_z);
  num("beta", &p->beta);
  num("max_route_distance_factor", &p->max_route_distance_factor);
  num("breakage_distance", &p->breakage_distance);
  num("interpolation_distance", &p->interpolation_distance);
  num("search_radius", &p->search_radius);
  num("max_search_radius", &p->max_search_radius);
  num("gps_accuracy", &p->gps_accuracy);
  num("max_route_time_factor", &p->max_route_time_factor);
  num("turn_penalty_factor", &p->turn_penalty_factor);
  const Value* k = o->get("max_candidates");
  if (k && k->kind == Value::Number) p->kmax = (int32_t)k->as_int();
}

int parse_config(const Value& root, otr::Config* cfg, std::string* err) {
  cfg->mp = otr::default_mode_params();
  const Value* meili = root.get("meili");
  if (meili) {
    const Value* def = meili->get("default");
    for (int m = 0; m < OTR_MODES; ++m) apply_options(&cfg->mp.m[m], def);
    const char* names[OTR_MODES] = {"auto", "bicycle", "pedestrian"};
    for (int m = 0; m < OTR_MODES; ++m) apply_options(&cfg->mp.m[m], meili->get(names[m]));
  }
  for (int m = 0; m < OTR_MODES; ++m) otr::finalize_params(&cfg->mp.m[m]);
  const Value* o = root.get("otr");
  if (o) {
    const Value* gp = o->get("graph");
    if (gp && gp->kind == Value::String) cfg->graph_path = gp->str;
    const Value* dv = o->get("device");
    if (dv && dv->kind == Value::Number) cfg->device = (int)dv->as_int();
    const Value* dl = o->get("delta");
    if (dl && dl->kind == Value::Number) cfg->mp.delta = dl->as_double();
    // per-mode route speeds and queue thresholds: a number for
    // every mode or {"auto": .., "bicycle": .., "pedestrian": ..}
    const char* names[OTR_MODES] = {"auto", "bicycle", "pedestrian"};
    auto per_mode = [&](const char* key, double otr::MatchParams::*f) {
      const Value* v = o->get(key);
      if (!v) return;
      for (int m = 0; m < OTR_MODES; ++m) {
        const Value* x = v->kind == Value::Object ? v->get(names[m]) : v;
        if (x && x->kind == Value::Number) cfg->mp.m[m].*f = x->as_double();
      }
    };
    per_mode("speed_kph", &otr::MatchParams::speed_kph);
    per_mode("queue_kph", &otr::MatchParams::queue_kph);
  }
  if (cfg->graph_path.empty()) {
    const Value* mj = root.get("mjolnir");
    const Value* te = mj ? mj->get("tile_extract") : nullptr;
    if (te && te->kind == Value::String) cfg->graph_path = te->str;
  }
  if (const char* env = getenv("OTR_DEVICE")) cfg->device = atoi(env);
  if (cfg->graph_path.empty()) {
    *err = "config has no otr.graph (flattened graph file)";
    return OTR_BAD_REQUEST;
  }
  return OTR_OK;
}

int threshold_default(int t) {
  if (t >= 0) return t;
  const char* e = getenv("THRESHOLD_SEC");  // reporter_service.py:55-58
  return (e && *e) ? atoi(e) : 15;
}

// one request through the shared JSON path (coalesced across threads when enabled)
int run_item(otr_matcher* m, const char* json, size_t len, int threshold, bool report, char** out,
             size_t* out_len) {
  otrsvc::Item it;
  it.body = json;
  it.len = json ? len : 0;
  it.threshold = threshold;
  it.report = report;
  if (report && otrsvc::coalesce_enabled()) otrsvc::coalesce_submit(m->m, &it);
  else otrsvc::process(m->m, {&it});
  if (it.code != 200 && it.code != OTR_OK) {
    const size_t a = it.out.find(":\""), b = it.out.rfind('"');
    g_last_error = (a != std::string::npos && b > a + 2) ? it.out.substr(a + 2, b - a - 2) : it.out;
  }
  dup_out(it.out, out, out_len);
  return it.code;
}

}  // namespace

extern "C" {

const char* otr_last_error(void) { return g_last_error.c_str(); }

void otr_free(char* p) { free(p); }

int otr_configure_json(const char* json, size_t len) {
  std::string perr;
  otrjson::Parser ps(json, len);
  otrjson::Ptr root = ps.parse(&perr);
  if (!root || root->kind != Value::Object) {
    g_last_error = "Problem with config file: " + perr;
    return OTR_BAD_REQUEST;
  }
  otr::Config cfg;
  std::string err;
  int rc = parse_config(*root, &cfg, &err);
  if (rc == OTR_OK) rc = otr::engine_configure(cfg, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// valhalla.Configure(conf_path): reporter_service.py:284, simple_reporter.py:132
int otr_configure(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    g_last_error = std::string("Problem with config file: ") + strerror(errno);
    return OTR_BAD_REQUEST;
  }
  std::string s;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  fclose(f);
  return otr_configure_json(s.data(), s.size());
}

otr_matcher* otr_matcher_new(void) { return new otr_matcher(); }

void otr_matcher_free(otr_matcher* m) { delete m; }

void* otr_matcher_stream(otr_matcher* m) { return m ? (void*)m->m.stream : nullptr; }

int otr_device(void) { return otr::graph_state().device; }

int otr_graph_info(int64_t* n_nodes, int64_t* n_edges, int64_t* n_segments) {
  const otr::GraphState& gs = otr::graph_state();
  if (!gs.ready) return OTR_NOT_CONFIGURED;
  if (n_nodes) *n_nodes = (int64_t)gs.n_nodes;
  if (n_edges) *n_edges = (int64_t)gs.n_edges;
  if (n_segments) *n_segments = (int64_t)gs.n_segments;
  return OTR_OK;
}

// SegmentMatcher.Match(json) -> str: reporter_service.py:240, simple_reporter.py:166
int otr_match(otr_matcher* m, const char* json, size_t len, char** out, size_t* out_len) {
  if (!m) return fail(OTR_MATCH_ERROR, "null matcher", out, out_len);
  return run_item(m, json, len, 15, false, out, out_len);
}

// POST /report: Batch.java:68 → reporter_service.py handle_request 209-245
int otr_report(otr_matcher* m, const char* json, size_t len, int threshold_sec, char** out, size_t* out_len) {
  if (!json || len == 0) return fail(OTR_BAD_REQUEST, "No json provided", out, out_len);
  if (!m) return fail(OTR_MATCH_ERROR, "null matcher", out, out_len);
  return run_item(m, json, len, threshold_default(threshold_sec), true, out, out_len);
}

// n POST /report bodies in shared device batches (Batch.java:68 × n)
int otr_report_batch(otr_matcher* m, int32_t n, const char* const* bodies, const size_t* lens, int threshold_sec,
                     int32_t* codes, char** outs, size_t* out_lens) {
  if (!m || n < 0 || (n > 0 && (!bodies || !lens || !codes || !outs))) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  std::vector<otrsvc::Item> items(n);
  std::vector<otrsvc::Item*> ptrs(n);
  const int thr = threshold_default(threshold_sec);
  for (int32_t i = 0; i < n; ++i) {
    items[i].body = bodies[i];
    items[i].len = bodies[i] ? lens[i] : 0;
    items[i].threshold = thr;
    items[i].report = true;
    ptrs[i] = &items[i];
  }
  otrsvc::process(m->m, ptrs);
  // the responses' copies on the host threads (C2: 70 MB of report() bodies per 2,000 traces)
  otrsvc::parallel(n, [&](int i) {
    codes[i] = items[i].code;
    dup_out(items[i].out, &outs[i], out_lens ? &out_lens[i] : nullptr);
    std::string().swap(items[i].out);  // (freed here, in parallel, not at return)
  });
  return OTR_OK;
}

int otr_coalesce(int32_t max_traces, int32_t max_wait_us) { return otrsvc::coalesce_configure(max_traces, max_wait_us); }

int otr_service_stats(otr_service_split* out, int reset) {
  otrsvc::stats(out, reset != 0);
  return OTR_OK;
}

// report() alone: reporter_service.py:79-179 (as simple_reporter.py:168 calls it)
int otr_report_segments(const char* match_json, size_t match_len, const char* trace_json, size_t trace_len,
                        int threshold_sec, const int32_t* report_levels, int n_report_levels,
                        const int32_t* transition_levels, int n_transition_levels, char** out, size_t* out_len) {
  std::string perr;
  otrjson::Parser pm(match_json, match_len);
  otrjson::Ptr mj = pm.parse(&perr);
  if (!mj || mj->kind != Value::Object) return fail(OTR_MATCH_ERROR, perr, out, out_len);
  otrjson::Parser pt(trace_json, trace_len);
  otrjson::Ptr tj = pt.parse(&perr);
  if (!tj || tj->kind != Value::Object) return fail(OTR_MATCH_ERROR, perr, out, out_len);
  const Value* segs = mj->get("segments");
  const Value* pts = tj->get("trace");
  if (!segs || segs->kind != Value::Array || !pts || pts->kind != Value::Array || pts->arr.empty())
    return fail(OTR_MATCH_ERROR, "segments and trace are required", out, out_len);
  const Value* last_t = pts->arr.back()->get("time");
  if (!last_t || last_t->kind != Value::Number) return fail(OTR_MATCH_ERROR, "time", out, out_len);
  const size_t n = segs->arr.size();
  std::vector<unsigned long long> id(n + 1), rid(n + 1), rnx(n + 1);
  std::vector<double> st(n + 1), en(n + 1), t0(n + 1), t1(n + 1);
  std::vector<uint8_t> internal(n + 1), has_len(n + 1);
  std::vector<int32_t> q(n + 1), len(n + 1), bs(n + 1), rl(n + 1), rq(n + 1);
  for (size_t k = 0; k < n; ++k) {
    const Value& s = *segs->arr[k];
    const Value* v = s.get("segment_id");
    id[k] = (v && v->kind == Value::Number) ? (unsigned long long)v->as_int() : OTR_NO_ID;
    v = s.get("start_time");
    st[k] = v ? v->as_double() : 0;
    v = s.get("end_time");
    en[k] = v ? v->as_double() : 0;
    v = s.get("internal");
    internal[k] = v && v->kind == Value::Bool && v->b;
    v = s.get("queue_length");
    q[k] = v ? (int32_t)v->as_int() : 0;
    v = s.get("length");
    has_len[k] = v && v->kind == Value::Number;
    len[k] = has_len[k] ? (int32_t)v->as_int() : 0;
    v = s.get("begin_shape_index");
    bs[k] = v ? (int32_t)v->as_int() : 0;
  }
  uint32_t rmask = 0, tmask = 0;
  for (int i = 0; i < n_report_levels; ++i)
    if (report_levels[i] >= 0 && report_levels[i] < 32) rmask |= 1u << report_levels[i];
  for (int i = 0; i < n_transition_levels; ++i)
    if (transition_levels[i] >= 0 && transition_levels[i] < 32) tmask |= 1u << transition_levels[i];
  otr::ReportStats rs;
  const int64_t end_time = last_t->is_int ? last_t->i : (int64_t)last_t->num;
  otr::report_segments((int32_t)n, id.data(), st.data(), en.data(), internal.data(), q.data(), has_len.data(),
                       len.data(), bs.data(), nullptr, end_time, (double)threshold_default(threshold_sec), rmask,
                       tmask, rid.data(), rnx.data(), t0.data(), t1.data(), rl.data(), rq.data(), nullptr, &rs);
  std::string o = "{";
  otrfmt::put_stats(o, rs.counts, rs.lengths, rs.length_set);
  if (rs.shape_used >= 0) o += ",\"shape_used\":" + std::to_string(rs.shape_used);
  // segment_matcher echoes the match with mode forced to auto (reporter_service.py:96,167)
  Value echo = *mj;
  bool has_mode = false;
  for (auto& kv : echo.obj)
    if (kv.first == "mode") {
      auto mv = std::make_shared<Value>();
      mv->kind = Value::String;
      mv->str = "auto";
      kv.second = mv;
      has_mode = true;
    }
  if (!has_mode) {
    auto mv = std::make_shared<Value>();
    mv->kind = Value::String;
    mv->str = "auto";
    echo.obj.emplace_back("mode", mv);
  }
  o += ",\"segment_matcher\":";
  otrjson::put_value(o, echo);
  o += ",";
  otrfmt::put_reports(o, 0, rs.n_rep, rid.data(), rnx.data(), t0.data(), t1.data(), rl.data(), rq.data());
  o += "}";
  dup_out(o, out, out_len);
  return OTR_OK;
}

// report() on the device over many segment lists (the K7 tail; tests)
int otr_report_lists_device(int32_t n, const int64_t* seg_off, const uint64_t* seg_id, const double* start,
                            const double* end, const uint8_t* internal, const int32_t* queue,
                            const uint8_t* has_length, const int32_t* length, const int32_t* begin_shape,
                            const int64_t* end_time, const double* threshold, const uint32_t* report_levels,
                            const uint32_t* transition_levels, uint64_t* rep_id, uint64_t* rep_next, double* rep_t0,
                            double* rep_t1, int32_t* rep_length, int32_t* rep_queue, int32_t* n_rep,
                            int32_t* shape_used, int32_t* counts, double* lengths, int32_t* length_set) {
  if (n < 0 || (n > 0 && (!seg_off || !end_time || !threshold || !report_levels || !transition_levels || !n_rep ||
                          !shape_used || !counts || !lengths || !length_set))) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  otr::ReportLists h{};
  h.n = n;
  h.seg_off = seg_off;
  h.seg_id = (const unsigned long long*)seg_id;
  h.start = start;
  h.end = end;
  h.internal = internal;
  h.queue = queue;
  h.has_length = has_length;
  h.length = length;
  h.begin_shape = begin_shape;
  h.end_time = end_time;
  h.threshold = threshold;
  h.rl = report_levels;
  h.tl = transition_levels;
  h.rep_id = (unsigned long long*)rep_id;
  h.rep_next = (unsigned long long*)rep_next;
  h.rep_t0 = rep_t0;
  h.rep_t1 = rep_t1;
  h.rep_length = rep_length;
  h.rep_queue = rep_queue;
  h.n_rep = n_rep;
  h.shape_used = shape_used;
  h.counts = counts;
  h.lengths = lengths;
  h.length_set = length_set;
  std::string err;
  const int rc = otr::report_lists_device(h, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// batched throughput API (new)
int otr_match_batch(otr_matcher* m, const otr_trace_batch* in, otr_batch_result* out) {
  if (!m || !in || !out) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  std::string err;
  int rc = m->m.run(in, otr::graph_state().defaults, out, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// simple_reporter.py:211-239 (sort + privacy cull) on device
int otr_tiles_cull(otr_matcher* m, const otr_tile_row* rows, int64_t n, int32_t memory, int32_t privacy,
                   int32_t rules, const otr_tile_row** out, int64_t* n_out) {
  if (!m || !out || !n_out || (n > 0 && !rows)) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  std::string err;
  const int rc = m->m.tiles_cull(rows, n, memory, privacy, rules, out, n_out, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// keyed speed histogram: per-GPU sort-reduce and the owner's merge + privacy cull
int otr_hist_reduce(otr_matcher* m, const void* in, int64_t n, int32_t memory, int32_t rows_in, int32_t privacy,
                    otr_hist_entry* out, int64_t out_cap, int32_t out_memory, int64_t* n_out) {
  if (!m || !n_out || (n > 0 && (!in || !out))) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  std::string err;
  const otr_hist_entry* dev = nullptr;
  int rc = m->m.hist_reduce(in, n, memory, rows_in, privacy, &dev, n_out, &err);
  if (rc == OTR_OK && *n_out > out_cap) {
    err = "otr_hist_reduce: output buffer too small";
    rc = OTR_BAD_REQUEST;
  }
  if (rc == OTR_OK && *n_out > 0)
    rc = m->m.copy_out(out, dev, sizeof(otr_hist_entry) * (size_t)*n_out, out_memory, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// simple_reporter.py:140-160 (shard lines), :99-111 (raw feed), Formatter.java:103-114
int otr_ingest(otr_matcher* m, const char* text, int64_t len, int32_t memory, const otr_ingest_format* fmt,
               otr_ingest_result* out) {
  if (!m || !fmt || !out || (len > 0 && !text)) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  std::string err;
  const int rc = m->m.ingest(text, len, memory, fmt, out, &err);
  if (rc != OTR_OK) g_last_error = err;
  return rc;
}

// simple_reporter.py:188-195: ','.join([id, next, duration, '1', length, queue, start, end,
// source, mode.upper()]) + os.linesep
// Segment.appendToStringBuffer (Segment.java:59-74) for OTR_TILE_RULES_STREAM
int otr_tiles_format(const otr_tile_row* rows, int64_t n, const char* source, const char* mode, int32_t rules,
                     char** out, size_t* out_len) {
  if ((n > 0 && !rows) || !out) {
    g_last_error = "null argument";
    return OTR_BAD_REQUEST;
  }
  const bool stream = rules == OTR_TILE_RULES_STREAM;
  std::string tail = ",";
  tail += source ? source : "";
  tail += ",";
  for (const char* c = mode ? mode : ""; *c; ++c) tail.push_back((*c >= 'a' && *c <= 'z') ? (char)(*c - 32) : *c);
  if (!stream) tail += "\n";
  std::string o;
  o.reserve((size_t)(n > 0 ? n : 0) * (72 + tail.size()));
  for (int64_t k = 0; k < n; ++k) {
    const otr_tile_row& r = rows[k];
    if (stream) o.push_back('\n');
    otrfmt::put_u64(o, r.id);
    o.push_back(',');
    if (!stream || r.next_id != OTR_INVALID_SEGMENT_ID) otrfmt::put_u64(o, r.next_id);
    o.push_back(',');
    otrfmt::put_i64(o, r.duration);
    o += ",1,";
    otrfmt::put_i64(o, r.length);
    o.push_back(',');
    otrfmt::put_i64(o, r.queue_length);
    o.push_back(',');
    otrfmt::put_i64(o, r.start);
    o.push_back(',');
    otrfmt::put_i64(o, r.end);
    o += tail;
  }
  dup_out(o, out, out_len);
  return OTR_OK;
}

}  // extern "C"

extern "C" int64_t otr_max_batch_probes(void) { return otr::kMaxBatchProbes; }

extern "C" uint64_t otr_launch_max_items(int64_t n_states, int64_t n_traces, int32_t states_per_wave) {
  return otr::max_launch_items(n_states, n_traces, states_per_wave == 2 ? 2 : 1);
}
