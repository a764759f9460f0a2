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
#include "otr_json.h"
#include "otr_report.h"

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

int mode_index(const std::string& m) {
  if (m == "bicycle") return 1;
  if (m == "pedestrian" || m == "foot") return 2;
  return 0;  // auto and the other motor modes share auto access
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

uint32_t levels_mask(const Value* arr) {
  uint32_t m = 0;
  if (!arr) return 0;
  for (auto& v : arr->arr)
    if (v->kind == Value::Number) {
      int64_t l = v->as_int();
      if (l >= 0 && l < 32) m |= 1u << l;
    }
  return m;
}

int threshold_default(int t) {
  if (t >= 0) return t;
  const char* e = getenv("THRESHOLD_SEC");  // reporter_service.py:55-58
  return (e && *e) ? atoi(e) : 15;
}

struct SingleTrace {
  std::vector<int64_t> off{0, 0};
  std::vector<double> lat, lon;
  std::vector<int64_t> time;
  std::vector<float> acc;
  uint8_t mode = 0;
  bool any_acc = false;
};

// trace JSON (Batch.java:56-65, simple_reporter.py:164) → SoA; options into mp
int load_trace(const Value& tr, SingleTrace* st, otr::ModeParams* mp, std::string* err) {
  const Value* pts = tr.get("trace");
  if (!pts || pts->kind != Value::Array) {
    *err = "trace must be a non zero length array of object each of which must have at least lat, lon and time";
    return OTR_BAD_REQUEST;
  }
  for (auto& p : pts->arr) {
    const Value* la = p->get("lat");
    const Value* lo = p->get("lon");
    const Value* tm = p->get("time");
    if (!la || !lo || !tm || la->kind != Value::Number || lo->kind != Value::Number || tm->kind != Value::Number) {
      *err = "trace must be a non zero length array of object each of which must have at least lat, lon and time";
      return OTR_BAD_REQUEST;
    }
    st->lat.push_back(la->as_double());
    st->lon.push_back(lo->as_double());
    st->time.push_back(tm->is_int ? tm->i : (int64_t)std::floor(tm->num));
    const Value* a = p->get("accuracy");
    if (a && a->kind == Value::Number) {
      st->acc.push_back((float)a->as_double());
      st->any_acc = true;
    } else {
      st->acc.push_back(-1.f);
    }
  }
  st->off[1] = (int64_t)st->lat.size();
  *mp = otr::graph_state().defaults;
  const Value* mo = tr.get("match_options");
  std::string mode = "auto";
  if (mo) {
    const Value* m = mo->get("mode");
    if (m && m->kind == Value::String) mode = m->str;
  }
  st->mode = (uint8_t)mode_index(mode);
  otr::MatchParams& P = mp->m[st->mode];
  apply_options(&P, mo);
  otr::finalize_params(&P);
  return OTR_OK;
}

void put_segments(std::string& o, const otr_batch_result& r) {
  o += "[";
  for (int64_t k = 0; k < r.n_seg; ++k) {
    if (k) o += ",";
    o += "{";
    if (r.seg_id[k] != OTR_NO_ID) o += "\"segment_id\":" + std::to_string((unsigned long long)r.seg_id[k]) + ",";
    o += "\"way_ids\":[";
    for (int64_t w = r.seg_way_off[k]; w < r.seg_way_off[k + 1]; ++w) {
      if (w != r.seg_way_off[k]) o += ",";
      o += std::to_string(r.seg_way[w]);
    }
    o += "],\"start_time\":";
    if (r.seg_start[k] == -1.0) o += "-1"; else otrjson::put_double(o, r.seg_start[k]);
    o += ",\"end_time\":";
    if (r.seg_end[k] == -1.0) o += "-1"; else otrjson::put_double(o, r.seg_end[k]);
    o += ",\"queue_length\":" + std::to_string(r.seg_queue[k]);
    o += ",\"length\":" + std::to_string(r.seg_length[k]);
    o += std::string(",\"internal\":") + (r.seg_internal[k] ? "true" : "false");
    o += ",\"begin_shape_index\":" + std::to_string(r.seg_begin_shape[k]);
    o += ",\"end_shape_index\":" + std::to_string(r.seg_end_shape[k]);
    o += "}";
  }
  o += "]";
}

void put_stats(std::string& o, const int32_t* c, const double* len, const int32_t* len_set) {
  auto L = [&](int i) {
    if (len_set[i]) otrjson::put_double(o, len[i]);
    else o += "0";
  };
  o += "\"stats\":{\"successful_matches\":{\"count\":" + std::to_string(c[0]) + ",\"length\":";
  L(0);
  o += "},\"unreported_matches\":{\"count\":" + std::to_string(c[1]) + ",\"length\":";
  L(1);
  o += "},\"match_errors\":{\"discontinuities\":" + std::to_string(c[2]) + ",\"invalid_speeds\":" +
       std::to_string(c[3]) + ",\"invalid_times\":" + std::to_string(c[4]) + "},\"unassociated_segments\":" +
       std::to_string(c[5]) + "}";
}

void put_reports(std::string& o, int64_t n, const unsigned long long* id, const unsigned long long* nx,
                 const double* t0, const double* t1, const int32_t* len, const int32_t* q) {
  o += "\"datastore\":{\"mode\":\"auto\",\"reports\":[";
  for (int64_t k = 0; k < n; ++k) {
    if (k) o += ",";
    o += "{\"id\":" + std::to_string(id[k]) + ",\"t0\":";
    otrjson::put_double(o, t0[k]);
    o += ",\"t1\":";
    otrjson::put_double(o, t1[k]);
    o += ",\"length\":" + std::to_string(len[k]) + ",\"queue_length\":" + std::to_string(q[k]);
    if (nx[k] != OTR_NO_ID) o += ",\"next_id\":" + std::to_string(nx[k]);
    o += "}";
  }
  o += "]}";
}

int run_single(otr_matcher* m, const Value& tr, uint32_t rl, uint32_t tl, int threshold, otr_batch_result* res,
               std::string* err) {
  SingleTrace st;
  otr::ModeParams mp;
  int rc = load_trace(tr, &st, &mp, err);
  if (rc) return rc;
  otr_trace_batch b{};
  b.n_traces = 1;
  b.memory = OTR_MEM_HOST;
  b.trace_offsets = st.off.data();
  b.lat = st.lat.data();
  b.lon = st.lon.data();
  b.time = st.time.data();
  b.accuracy = st.any_acc ? st.acc.data() : nullptr;
  b.mode = &st.mode;
  b.report_levels = rl;
  b.transition_levels = tl;
  b.threshold_sec = threshold;
  b.quantisation = 3600;
  b.flags = OTR_BATCH_COPY_OUT;
  if (st.lat.empty()) {
    memset(res, 0, sizeof(*res));
    return OTR_OK;
  }
  rc = m->m.run(&b, mp, res, err);
  if (rc == OTR_OK && res->status != OTR_OK) {
    *err = "route search exceeded the device table";
    return OTR_MATCH_ERROR;
  }
  return rc;
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
  std::string perr;
  otrjson::Parser ps(json, len);
  otrjson::Ptr tr = ps.parse(&perr);
  if (!tr || tr->kind != Value::Object) return fail(OTR_MATCH_ERROR, perr, out, out_len);
  otr_batch_result res;
  std::string err;
  int rc = run_single(m, *tr, 0, 0, 15, &res, &err);
  if (rc != OTR_OK) return fail(rc == OTR_BAD_REQUEST ? OTR_MATCH_ERROR : rc, err, out, out_len);
  std::string o = "{\"segments\":";
  put_segments(o, res);
  o += "}";
  dup_out(o, out, out_len);
  return OTR_OK;
}

// POST /report: Batch.java:68 → reporter_service.py handle_request 209-245
int otr_report(otr_matcher* m, const char* json, size_t len, int threshold_sec, char** out, size_t* out_len) {
  std::string perr;
  if (!json || len == 0) return fail(OTR_BAD_REQUEST, "No json provided", out, out_len);
  otrjson::Parser ps(json, len);
  otrjson::Ptr tr = ps.parse(&perr);
  if (!tr || tr->kind != Value::Object) return fail(OTR_BAD_REQUEST, perr, out, out_len);
  const Value* uuid = tr->get("uuid");  // :217-219
  if (!uuid || uuid->kind == Value::Null) return fail(OTR_BAD_REQUEST, "uuid is required", out, out_len);
  const Value* pts = tr->get("trace");  // :222-225
  if (!pts || pts->kind != Value::Array || pts->arr.size() < 2)
    return fail(OTR_BAD_REQUEST,
                "trace must be a non zero length array of object each of which must have at least lat, lon and time",
                out, out_len);
  const Value* mo = tr->get("match_options");  // :228-235
  const Value* rl = mo ? mo->get("report_levels") : nullptr;
  if (!rl || rl->kind != Value::Array)
    return fail(OTR_BAD_REQUEST, "match_options must include report_levels array", out, out_len);
  const Value* tl = mo->get("transition_levels");
  if (!tl || tl->kind != Value::Array)
    return fail(OTR_BAD_REQUEST, "match_options must include transition_levels array", out, out_len);
  if (!m) return fail(OTR_MATCH_ERROR, "null matcher", out, out_len);
  const int thr = threshold_default(threshold_sec);
  otr_batch_result res;
  std::string err;
  int rc = run_single(m, *tr, levels_mask(rl), levels_mask(tl), thr, &res, &err);
  if (rc != OTR_OK) return fail(OTR_MATCH_ERROR, err, out, out_len);  // :244-245
  // report() output, reporter_service.py:164-179 (computed on device by k_segments)
  std::string o = "{";
  int32_t length_set[2] = {0, 0};
  const int32_t* c = res.stats;
  // a length is "set" iff the matching counter is non-zero (report() assigns it then)
  length_set[0] = c[0] > 0;
  length_set[1] = c[1] > 0;
  put_stats(o, c, res.stats_len, length_set);
  if (res.shape_used && res.shape_used[0] >= 0) o += ",\"shape_used\":" + std::to_string(res.shape_used[0]);
  o += ",\"segment_matcher\":{\"segments\":";
  put_segments(o, res);
  o += ",\"mode\":\"auto\"},";
  put_reports(o, res.n_rep, (const unsigned long long*)res.rep_id, (const unsigned long long*)res.rep_next,
              res.rep_t0, res.rep_t1, res.rep_length, res.rep_queue);
  o += "}";
  dup_out(o, out, out_len);
  return 200;
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
  put_stats(o, rs.counts, rs.lengths, rs.length_set);
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
  put_reports(o, rs.n_rep, rid.data(), rnx.data(), t0.data(), t1.data(), rl.data(), rq.data());
  o += "}";
  dup_out(o, out, out_len);
  return OTR_OK;
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

}  // extern "C"
