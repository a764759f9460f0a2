// otr_service.cpp — JSON requests → device batches → JSON responses, and the
// cross-thread request coalescer (see otr_service.h).
#include "otr_service.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <cstdio>
#include <thread>

#include "otr_format.h"
#include "otr_request.h"

namespace otrsvc {
namespace {

// OTR_SERVICE_TIMING=1: also print every process() call's host split on stderr
bool service_timing() {
  static const bool on = getenv("OTR_SERVICE_TIMING") != nullptr;
  return on;
}
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// per calling thread: concurrent process() calls (coalescer off) never share them
thread_local double g_t_soa = 0, g_t_run = 0, g_t_fmt = 0;
thread_local int64_t g_batches = 0;
// the process-wide split (otr_service_stats)
std::mutex g_stats_mu;
otr_service_split g_stats{};

int host_threads() {
  static const int n = [] {
    if (const char* e = getenv("OTR_HOST_THREADS")) return std::max(1, atoi(e));
    const int hw = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(hw > 0 ? hw : 1, 16));
  }();
  return n;
}

// f(i) for i in [0, n) over the host threads, in chunks
template <class F>
void parallel_for(int n, F f) {
  const int chunk = 16;
  int nt = std::min(host_threads(), (n + chunk - 1) / chunk);
  if (nt <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<int> next{0};
  auto work = [&] {
    for (;;) {
      const int i0 = next.fetch_add(chunk);
      if (i0 >= n) return;
      const int i1 = std::min(n, i0 + chunk);
      for (int i = i0; i < i1; ++i) f(i);
    }
  };
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (int k = 1; k < nt; ++k) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

void error_body(Item* it, int code, const std::string& msg) {
  it->code = code;
  it->out = "{\"error\":\"" + msg + "\"}";  // reporter_service.py:214-245 builds it the same way
}

// Options that must be uniform within one device batch
std::string group_key(const Item& it, const otrreq::Request& r) {
  std::string k;
  auto put = [&](const void* p, size_t n) { k.append((const char*)p, n); };
  const uint32_t rl = it.report ? r.rl : 0, tl = it.report ? r.tl : 0;
  const int thr = it.report ? it.threshold : 15;
  put(&rl, 4);
  put(&tl, 4);
  put(&thr, 4);
  put(&r.ov_mask, 4);
  if (r.ov_mask) {  // overrides apply to the trace's mode only
    put(&r.mode, 1);
    for (int o = 0; o < otrreq::OV_COUNT; ++o)
      if (r.ov_mask & (1u << o)) put(&r.ov[o], 8);
  }
  return k;
}

otr::ModeParams group_params(const otrreq::Request& r) {
  otr::ModeParams mp = otr::graph_state().defaults;
  if (!r.ov_mask) return mp;
  otr::MatchParams& p = mp.m[r.mode < OTR_MODES ? r.mode : 0];
  double* dst[otrreq::OV_COUNT] = {&p.sigma_z,          &p.beta,          &p.max_route_distance_factor,
                                   &p.breakage_distance, &p.interpolation_distance, &p.search_radius,
                                   &p.max_search_radius, &p.gps_accuracy, nullptr,
                                   &p.max_route_time_factor, &p.turn_penalty_factor};
  for (int o = 0; o < otrreq::OV_COUNT; ++o) {
    if (!(r.ov_mask & (1u << o))) continue;
    if (o == otrreq::OV_MAX_CANDIDATES) p.kmax = (int32_t)(int64_t)r.ov[o];
    else *dst[o] = r.ov[o];
  }
  otr::finalize_params(&p);
  return mp;
}

int64_t max_batch_probes() {
  static const int64_t n = [] {
    const char* e = getenv("OTR_MAX_BATCH_PROBES");
    return e ? std::max<int64_t>(1, atoll(e)) : (int64_t)16 << 20;
  }();
  return n;
}

// One device batch over items idx (all valid, same group), results formatted in place.
void run_group(otr::Matcher& m, const std::vector<Item*>& items, std::vector<otrreq::Request>& req,
               const std::vector<int>& idx) {
  const otrreq::Request& r0 = req[idx[0]];
  const Item& i0 = *items[idx[0]];
  const otr::ModeParams mp = group_params(r0);
  std::vector<int> run;  // items with points
  for (int i : idx) {
    if (req[i].lat.empty()) {
      items[i]->code = i0.report ? 200 : OTR_OK;
      items[i]->out = i0.report ? std::string() : "{\"segments\":[]}";
    } else {
      run.push_back(i);
    }
  }
  size_t a = 0;
  while (a < run.size()) {
    // chunk by probes so one batch's workspace stays bounded
    size_t b = a;
    int64_t np = 0;
    bool any_acc = false;
    while (b < run.size() && (b == a || np + (int64_t)req[run[b]].lat.size() <= max_batch_probes())) {
      np += (int64_t)req[run[b]].lat.size();
      any_acc = any_acc || req[run[b]].any_acc;
      ++b;
    }
    const int T = (int)(b - a);
    const double ta = now_s();
    std::vector<int64_t> off(T + 1, 0);
    for (int t = 0; t < T; ++t) off[t + 1] = off[t] + (int64_t)req[run[a + t]].lat.size();
    std::vector<double> lat(np), lon(np);
    std::vector<int64_t> tm(np);
    std::vector<float> acc(any_acc ? np : 0);
    std::vector<uint8_t> mode(T);
    parallel_for(T, [&](int t) {
      const otrreq::Request& r = req[run[a + t]];
      const size_t n = r.lat.size(), o = (size_t)off[t];
      memcpy(&lat[o], r.lat.data(), 8 * n);
      memcpy(&lon[o], r.lon.data(), 8 * n);
      memcpy(&tm[o], r.time.data(), 8 * n);
      if (any_acc) memcpy(&acc[o], r.acc.data(), 4 * n);
      mode[t] = r.mode;
    });
    otr_trace_batch bt{};
    bt.n_traces = T;
    bt.memory = OTR_MEM_HOST;
    bt.trace_offsets = off.data();
    bt.lat = lat.data();
    bt.lon = lon.data();
    bt.time = tm.data();
    bt.accuracy = any_acc ? acc.data() : nullptr;
    bt.mode = mode.data();
    bt.report_levels = i0.report ? r0.rl : 0;
    bt.transition_levels = i0.report ? r0.tl : 0;
    bt.threshold_sec = i0.report ? i0.threshold : 15;
    bt.quantisation = 3600;
    bt.flags = OTR_BATCH_COPY_REPORTS;
    otr_batch_result res;
    std::string err;
    const double tb = now_s();
    const int rc = m.run(&bt, mp, &res, &err);
    const double tc = now_s();
    parallel_for(T, [&](int t) {
      Item* it = items[run[a + t]];
      if (rc != OTR_OK) {
        error_body(it, it->report ? OTR_MATCH_ERROR : (rc == OTR_BAD_REQUEST ? OTR_MATCH_ERROR : rc), err);
      } else if (res.trace_status && res.trace_status[t] != OTR_OK) {
        error_body(it, OTR_MATCH_ERROR, "route search exceeded the device table");
      } else if (it->report) {
        it->code = 200;
        otrfmt::report_body(it->out, res, t);
      } else {
        it->code = OTR_OK;
        otrfmt::match_body(it->out, res, t);
      }
    });
    g_t_soa += tb - ta;
    g_t_run += tc - tb;
    g_t_fmt += now_s() - tc;
    ++g_batches;
    a = b;
  }
}

}  // namespace

void parallel(int n, const std::function<void(int)>& f) { parallel_for(n, f); }

void stats(otr_service_split* out, bool reset) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  if (out) *out = g_stats;
  if (reset) g_stats = otr_service_split{};
}

void process(otr::Matcher& m, const std::vector<Item*>& items) {
  const int n = (int)items.size();
  if (n == 0) return;
  const double t0 = now_s();
  std::vector<otrreq::Request> req(n);
  const bool configured = otr::graph_state().ready;
  parallel_for(n, [&](int i) {
    Item* it = items[i];
    it->out.clear();
    otrreq::Request& r = req[i];
    if (!it->body || it->len == 0) {
      r.code = it->report ? 400 : OTR_MATCH_ERROR;
      r.err = "No json provided";
    } else {
      otrreq::Scanner sc(it->body, it->len);
      sc.request(&r, !it->report);
    }
    if (r.code == 0 && r.ov_mask && configured) {
      // match_options values the engine cannot honour are refused by name, never ignored
      const otr::ModeParams mp = group_params(r);
      if (const char* bad = otr::check_params(mp.m[r.mode < OTR_MODES ? r.mode : 0])) {
        r.code = 400;
        r.err = std::string("match_options: ") + bad;
      }
    }
    if (r.code) {
      error_body(it, it->report ? r.code : OTR_MATCH_ERROR, r.err);
    } else if (!configured) {
      error_body(it, it->report ? OTR_MATCH_ERROR : OTR_NOT_CONFIGURED, "otr_configure has not been called");
      r.code = it->code;
    }
  });
  const double t1 = now_s();
  g_t_soa = g_t_run = g_t_fmt = 0;
  g_batches = 0;
  std::map<std::string, std::vector<int>> groups;
  for (int i = 0; i < n; ++i)
    if (req[i].code == 0) groups[group_key(*items[i], req[i]) + (items[i]->report ? "R" : "M")].push_back(i);
  for (auto& g : groups) run_group(m, items, req, g.second);
  {
    std::lock_guard<std::mutex> lk(g_stats_mu);
    g_stats.calls += 1;
    g_stats.items += n;
    g_stats.device_batches += g_batches;
    g_stats.scan_s += t1 - t0;
    g_stats.soa_s += g_t_soa;
    g_stats.device_s += g_t_run;
    g_stats.format_s += g_t_fmt;
    g_stats.total_s += now_s() - t0;
  }
  if (service_timing())
    fprintf(stderr, "otr_service: %d items, %zu groups, %d host threads: scan %.1f ms, soa %.1f ms, "
                    "device batch %.1f ms, format %.1f ms, total %.1f ms\n",
            n, groups.size(), host_threads(), 1e3 * (t1 - t0), 1e3 * g_t_soa, 1e3 * g_t_run, 1e3 * g_t_fmt,
            1e3 * (now_s() - t0));
}

// ---------------------------------------------------------------------------------
// Coalescer: callers on many threads (Kafka stream threads, HTTP server threads) hand
// their request to dispatcher threads that run them as shared device batches.  Several
// dispatchers (OTR_COALESCE_DISPATCHERS, default 2), each with its own matcher and HIP
// stream: while one batch's kernels run, the next batch is gathered, scanned and launched
// and the previous one formatted, so small requests (BatchingProcessor.java:26-29: ~10
// points each) do not leave the GPU idle between batches.
namespace {

// a gathering dispatcher stops waiting once no request has arrived for this long
// (OTR_COALESCE_GAP_US, default 100): blocked callers resubmit within microseconds of
// their responses, so a quiet gap means every active caller is queued, and waiting the
// rest of max_wait_us would only idle the GPU
int coalesce_gap_us() {
  static const int n = [] {
    const char* e = getenv("OTR_COALESCE_GAP_US");
    return e ? std::max(0, atoi(e)) : 100;
  }();
  return n;
}

int coalesce_dispatchers() {
  static const int n = [] {
    const char* e = getenv("OTR_COALESCE_DISPATCHERS");
    return e ? std::max(1, std::min(8, atoi(e))) : 2;
  }();
  return n;
}

struct Pending {
  Item* item;
  bool done = false;
};

struct Coalescer {
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<Pending*> q;
  int max_traces = 0, max_wait_us = 0;
  bool running = false, stop = false;
  int active = 0;  // dispatcher threads alive
  std::chrono::steady_clock::time_point last_arrival{};

  void loop() {
    {
      otr::Matcher m;  // (destroyed before this dispatcher reports itself gone: a caller
                       // that stops the coalescer may then tear the process down)
      std::unique_lock<std::mutex> lk(mu);
      run(m, lk);
    }
    std::lock_guard<std::mutex> lk(mu);
    if (--active == 0) running = false;
    cv_done.notify_all();
    cv_work.notify_all();  // (the other dispatchers see the drained queue too)
  }

  void run(otr::Matcher& m, std::unique_lock<std::mutex>& lk) {
    for (;;) {
      cv_work.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) break;  // stop requested and drained
      // gather: until max_traces are queued, max_wait_us after the first, or a quiet gap
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(max_wait_us);
      const auto gap = std::chrono::microseconds(coalesce_gap_us());
      for (;;) {
        const auto until = std::min(deadline, last_arrival + gap);
        if (cv_work.wait_until(lk, until, [&] { return stop || (int)q.size() >= max_traces; })) break;
        const auto now = std::chrono::steady_clock::now();
        if (now >= deadline || now >= last_arrival + gap) break;
      }
      std::vector<Pending*> batch;
      while (!q.empty() && (int)batch.size() < max_traces) {
        batch.push_back(q.front());
        q.pop_front();
      }
      lk.unlock();
      std::vector<Item*> items;
      items.reserve(batch.size());
      for (Pending* p : batch) items.push_back(p->item);
      process(m, items);
      lk.lock();
      for (Pending* p : batch) p->done = true;
      cv_done.notify_all();
      if (!q.empty()) cv_work.notify_one();  // (another dispatcher may be idle)
    }
  }
};

Coalescer& coalescer() {
  static Coalescer* c = new Coalescer();  // never destroyed: the dispatcher may outlive statics
  return *c;
}

}  // namespace

bool coalesce_enabled() {
  Coalescer& c = coalescer();
  std::lock_guard<std::mutex> lk(c.mu);
  return c.running && !c.stop;
}

int coalesce_configure(int max_traces, int max_wait_us) {
  Coalescer& c = coalescer();
  std::unique_lock<std::mutex> lk(c.mu);
  if (max_traces <= 0) {  // stop: drain what is queued, then end the dispatcher
    if (c.running) {
      c.stop = true;
      c.cv_work.notify_all();
      c.cv_done.wait(lk, [&] { return !c.running; });
    }
    c.stop = false;
    return OTR_OK;
  }
  c.max_traces = max_traces;
  c.max_wait_us = max_wait_us < 0 ? 0 : max_wait_us;
  if (!c.running) {
    c.running = true;
    c.active = coalesce_dispatchers();
    for (int k = 0; k < c.active; ++k) std::thread([&c] { c.loop(); }).detach();
  }
  return OTR_OK;
}

void coalesce_submit(otr::Matcher& fallback, Item* item) {
  Coalescer& c = coalescer();
  Pending p{item};
  std::unique_lock<std::mutex> lk(c.mu);
  if (!c.running || c.stop) {
    lk.unlock();
    process(fallback, {item});
    return;
  }
  c.q.push_back(&p);
  c.last_arrival = std::chrono::steady_clock::now();
  if ((int)c.q.size() >= c.max_traces || c.q.size() == 1) c.cv_work.notify_one();
  c.cv_done.wait(lk, [&] { return p.done; });
}

}  // namespace otrsvc
