// loadgen — many caller threads hitting otr_report concurrently, as the Kafka stream
// threads of the Java reporter (BatchingProcessor.java:58-141 → Batch.java:68) or the
// HTTP server threads of reporter_service.py (:28-29,51-52) would, with and without
// the coalescer (otr_coalesce).  Every response is checked byte for byte against the
// one otr_report_batch returns for the same body.
//
//   loadgen <config.json> <bodies.txt (one body per line)> <threads> <coalesce_max> <wait_us>
// Prints one JSON line: {"threads":..,"coalesce":..,"traces_per_s":..,"probes_per_s":..,"seconds":..,
// "identical":.., "split": the host split of the coalesced run (otr_service_stats)}
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/otr.h"

// a crash names its stack on stderr (host code; the tool runs as a child of bench.py)
static void on_fault(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  fprintf(stderr, "loadgen: signal %d\n", sig);
  backtrace_symbols_fd(fr, n, 2);
  _exit(128 + sig);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_fault);
  signal(SIGBUS, on_fault);
  if (argc < 6) {
    fprintf(stderr, "usage: %s config.json bodies.txt threads coalesce_max wait_us\n", argv[0]);
    return 2;
  }
  const int threads = atoi(argv[3]), cmax = atoi(argv[4]), wait_us = atoi(argv[5]);
  if (otr_configure(argv[1]) != OTR_OK) {
    fprintf(stderr, "configure: %s\n", otr_last_error());
    return 1;
  }
  std::vector<std::string> bodies;
  {
    std::ifstream f(argv[2]);
    std::string line;
    while (std::getline(f, line))
      if (!line.empty()) bodies.push_back(line);
  }
  const int n = (int)bodies.size();
  // reference responses: one batch call
  std::vector<const char*> ptrs(n);
  std::vector<size_t> lens(n), olens(n);
  std::vector<int32_t> codes(n);
  std::vector<char*> outs(n);
  for (int i = 0; i < n; ++i) {
    ptrs[i] = bodies[i].data();
    lens[i] = bodies[i].size();
  }
  otr_matcher* m0 = otr_matcher_new();
  fprintf(stderr, "loadgen: %d bodies, reference batch call\n", n);
  otr_report_batch(m0, n, ptrs.data(), lens.data(), -1, codes.data(), outs.data(), olens.data());
  fprintf(stderr, "loadgen: %d threads, coalescer %d / %d us\n", threads, cmax, wait_us);
  std::vector<std::string> want(n);
  for (int i = 0; i < n; ++i) {
    want[i] = std::to_string(codes[i]) + ":" + std::string(outs[i], olens[i]);
    otr_free(outs[i]);
  }
  int64_t probes = 0;  // points of every body ("lat" keys)
  for (const auto& b : bodies)
    for (size_t p = b.find("\"lat\""); p != std::string::npos; p = b.find("\"lat\"", p + 5)) ++probes;
  if (cmax > 0) otr_coalesce(cmax, wait_us);
  otr_service_stats(nullptr, 1);
  std::atomic<int> next{0}, mismatches{0};
  auto worker = [&] {
    otr_matcher* m = otr_matcher_new();
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n) break;
      char* out = nullptr;
      size_t ol = 0;
      const int code = otr_report(m, bodies[i].data(), bodies[i].size(), -1, &out, &ol);
      if (std::to_string(code) + ":" + std::string(out, ol) != want[i]) mismatches.fetch_add(1);
      otr_free(out);
    }
    otr_matcher_free(m);
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k) th.emplace_back(worker);
  for (auto& t : th) t.join();
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (cmax > 0) otr_coalesce(0, 0);
  otr_service_split st{};
  otr_service_stats(&st, 0);
  otr_matcher_free(m0);
  printf("{\"threads\": %d, \"coalesce_max\": %d, \"wait_us\": %d, \"traces\": %d, \"probes\": %lld, "
         "\"seconds\": %.4f, \"traces_per_s\": %.1f, \"probes_per_s\": %.1f, \"identical\": %s, "
         "\"split\": {\"calls\": %lld, \"device_batches\": %lld, \"scan_ms\": %.2f, \"soa_ms\": %.2f, "
         "\"device_ms\": %.2f, \"format_ms\": %.2f, \"total_ms\": %.2f}}\n",
         threads, cmax, wait_us, n, (long long)probes, dt, n / dt, probes / dt,
         mismatches.load() == 0 ? "true" : "false", (long long)st.calls, (long long)st.device_batches,
         1e3 * st.scan_s, 1e3 * st.soa_s, 1e3 * st.device_s, 1e3 * st.format_s, 1e3 * st.total_s);
  return mismatches.load() == 0 ? 0 : 3;
}
