// otr_service.h — the JSON request path shared by otr_match / otr_report /
// otr_report_batch and the process-wide request coalescer.
//
// The reference serves one trace per HTTP request (reporter_service.py:209-245), one
// valhalla.SegmentMatcher per server thread (:28-29,51-52).  Here every JSON request,
// however it arrives, becomes a trace of a device batch: bodies are scanned on host
// threads straight into SoA, grouped by the options that must be uniform within a
// batch (report/transition levels, threshold, match_options overrides), matched in one
// otr_match_batch per group, and formatted back on host threads.
#pragma once
#include <functional>
#include <string>
#include <vector>

#include "otr_engine.h"

namespace otrsvc {

struct Item {
  const char* body = nullptr;
  size_t len = 0;
  int threshold = 15;   // report() threshold_sec (reporter_service.py:55-58)
  bool report = true;   // true: POST /report body → report() JSON; false: Match() JSON
  int code = 0;         // out: 200 / 400 / 500 (report) or OTR_OK / error (match)
  std::string out;      // out: response body
};

// Runs every item through one or more device batches on matcher m.
void process(otr::Matcher& m, const std::vector<Item*>& items);
// The host split of every process() call so far (otr_service_stats); reset: start over.
void stats(otr_service_split* out, bool reset);
// f(i) for i in [0, n) over the service's host threads
void parallel(int n, const std::function<void(int)>& f);

// Request coalescing across threads (otr_coalesce in include/otr.h).
bool coalesce_enabled();
int coalesce_configure(int max_traces, int max_wait_us);
// Blocks until the item has been processed; runs it on `fallback` when the coalescer
// is not running.
void coalesce_submit(otr::Matcher& fallback, Item* item);

}  // namespace otrsvc
