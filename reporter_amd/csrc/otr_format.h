// otr_format.h — response bodies from a batch result, one trace at a time:
// Match() output {"segments":[...]} (README.md:288-300) and the report() output of
// reporter_service.py:164-179 as json.dumps(separators=(',',':')) writes it (:243).
#pragma once
#include <cstdint>
#include <string>

#include "../../include/otr.h"
#include "otr_request.h"

namespace otrfmt {

inline void put_u64(std::string& o, unsigned long long v) {
  char b[24];
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) o.push_back(b[--n]);
}

inline void put_i64(std::string& o, long long v) {
  if (v < 0) {
    o.push_back('-');
    put_u64(o, (unsigned long long)(-(v + 1)) + 1ull);
  } else {
    put_u64(o, (unsigned long long)v);
  }
}

// segments k0..k1 of a COPY_OUT / COPY_REPORTS result
inline void put_segments(std::string& o, const otr_batch_result& r, int64_t k0, int64_t k1) {
  o += "[";
  for (int64_t k = k0; k < k1; ++k) {
    if (k != k0) o += ",";
    o += "{";
    if (r.seg_id[k] != OTR_NO_ID) {
      o += "\"segment_id\":";
      put_u64(o, (unsigned long long)r.seg_id[k]);
      o += ",";
    }
    o += "\"way_ids\":[";
    for (int64_t w = r.seg_way_off[k]; w < r.seg_way_off[k + 1]; ++w) {
      if (w != r.seg_way_off[k]) o += ",";
      put_u64(o, r.seg_way[w]);
    }
    o += "],\"start_time\":";
    if (r.seg_start[k] == -1.0) o += "-1"; else otrreq::put_repr(o, r.seg_start[k]);
    o += ",\"end_time\":";
    if (r.seg_end[k] == -1.0) o += "-1"; else otrreq::put_repr(o, r.seg_end[k]);
    o += ",\"queue_length\":";
    put_i64(o, r.seg_queue[k]);
    o += ",\"length\":";
    put_i64(o, r.seg_length[k]);
    o += r.seg_internal[k] ? ",\"internal\":true" : ",\"internal\":false";
    o += ",\"begin_shape_index\":";
    put_i64(o, r.seg_begin_shape[k]);
    o += ",\"end_shape_index\":";
    put_i64(o, r.seg_end_shape[k]);
    o += "}";
  }
  o += "]";
}

// report() "stats" (reporter_service.py:164,170-177).  A length that report() never
// assigned is still the Python int 0.
inline void put_stats(std::string& o, const int32_t* c, const double* len, const int32_t* len_set) {
  auto L = [&](int i) {
    if (len_set[i]) otrreq::put_repr(o, len[i]);
    else o += "0";
  };
  o += "\"stats\":{\"successful_matches\":{\"count\":";
  put_i64(o, c[0]);
  o += ",\"length\":";
  L(0);
  o += "},\"unreported_matches\":{\"count\":";
  put_i64(o, c[1]);
  o += ",\"length\":";
  L(1);
  o += "},\"match_errors\":{\"discontinuities\":";
  put_i64(o, c[2]);
  o += ",\"invalid_speeds\":";
  put_i64(o, c[3]);
  o += ",\"invalid_times\":";
  put_i64(o, c[4]);
  o += "},\"unassociated_segments\":";
  put_i64(o, c[5]);
  o += "}";
}

// report() "datastore" (reporter_service.py:96,149-158); mode is always "auto" (:96)
inline void put_reports(std::string& o, int64_t k0, int64_t k1, const unsigned long long* id,
                        const unsigned long long* nx, const double* t0, const double* t1, const int32_t* len,
                        const int32_t* q) {
  o += "\"datastore\":{\"mode\":\"auto\",\"reports\":[";
  for (int64_t k = k0; k < k1; ++k) {
    if (k != k0) o += ",";
    o += "{\"id\":";
    put_u64(o, id[k]);
    o += ",\"t0\":";
    otrreq::put_repr(o, t0[k]);
    o += ",\"t1\":";
    otrreq::put_repr(o, t1[k]);
    o += ",\"length\":";
    put_i64(o, len[k]);
    o += ",\"queue_length\":";
    put_i64(o, q[k]);
    if (nx[k] != OTR_NO_ID) {
      o += ",\"next_id\":";
      put_u64(o, nx[k]);
    }
    o += "}";
  }
  o += "]}";
}

// Match() body of trace t
inline void match_body(std::string& o, const otr_batch_result& r, int t) {
  o += "{\"segments\":";
  put_segments(o, r, r.trace_seg_off[t], r.trace_seg_off[t + 1]);
  o += "}";
}

// report() body of trace t (reporter_service.py:164-179, computed on device by k_segments)
inline void report_body(std::string& o, const otr_batch_result& r, int t) {
  const int32_t* c = r.stats + 7 * (size_t)t;
  // a length is "set" iff its counter is non-zero (report() assigns it then)
  const int32_t length_set[2] = {c[0] > 0, c[1] > 0};
  o += "{";
  put_stats(o, c, r.stats_len + 2 * (size_t)t, length_set);
  if (r.shape_used && r.shape_used[t] >= 0) {
    o += ",\"shape_used\":";
    put_i64(o, r.shape_used[t]);
  }
  o += ",\"segment_matcher\":{\"segments\":";
  put_segments(o, r, r.trace_seg_off[t], r.trace_seg_off[t + 1]);
  o += ",\"mode\":\"auto\"},";
  put_reports(o, r.trace_rep_off[t], r.trace_rep_off[t + 1], (const unsigned long long*)r.rep_id,
              (const unsigned long long*)r.rep_next, r.rep_t0, r.rep_t1, r.rep_length, r.rep_queue);
  o += "}";
}

}  // namespace otrfmt
