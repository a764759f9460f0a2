// otr_report.h — report() of reporter_service.py:79-179 and the simple_reporter
// bucketing rules (simple_reporter.py:176-196), as __host__ __device__ code shared
// by the segment-scan kernel (K7/K8) and the host JSON path (otr_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#ifndef OTR_NO_ID_U64
#define OTR_NO_ID_U64 0xFFFFFFFFFFFFFFFFull
#endif

namespace otr {

struct ReportStats {
  int32_t n_rep;
  int32_t shape_used;      // -1 = key absent (reporter_service.py:165 drops 0/None)
  int32_t counts[6];       // successful, unreported, discontinuities, invalid_speeds, invalid_times, unassociated
  double lengths[2];       // successful_length, unreported_length (km, rounded to 3 dp)
  int32_t length_set[2];   // 0: still the Python int 0
};

// Segment arrays are strided by `stride` so the kernel can read SoA slices in place.
// has_length==nullptr means every segment carries a length.
__host__ __device__ inline void report_segments(
    int32_t n, const unsigned long long* seg_id, const double* start, const double* end, const uint8_t* internal,
    const int32_t* queue, const uint8_t* has_length, const int32_t* length, const int32_t* begin_shape,
    const uint32_t* seg_index, int64_t trace_end_time, double threshold, uint32_t report_levels,
    uint32_t transition_levels, unsigned long long* rep_id, unsigned long long* rep_next, double* rep_t0,
    double* rep_t1, int32_t* rep_length, int32_t* rep_queue, uint32_t* rep_seg_index, ReportStats* out) {
  for (int k = 0; k < 6; ++k) out->counts[k] = 0;
  out->lengths[0] = out->lengths[1] = 0.0;
  out->length_set[0] = out->length_set[1] = 0;
  const double end_time = (double)trace_end_time;
  int32_t last_idx = n - 1;  // :85-87
  while (last_idx >= 0 && end_time - start[last_idx] < threshold) last_idx--;
  out->shape_used = -1;      // :90-92, :165
  if (last_idx >= 0 && begin_shape[last_idx] != 0) out->shape_used = begin_shape[last_idx];
  bool prior_valid = false, prior_has_len = false, first_seg = true;
  unsigned long long prior_id = 0;
  double prior_start = 0, prior_end = 0;
  int32_t prior_len = 0, prior_queue = 0, prior_level = -1;
  uint32_t prior_index = 0xFFFFFFFFu;
  int32_t nrep = 0;
  for (int32_t idx = 0; idx <= last_idx; ++idx) {
    const bool has_id = seg_id[idx] != OTR_NO_ID_U64;
    const int lvl = has_id ? (int)(seg_id[idx] & 7ull) : -1;  // :119
    if (idx != 0 && start[idx] == -1.0 && end[idx - 1] == -1.0) out->counts[2]++;  // :115-116
    const bool lvl_trans = lvl >= 0 && ((transition_levels >> lvl) & 1u);
    if (prior_valid && prior_has_len && prior_len > 0 && !internal[idx]) {  // :122
      if (prior_level >= 0 && ((report_levels >> prior_level) & 1u)) {      // :123
        const double t0 = prior_start;
        const double t1 = lvl_trans ? start[idx] : prior_end;                // :125
        const double dt = t1 - t0;                                           // :130
        if (dt <= 0 || isinf(dt) || isnan(dt)) {
          out->counts[4]++;
        } else if (((double)prior_len / dt) * 3.6 > 160) {                   // :133
          out->counts[3]++;
        } else {
          rep_id[nrep] = prior_id;
          rep_next[nrep] = (lvl_trans && has_id) ? seg_id[idx] : OTR_NO_ID_U64;  // :126-127
          rep_t0[nrep] = t0;
          rep_t1[nrep] = t1;
          rep_length[nrep] = prior_len;
          rep_queue[nrep] = prior_queue;
          if (rep_seg_index) rep_seg_index[nrep] = prior_index;
          nrep++;
          out->counts[0]++;
          out->lengths[0] = (double)prior_len / 1000.0;  // round(len*0.001, 3) for integer len
          out->length_set[0] = 1;
        }
      } else {
        out->counts[1]++;
        out->lengths[1] = (double)prior_len / 1000.0;
        out->length_set[1] = 1;
      }
    }
    if (!(internal[idx] && !first_seg)) {  // :145-155
      prior_valid = has_id;
      prior_id = seg_id[idx];
      prior_start = start[idx];
      prior_end = end[idx];
      prior_has_len = has_length ? has_length[idx] != 0 : true;
      prior_len = length[idx];
      prior_level = lvl;
      prior_queue = queue[idx];
      prior_index = seg_index ? seg_index[idx] : 0xFFFFFFFFu;
    }
    first_seg = false;
    if (!has_id && !internal[idx]) out->counts[5]++;  // :161-162
  }
  out->n_rep = nrep;
}

// Python-2 round() to an integer, half away from zero (simple_reporter.py:179)
__host__ __device__ inline int64_t py2_round_int(double v) {
  double f = floor(v);
  double r = v - f;  // exact for |v| < 2^52
  return (int64_t)(r >= 0.5 ? f + 1.0 : f);
}

// floor division of Python 2 ints (simple_reporter.py:176,182-183)
__host__ __device__ inline int64_t py2_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// simple_reporter.py:177 filter
__host__ __device__ inline bool bucket_keep(double t0, double t1, int32_t length, int32_t queue) {
  return t0 > 0 && t1 > 0 && t1 - t0 > .5 && length > 0 && queue >= 0;
}

struct BucketSpan {
  int64_t duration, start, end, min_bucket, max_bucket;
  bool ok;
};

// simple_reporter.py:176,179-187
__host__ __device__ inline BucketSpan bucket_span(double t0, double t1, int64_t first_time, int64_t last_time,
                                                  int64_t q) {
  BucketSpan s;
  const int64_t buckets = py2_div(last_time - first_time, q) + 1;
  s.duration = py2_round_int(t1 - t0);
  s.start = (int64_t)floor(t0);
  s.end = (int64_t)ceil(t1);
  s.min_bucket = py2_div(s.start, q);
  s.max_bucket = py2_div(s.end, q);
  s.ok = (s.max_bucket - s.min_bucket) <= buckets;
  return s;
}

}  // namespace otr
