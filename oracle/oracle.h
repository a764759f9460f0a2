/*
 * oracle.h — CPU restatement of the reference's map-matching hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / the timed CPU
 * baseline.  The product (libotr.so) never links or calls it.
 *
 * What it restates (file:line in /root/reference unless UPSTREAM):
 *   - trace request semantics: reporter_service.py:184-245, simple_reporter.py:136-168
 *   - the matcher, Valhalla meili 2.3.6 (UPSTREAM, NOT present in this container,
 *     PPA pin Dockerfile:7,29-32): candidate search, emission, bounded one-to-many
 *     routing, transition, Viterbi, route construction, OSMLR segment formation
 *     (output schema README.md:269-302).  PARITY WITH MEILI IS UNPINNED: no meili
 *     source, binary, tile or golden output exists here or in the reference's tests
 *     (SURVEY.md §8c).  This file is the written-down algorithm the HIP path must
 *     match bit-exactly; DESIGN.md §3 lists every rule re-derived here.
 *   - report(): reporter_service.py:79-179 (pinned by tests/golden/report_cases.json)
 *   - filter + hour bucketing: simple_reporter.py:176-196 (tests/golden/bucket_cases.json)
 *   - privacy cull: simple_reporter.py:218-239 (tests/golden/cull_cases.json)
 */
#ifndef OTR_ORACLE_H
#define OTR_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_KMAX 64
#define ORC_INVALID_SEGMENT_ID 0x3fffffffffffull /* simple_reporter.py:43 */
#define ORC_NO_ID 0xFFFFFFFFFFFFFFFFull

/* Matching parameters of ONE travel mode (meili.default merged with meili.<mode>, then
 * the request's match_options).  orc_match_batch takes an array of three: auto,
 * bicycle, pedestrian (the trace's mode selects one). */
typedef struct orc_params {
  double sigma_z;                    /* 4.07  Dockerfile:14 */
  double beta;                       /* 3     Dockerfile:15 */
  double max_route_distance_factor;  /* 5     Dockerfile:16 */
  double max_route_time_factor;      /* 2     Dockerfile:17,48 */
  double breakage_distance;          /* 2000  generate_test_trace.py:48 (<= ORC_MAX_BREAKAGE) */
  double interpolation_distance;     /* 10 */
  double search_radius;              /* 50    generate_test_trace.py:51 */
  double max_search_radius;          /* 100 */
  double gps_accuracy;               /* 5 */
  double turn_penalty_factor;        /* per mode: auto 200, bicycle 140, pedestrian 100; requests
                                        of generate_test_trace.py:47 send 0 */
  double speed_kph;                  /* mode speed cap for route times, 0 = edge speed (auto);
                                        bicycle 18, pedestrian 5.1 */
  double queue_kph;                  /* queue_length speed threshold (README.md:283,295; §3.8) */
  int32_t max_candidates;            /* <= ORC_KMAX */
  int32_t threshold_sec;             /* 15    reporter_service.py:55 */
} orc_params;

#define ORC_MODES 3
#define ORC_MAX_BREAKAGE 30000.0     /* metres: route length <= 3e7 mm */
#define ORC_TB_MAX 131070            /* time bounds above this are not applied (0.1 s; t < 2^17) */
#define ORC_TCCAP 2097151            /* routes whose turn cost exceeds this are pruned (mm, 21 bits):
                                        key = length + turn < 2^25, so (key, length, time) packs in
                                        one 64-bit word on the GPU */

typedef struct orc_graph orc_graph;

orc_graph* orc_graph_load(const char* path);
void orc_graph_free(orc_graph* g);

/* One batch of traces in, everything the parity tests compare out.  All output
 * arrays are malloc'd by the oracle and released with orc_result_free. */
typedef struct orc_result {
  int32_t n_traces;
  /* states (selected probes), concatenated over traces */
  int64_t n_states;
  int64_t* trace_state_off;   /* n_traces+1 */
  int64_t* state_probe;       /* global probe index */
  int32_t* cand_count;        /* n_states */
  uint32_t* cand_edge;        /* n_states*ORC_KMAX */
  double* cand_p;             /* fraction along edge */
  double* cand_sqd;           /* squared snap distance, m^2 */
  int32_t* winner;            /* n_states; -1 = no candidate / not matched */
  int32_t* subpath;           /* n_states; sub-path ordinal within trace, -1 if none */
  /* matched route: edges per trace; a 0xFFFFFFFF entry separates sub-paths */
  int64_t* trace_route_off;   /* n_traces+1 */
  uint32_t* route_edge;
  int64_t n_route;
  /* traffic segments (README.md:288-300) */
  int64_t* trace_seg_off;     /* n_traces+1 */
  int64_t n_seg;
  uint64_t* seg_id;           /* ORC_NO_ID when absent */
  double* seg_start;
  double* seg_end;
  int32_t* seg_length;
  int32_t* seg_queue;
  uint8_t* seg_internal;
  int32_t* seg_begin_shape;
  int32_t* seg_end_shape;
  int64_t* seg_way_off;       /* n_seg+1 */
  uint32_t* seg_way;
  /* report() output per trace */
  int64_t* trace_rep_off;     /* n_traces+1 */
  int64_t n_rep;
  uint64_t* rep_id;
  uint64_t* rep_next;         /* ORC_NO_ID when next_id absent */
  double* rep_t0;
  double* rep_t1;
  int32_t* rep_length;
  int32_t* rep_queue;
  int32_t* shape_used;        /* per trace, -1 = absent */
  int32_t* stats;             /* per trace 7 counts: successful, unreported, discontinuities,
                                 invalid_speeds, invalid_times, unassociated, (pad) */
  double* stats_len;          /* per trace 2: successful_length, unreported_length */
} orc_result;

/* lat/lon/time/accuracy are per probe, trace_off has n_traces+1 entries,
 * accuracy < 0 means "not given"; mode[t]: 0 auto, 1 bicycle, 2 pedestrian.
 * p points to ORC_MODES parameter sets (one per mode). */
int orc_match_batch(const orc_graph* g, const orc_params* p, int32_t n_traces, const int64_t* trace_off,
                    const double* lat, const double* lon, const int64_t* time, const float* accuracy,
                    const uint8_t* mode, uint32_t report_levels_mask, uint32_t transition_levels_mask,
                    int32_t n_threads, orc_result* out);
void orc_result_free(orc_result* r);

/* report() alone over explicit segment arrays (pinned by golden vectors).
 * seg_has_id/has_length flags model Python's None. */
typedef struct orc_report_out {
  int32_t n_rep;
  int32_t shape_used;          /* -1 = key absent */
  int32_t counts[6];
  double lengths[2];
  int32_t length_set[2];       /* 0 => the Python int 0 was never replaced */
} orc_report_out;

int orc_report(int32_t n, const uint8_t* has_id, const uint64_t* seg_id, const double* start,
               const double* end, const uint8_t* internal, const int32_t* queue, const uint8_t* has_length,
               const int32_t* length, const int32_t* begin_shape, int64_t trace_end_time, double threshold,
               uint32_t report_levels_mask, uint32_t transition_levels_mask, uint64_t* rep_id, uint64_t* rep_next,
               double* rep_t0, double* rep_t1, int32_t* rep_length, int32_t* rep_queue, orc_report_out* out);

/* One transition's route from candidate (src_edge, src_p) to (dst_edge, dst_p) under
 * the mode's parameters p: distance bound `bound` metres, time
 * bound from the probes' time difference dt_sec (<= 0: none), both pruning the search.
 * The route is the lexicographic minimum of (length + turn cost, length, time) over the
 * search's labels.  Returns 1 and the route length (m), time (0.1 s) and turn cost (mm)
 * when valid, 0 when no valid route. */
int orc_route(const orc_graph* g, const orc_params* p, int mode, uint32_t src_edge, double src_p, uint32_t dst_edge,
              double dst_p, double bound, int64_t dt_sec, double* out_dist, int64_t* out_time_ds,
              int64_t* out_turn_mm);

/* graph-derived per-edge data the routing semantics use (for tests): heading of the
 * first / last shape segment (integer degrees clockwise from north), route time
 * (0.1 s) under the mode's speed, and the mode's turn cost table (mm, 181 entries). */
int orc_edge_info(const orc_graph* g, const orc_params* p, uint32_t edge, int32_t* h_begin, int32_t* h_end,
                  int64_t* time_ds);
void orc_turn_table(const orc_params* p, int32_t* table181);

#ifdef __cplusplus
}
#endif
#endif
