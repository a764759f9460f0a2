/*
 * otr.h — C-ABI of libotr.so, the MI355X-native drop-in for Open Traffic Reporter's
 * matching hot path (trace JSON → map-match → OSMLR segment / speed JSON).
 *
 * Plain C: pointers, sizes, status codes.  No torch or HIP types cross this line.
 * Every entry point names the reference interface it replaces.
 *
 * Threading: otr_configure() is process-global and not thread-safe (call once, as
 * reporter_service.py:284 / simple_reporter.py:132 call valhalla.Configure once).
 * An otr_matcher is owned by one thread at a time (reporter_service.py:51-52 keeps
 * one valhalla.SegmentMatcher per thread); matchers share the read-only graph that
 * otr_configure placed in HBM.
 */
#ifndef OTR_H
#define OTR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (HTTP codes of reporter_service.py:209-245 are kept) ---- */
#define OTR_OK 0
#define OTR_BAD_REQUEST 400   /* reporter_service.py:214,219,225,231,235 */
#define OTR_MATCH_ERROR 500   /* reporter_service.py:244-245 */
#define OTR_NOT_CONFIGURED 503
#define OTR_DEVICE_ERROR 504

typedef struct otr_matcher otr_matcher;

/* Replaces valhalla.Configure(conf_path) (reporter_service.py:284, simple_reporter.py:132).
 * Reads a Valhalla-style JSON config: {"meili": {"default": {...}, "auto": {...}, ...},
 * "otr": {"graph": "<flattened graph file>", "device": 0}} (meili values:
 * Dockerfile:14-17,42-49).  Loads the graph once and uploads it to HBM.  Returns
 * OTR_OK or an error code; otr_last_error() holds the message. */
int otr_configure(const char* config_json_path);

/* Same, with the config given as a JSON string (for embedders without files). */
int otr_configure_json(const char* config_json, size_t len);

/* Replaces valhalla.SegmentMatcher() (reporter_service.py:52, simple_reporter.py:133). */
otr_matcher* otr_matcher_new(void);
void otr_matcher_free(otr_matcher* m);

/* Replaces SegmentMatcher.Match(json) -> str (reporter_service.py:240,
 * simple_reporter.py:166): trace JSON in, {"segments":[...],"mode":...} out
 * (schema README.md:288-300).  *out is owned by the library: release with otr_free.
 * Returns OTR_OK, or an error code with *out = {"error":"..."}. */
int otr_match(otr_matcher* m, const char* json, size_t len, char** out, size_t* out_len);

/* Replaces the HTTP POST /report round trip (Batch.java:68 → reporter_service.py
 * handle_request 209-245): request validation, Match, then report() with
 * report_levels / transition_levels from match_options (reporter_service.py:228-235).
 * Returns 200 with the report() JSON, or 400/500 with {"error":"..."} carrying the
 * reference's messages.  threshold_sec < 0 selects THRESHOLD_SEC or 15
 * (reporter_service.py:55-58). */
int otr_report(otr_matcher* m, const char* json, size_t len, int threshold_sec, char** out, size_t* out_len);

/* report() alone (reporter_service.py:79-179) over a Match() output string and the
 * original trace JSON; for callers that already hold a match (simple_reporter.py:168). */
int otr_report_segments(const char* match_json, size_t match_len, const char* trace_json, size_t trace_len,
                        int threshold_sec, const int32_t* report_levels, int n_report_levels,
                        const int32_t* transition_levels, int n_transition_levels, char** out, size_t* out_len);

/* n POST /report bodies at once (the reference serves one per HTTP request,
 * reporter_service.py:209-245; a batching caller such as BatchingProcessor.java:58-141
 * holds many).  Bodies are scanned on host threads, grouped by the options that must
 * be uniform within a device batch (report/transition levels, match_options
 * overrides) and matched in shared device batches.  codes[i] / outs[i] / out_lens[i]
 * are exactly what otr_report returns for bodies[i] (release each outs[i] with
 * otr_free).  Returns OTR_OK once every item has its code. */
int otr_report_batch(otr_matcher* m, int32_t n, const char* const* bodies, const size_t* lens, int threshold_sec,
                     int32_t* codes, char** outs, size_t* out_lens);

/* Process-wide request coalescing (SURVEY §8b threading row): while enabled,
 * otr_report calls from any number of threads are handed to one dispatcher thread
 * that runs them as shared device batches of up to max_traces, waiting at most
 * max_wait_us after the first queued request.  Each caller still blocks until its
 * own response is ready and receives exactly what the uncoalesced call returns.
 * max_traces <= 0 drains the queue and stops the dispatcher. */
int otr_coalesce(int32_t max_traces, int32_t max_wait_us);

/* Where the JSON request path's host time goes (new; diagnostics for the drop-in
 * callers of otr_report / otr_report_batch / the coalescer): summed over every internal
 * request-processing call of the process since the last reset — calls (a batch call, or
 * one coalesced batch), items (bodies), device batches, and the wall seconds of its
 * phases: scan (body parse + validation into SoA, host threads), soa (gather of each
 * device batch's arrays), device (otr_match_batch: H2D, kernels, D2H of the compacted
 * reports), format (report() bodies, host threads); total is their sum plus grouping. */
typedef struct otr_service_split {
  int64_t calls, items, device_batches;
  double scan_s, soa_s, device_s, format_s, total_s;
} otr_service_split;
int otr_service_stats(otr_service_split* out, int reset);

void otr_free(char* p);
const char* otr_last_error(void);

/* ---- batched throughput API (new; the reference matches one trace per call) ---- */

#define OTR_MEM_HOST 0
#define OTR_MEM_DEVICE 1

typedef struct otr_trace_batch {
  int32_t n_traces;
  int32_t memory;              /* OTR_MEM_HOST or OTR_MEM_DEVICE (pointers in HBM) */
  const int64_t* trace_offsets;  /* n_traces+1 probe offsets */
  const double* lat;
  const double* lon;
  const int64_t* time;         /* epoch seconds */
  const float* accuracy;       /* metres, NULL or <0 entries = not given */
  const uint8_t* mode;         /* per trace: 0 auto, 1 bicycle, 2 pedestrian */
  uint32_t report_levels;      /* bit mask of OSMLR levels, simple_reporter --report-levels */
  uint32_t transition_levels;  /* bit mask, --transition-levels */
  int32_t threshold_sec;       /* report() tail threshold, 15 */
  int32_t quantisation;        /* hour bucket seconds, 3600 (simple_reporter.py:343) */
  int64_t hist_base_time;      /* histogram covers [base, base + hist_hours*quantisation) */
  int32_t hist_hours;
  int32_t flags;               /* OTR_BATCH_* */
  uint32_t* hist_device;       /* optional caller-owned device histogram (else library-owned) */
  int32_t tile_rules;          /* OTR_TILE_RULES_* for OTR_BATCH_TILE_ROWS */
  int32_t reserved;
} otr_trace_batch;

#define OTR_BATCH_COPY_OUT 1   /* fill the host arrays of otr_batch_result */
#define OTR_BATCH_TIMING 2     /* record per-kernel HIP-event timings */
#define OTR_BATCH_COPY_REPORTS 4  /* host copies of segments, reports, stats only (the JSON path) */
#define OTR_BATCH_TILE_ROWS 8  /* also emit simple_reporter tile rows on device (d_rows / n_rows) */
#define OTR_BATCH_ROUTE_WORK 16  /* count the LDS route tiers' work (route_tier_work, counters
                                    3, 4, 9, 10, 13, 14): instrumentation, ~7% of the first tier */

/* One simple_reporter tile line (simple_reporter.py:188-195) in binary form: the line
 * "id,next_id,duration,1,length,queue_length,start,end,source,MODE" of the file
 * "{b*q}_{(b+1)*q-1}/{level}/{tile_index}" (q = quantisation). */
typedef struct otr_tile_row {
  uint64_t file;       /* bucket b << 25 | level << 22 | tile index (get_tile_level/_index, :45-49) */
  uint64_t id;         /* segment id */
  uint64_t next_id;    /* next segment id, or INVALID_SEGMENT_ID 0x3fffffffffff (:43,193) */
  int64_t start;       /* floor(t0) */
  int64_t end;         /* ceil(t1) */
  int32_t duration;    /* int(round(t1 - t0)), Python 2 rounding (:179) */
  int32_t length;
  int32_t queue_length;
  int32_t speed_bin;   /* min(int(length / (t1 - t0) * 3.6 / 20), 7): the report's 20 km/h speed bin */
} otr_tile_row;
#define OTR_INVALID_SEGMENT_ID 0x3fffffffffffull

/* Which reference path the tile rows follow.
 * OTR_TILE_RULES_SIMPLE: simple_reporter.py:176-196 (t1 - t0 > .5, floor/ceil hour buckets,
 *   bucket-span limit), files sorted as text lines (:218).
 * OTR_TILE_RULES_STREAM: the Java streaming path — Segment.valid (Segment.java:38-40) as
 *   BatchingProcessor.forward applies it (:119-126), TimeQuantisedTile.getTiles buckets
 *   (TimeQuantisedTile.java:26-35), files sorted by Segment.compareTo (numeric id,
 *   next_id; stable: arrival order within a pair) and written by
 *   Segment.appendToStringBuffer (Segment.java:59-74) as AnonymisingProcessor.store does. */
#define OTR_TILE_RULES_SIMPLE 0
#define OTR_TILE_RULES_STREAM 1

#define OTR_NO_ID 0xFFFFFFFFFFFFFFFFull

/* kernel_ms slots (OTR_STAGE_LINK: K_link, the per-state search inputs and the task records) */
enum { OTR_STAGE_STATES = 0, OTR_STAGE_CANDIDATES, OTR_STAGE_LINK, OTR_STAGE_ROUTE, OTR_STAGE_ROUTE_BIG,
       OTR_STAGE_VITERBI, OTR_STAGE_PATHS, OTR_STAGE_PATHS_BIG, OTR_STAGE_SEGMENTS, OTR_STAGE_HISTOGRAM,
       OTR_STAGE_TOTAL };
#define OTR_HIST_BINS 8        /* speed bins of 20 km/h: [0,20) … [140,∞) */

/* All pointers below are owned by the matcher and stay valid until the next batch
 * call or otr_matcher_free.  Host arrays are filled only with OTR_BATCH_COPY_OUT;
 * the device histogram is always produced. */
typedef struct otr_batch_result {
  int32_t n_traces;
  int64_t n_probes;
  int64_t n_states;
  int64_t n_route;
  int64_t n_seg;
  int64_t n_rep;
  int64_t n_rows;              /* simple_reporter tile rows (after filter + hour fan-out) */
  int32_t status;              /* OTR_OK or first error */
  int32_t n_overflow_traces;   /* traces whose search exceeded the largest LDS table */
  /* host copies (OTR_BATCH_COPY_OUT) — same layout as oracle/oracle.h orc_result */
  int64_t* trace_state_off;  int64_t* state_probe;  int32_t* cand_count;
  uint32_t* cand_edge;  double* cand_p;  double* cand_sqd;   /* n_states * 64 slots */
  int32_t* winner;  int32_t* subpath;
  int64_t* trace_route_off;  uint32_t* route_edge;
  int64_t* trace_seg_off;  uint64_t* seg_id;  double* seg_start;  double* seg_end;
  int32_t* seg_length;  int32_t* seg_queue;  uint8_t* seg_internal;
  int32_t* seg_begin_shape;  int32_t* seg_end_shape;  int64_t* seg_way_off;  uint32_t* seg_way;
  int64_t* trace_rep_off;  uint64_t* rep_id;  uint64_t* rep_next;  double* rep_t0;  double* rep_t1;
  int32_t* rep_length;  int32_t* rep_queue;  int32_t* shape_used;  int32_t* stats;  double* stats_len;
  /* device outputs */
  uint32_t* d_hist;            /* [hist_hours][n_segments][OTR_HIST_BINS] observation counts */
  int64_t hist_len;            /* elements */
  /* algorithmic byte counters, summed over the batch */
  uint64_t counters[24];       /* algorithmic work counters: 0 cells visited,
                                  1 shape segments tested, 2 candidates, 3 settled nodes and
                                  4 relaxed edges (first-tier route launch), 5 search tasks,
                                  6 transition entries, 7 output segments, 8 tile rows,
                                  9/10 settled/relaxed of the large-table retry, 11/12 node
                                  searches resumed from / dumped to HBM (next retry table), 13 search rounds
                                  and 14 table keys (first-tier route launch),
                                  16-21 diagnostic-build search phase cycles, 22/23 edge-state
                                  searches resumed from / dumped to HBM (next table) */
  float kernel_ms[16];         /* OTR_BATCH_TIMING: device time per stage, OTR_STAGE_* */
  int32_t* trace_status;       /* host, per trace (with COPY_OUT / COPY_REPORTS): OTR_OK, or
                                  OTR_MATCH_ERROR when its search outgrew the largest LDS table */
  otr_tile_row* d_rows;        /* OTR_BATCH_TILE_ROWS: n_rows tile rows in HBM (matcher-owned),
                                  trace by trace in report order */
  /* per route-search kernel: slot 0 the first tier (k_route<160,2>), 1..5 the LDS retry
   * tiers in order, 6 / 7 the global-memory search (32K / 1M-state slabs), 8 the 64-bit
   * label LDS tier (steps whose length and time bits exceed 32), 10 the first edge-state
   * tier (modes with turn costs), 9 / 11 the larger edge-state tables (512, then 1024 states),
   * 12 the small-search first tier (k_route<80,4>: steps expected to stay small), 13 the
   * tiny-search first tier (k_route<40,8>: at most 8 targets, tinier still), 14..15 unused.
   * code: 6,000,000 + CAP*100 + targets of an edge-state tier, CAP*10+G of an LDS tier,
   * 900000 + CAP the 64-bit tier, -1 / -2 the global tiers, 0 unused (a tier with no task
   * kind to run: the node tiers when every mode has turn costs).
   * work: searches, settled nodes (expanded states), relaxed edges, transition entries
   * written.  ms (OTR_BATCH_TIMING): HIP-event time of the kernel on the matcher's stream. */
  int32_t route_tier_code[16];
  float route_tier_ms[16];
  uint64_t route_tier_work[16][4];
} otr_batch_result;

/* At most otr_max_batch_probes() = 2^26 - 64 (67,108,800) probes per call
 * (OTR_BAD_REQUEST beyond: split the input). */
int otr_match_batch(otr_matcher* m, const otr_trace_batch* in, otr_batch_result* out);

/* The batch limit and its reason: a kernel dispatch counts its work-items in 32 bits, and
 * the per-state / per-trace kernels give every state / trace a 64-lane wave.
 * otr_launch_max_items: the most work-items one of those launches dispatches for a batch
 * of n_states states and n_traces traces (states_per_wave 1 or 2: k_prep / k_tasks);
 * a batch of otr_max_batch_probes() probes stays below 2^32.  Host-only (no device). */
int64_t otr_max_batch_probes(void);
uint64_t otr_launch_max_items(int64_t n_states, int64_t n_traces, int32_t states_per_wave);

/* simple_reporter's tile stage (simple_reporter.py:211-239) on device: sort the rows
 * by file, then in the line order of segments.sort() (:218, string order of the whole
 * line), and delete the (id, next_id) runs seen fewer than `privacy` times with the
 * reference loop's exact rule (:221-239, including its trailing-singleton quirk).
 * With rules = OTR_TILE_RULES_STREAM the order is Segment.compareTo's instead and the
 * cull is AnonymisingProcessor.clean (AnonymisingProcessor.java:155-175, same rule).
 * rows: n rows in host (OTR_MEM_HOST) or device (OTR_MEM_DEVICE) memory, e.g. the
 * d_rows of a batch or rows received from other GPUs.  *out: the kept rows, sorted,
 * in host memory owned by the matcher (valid until its next call). */
int otr_tiles_cull(otr_matcher* m, const otr_tile_row* rows, int64_t n, int32_t memory, int32_t privacy,
                   int32_t rules, const otr_tile_row** out, int64_t* n_out);

/* ---- keyed speed histogram -------------------------------------------
 * One entry per (hour-tile file, segment pair, speed bin) with its observation count:
 * the per-GPU histogram is the tile rows sort-reduced by that key; GPUs exchange entries
 * with the rank owning their (hour, tile) file (RCCL all-to-all, simple_reporter.
 * file_owner) and each owner reduces what it received and applies the privacy cull to
 * complete pairs (a pair's total count over its bins >= privacy; the reference cull's
 * trailing-singleton rule belongs to the line-based tile files, otr_tiles_cull). */
typedef struct otr_hist_entry {
  uint64_t file;       /* bucket << 25 | level << 22 | tile index, as otr_tile_row.file */
  uint64_t id;
  uint64_t next_id;    /* or OTR_INVALID_SEGMENT_ID */
  uint32_t speed_bin;  /* 20 km/h bins 0..7 */
  uint32_t count;
} otr_hist_entry;

/* Sort-reduce n entries (in: host or device memory) by (file, id, next_id, speed_bin),
 * summing counts; with privacy > 1 also drop the (file, id, next_id) pairs whose total
 * count is below privacy.  The reduced entries, in key order, are copied to `out`
 * (out_memory: host or device; room for out_cap entries, n suffices) and *n_out is
 * their number.  rows_in != 0: the input is n tile rows, count 1 each. */
int otr_hist_reduce(otr_matcher* m, const void* in, int64_t n, int32_t memory, int32_t rows_in, int32_t privacy,
                    otr_hist_entry* out, int64_t out_cap, int32_t out_memory, int64_t* n_out);

/* The CSV lines of n (host) rows in order.  OTR_TILE_RULES_SIMPLE: "id,next,duration,1,
 * length,queue,start,end,source,MODE\n" each (simple_reporter.py:188-195).
 * OTR_TILE_RULES_STREAM: "\nid,[next],duration,1,length,queue,start,end,source,MODE"
 * each, next empty when invalid (Segment.java:59-74).  mode is upper-cased as both do. */
int otr_tiles_format(const otr_tile_row* rows, int64_t n, const char* source, const char* mode, int32_t rules,
                     char** out, size_t* out_len);

/* ---- graph building (§8 f rank 1) -------------------------------------------------------
 * Tile hierarchy of the reference's py/get_tiles.py:30-102 (Valhalla baldr): levels 0/1/2
 * tile the world with 4 / 1 / 0.25 degree tiles, tile id = row * ncolumns + col.
 *   otr_tilehier_row / otr_tilehier_col: Tiles.Row / Tiles.Col (:51-72), -1 outside the world.
 *   otr_tilehier_file: Tiles.GetFile (:81-102), e.g. level 2, id 745313, "gph" ->
 *     "2/000/745/313.gph"; out gets the NUL-terminated name (cap bytes of room).
 *   otr_tilehier_files: the script's listing (:132-171) for a bbox — split at the
 *     antimeridian, levels 0, 1, 2 (Python 2 dict order), rows then columns — as
 *     newline-terminated names in *out (release with otr_free). */
int32_t otr_tilehier_row(int32_t level, double lat);
int32_t otr_tilehier_col(int32_t level, double lon);
int otr_tilehier_file(int32_t level, int64_t tile_id, const char* suffix, char* out, size_t cap);
int otr_tilehier_files(double min_lon, double min_lat, double max_lon, double max_lat, const char* suffix, char** out,
                   size_t* out_len);

/* The flattener: decoded road-graph arrays (what a Valhalla GraphTile reader yields for
 * the tiles otr_tilehier_files lists: nodes, directed edges, edge shapes, way ids, OSMLR
 * associations) -> the .otrg file otr_configure uploads (include/otr_graph_format.h).
 * Edges may come in any order; the file's edges are sorted by (src, dst), stable.
 * Edges shorter than 5 cm are contracted (their end nodes merge into the smallest node
 * id; DESIGN.md §3.4: shorter edges only narrow the exact search rounds); a
 * contracted edge's OSMLR begin/end flag moves to its segment's neighbouring edge.
 * Routing lengths are the shapes' lengths.  Decoding the .gph binary itself needs
 * Valhalla 2.3.6's GraphTile layout (UPSTREAM, absent here): out of scope. */
typedef struct otr_flat_graph {
  uint32_t n_nodes;
  const int32_t* node_ll;      /* [2*n_nodes] lat_e6, lon_e6 */
  uint32_t n_edges;
  const uint32_t* edge_src;    /* node index */
  const uint32_t* edge_dst;
  const uint32_t* edge_attr;   /* OTR_ATTR_* fields of otr_graph_format.h (access, speed, level,
                                  internal, OSMLR segment begin / end) */
  const uint32_t* edge_seg;    /* OSMLR segment index into seg_id, OTR_NO_SEGMENT; may be NULL */
  const uint32_t* edge_way;    /* OSM way id (low 32 bits); may be NULL */
  const uint32_t* shape_off;   /* [n_edges+1] into shape_ll; a shape holds both end nodes */
  const int32_t* shape_ll;     /* lat_e6, lon_e6 pairs */
  uint32_t n_segments;
  const uint64_t* seg_id;      /* OSMLR ids: level(3) | tile(22) | index(21) */
  const uint32_t* seg_len;     /* whole metres */
  double cell_deg;             /* candidate grid cell (degrees); 0 = 0.0005 (meili's 500 per tile) */
} otr_flat_graph;

typedef struct otr_flat_stats {
  uint32_t n_nodes, n_edges;          /* written */
  uint32_t n_contracted_edges;        /* edges < 5 cm (and edges inside merged clusters) */
  uint32_t n_merged_nodes;
} otr_flat_stats;

int otr_flatten(const otr_flat_graph* in, const char* out_path, otr_flat_stats* stats);

/* ---- ingest: probe text → windowed traces in HBM (§8 f rank 4) -------------------------
 * OTR_INGEST_SHARD: the "uuid,time,lat,lon,acc" lines simple_reporter.match() reads
 *   (simple_reporter.py:140-160): line.strip().split(',') into exactly 5 fields,
 *   float() coordinates, int() time and accuracy.
 * OTR_INGEST_RAW: the raw feed simple_reporter.download() reads (:99-111) followed by the
 *   shard round trip into match(): fields by index after splitting on `separator`, the
 *   bbox filter (applied before time and accuracy are parsed, as :103-105), the fast
 *   "%Y-%m-%d %H:%M:%S" time (:106-107) or epoch seconds, accuracy min(ceil(x), 1000)
 *   (:110), and coordinates as match() re-reads them from the Python 2 str() text
 *   (12 significant digits, :111).
 * OTR_INGEST_JAVA_SV: Formatter.formatSV (Formatter.java:103-114): float32 coordinates,
 *   (int)ceil accuracy, Long.parseLong or "yyyy-MM-dd HH:mm:ss" time.
 * Then, for every rule: points grouped by uuid, sorted by time (stable), split at gaps
 *   > inactivity seconds, windows of fewer than 2 points dropped (:146-160).  Traces come
 *   out in order of the first appearance of their uuid, then by time. */
#define OTR_INGEST_SHARD 0
#define OTR_INGEST_RAW 1
#define OTR_INGEST_JAVA_SV 2
#define OTR_TIME_EPOCH 0
#define OTR_TIME_YMDHMS 1
/* bad_reason: why the first rejected line (bad_line) was rejected */
#define OTR_INGEST_E_FIELDS 1     /* wrong field count / index out of range (ValueError, IndexError) */
#define OTR_INGEST_E_FLOAT 2      /* coordinate not a finite decimal number */
#define OTR_INGEST_E_INT 3        /* time or accuracy not an integer (int()) */
#define OTR_INGEST_E_TIME 4       /* date fields out of range (datetime.date) */
#define OTR_INGEST_E_UUID 5       /* uuid holds the shard separator ',' */
#define OTR_INGEST_E_PRECISION 6  /* > 19 significant digits whose rounding needs big-number arithmetic */
#define OTR_INGEST_E_COLLISION 7  /* two uuids share a 64-bit hash (never seen; refused rather than merged) */
#define OTR_INGEST_E_ACCURACY 8   /* accuracy not finite or beyond ±2^24 */

typedef struct otr_ingest_format {
  int32_t rules;          /* OTR_INGEST_* */
  int32_t separator;      /* field separator byte: ',' (SHARD, fixed), '|' (raw feed) */
  int32_t uuid_index, time_index, lat_index, lon_index, accuracy_index;  /* RAW / JAVA_SV */
  int32_t time_format;    /* OTR_TIME_* (RAW / JAVA_SV) */
  int32_t inactivity;     /* seconds (--inactivity, 120) */
  int32_t mode;           /* 0 auto, 1 bicycle, 2 pedestrian: the batch's mode (--mode) */
  int32_t use_bbox;       /* RAW: apply bbox */
  int32_t reserved;
  double bbox[4];         /* min lat, min lon, max lat, max lon (--bbox) */
} otr_ingest_format;

typedef struct otr_ingest_result {
  int64_t n_lines;        /* lines in the text */
  int64_t n_kept;         /* lines inside the bbox */
  int64_t n_probes;       /* probes in windows of >= 2 points */
  int32_t n_traces;       /* windows */
  int32_t n_uuids;
  int64_t bad_line;       /* first rejected line (0-based), -1 if none */
  int32_t bad_reason;     /* OTR_INGEST_E_* */
  float parse_ms;         /* device time of the line parse kernel (HIP events on the matcher's stream) */
  float total_ms;         /* device time from the first kernel to the last (host syncs between included) */
  int32_t reserved;
  otr_trace_batch batch;  /* memory = OTR_MEM_DEVICE: offsets, lat, lon, time, accuracy, mode in HBM
                             (matcher-owned, valid until its next otr_ingest); levels/flags zero */
  const int64_t* d_trace_uuid_off;  /* per trace: byte offset of its uuid in the text */
  const int32_t* d_trace_uuid_len;
} otr_ingest_result;

/* Parse `len` bytes of probe lines (host or device memory) into traces in HBM.  Returns
 * OTR_OK, or OTR_BAD_REQUEST with bad_line / bad_reason set where the reference raises
 * (the whole text is refused, as the reference loses the file).  The batch can be
 * passed straight to otr_match_batch after setting its levels, threshold and flags. */
int otr_ingest(otr_matcher* m, const char* text, int64_t len, int32_t memory, const otr_ingest_format* fmt,
               otr_ingest_result* out);

/* report() (reporter_service.py:79-179) over n segment lists at once, evaluated by the
 * device code of the segment scan K7 (otr_report.h compiled for gfx950, one thread per
 * list) — what pins the device tail against the reference's own report() outputs.  Host
 * arrays; list c holds segments seg_off[c] .. seg_off[c+1]-1 (seg_id OTR_NO_ID: no id;
 * has_length 0: no length) and its reports go to rep_* from index seg_off[c]; per list:
 * n_rep, shape_used (-1 absent), counts[6] (successful, unreported, discontinuities,
 * invalid_speeds, invalid_times, unassociated), lengths[2], length_set[2]. */
int otr_report_lists_device(int32_t n, const int64_t* seg_off, const uint64_t* seg_id, const double* start,
                            const double* end, const uint8_t* internal, const int32_t* queue,
                            const uint8_t* has_length, const int32_t* length, const int32_t* begin_shape,
                            const int64_t* end_time, const double* threshold, const uint32_t* report_levels,
                            const uint32_t* transition_levels, uint64_t* rep_id, uint64_t* rep_next, double* rep_t0,
                            double* rep_t1, int32_t* rep_length, int32_t* rep_queue, int32_t* n_rep,
                            int32_t* shape_used, int32_t* counts, double* lengths, int32_t* length_set);

/* graph facts for callers sizing histograms */
int otr_graph_info(int64_t* n_nodes, int64_t* n_edges, int64_t* n_segments);

/* device + stream the matcher runs on (hipStream_t as void*), for callers that
 * place inputs in HBM themselves and bracket timing */
void* otr_matcher_stream(otr_matcher* m);
int otr_device(void);

#ifdef __cplusplus
}
#endif
#endif
