/*
 * asan_main.c — TEST INFRASTRUCTURE ONLY: a standalone driver for the sanitizer build of
 * the oracle (make -C oracle asan → oracle/_asan/oracle_asan, built with
 * -fsanitize=address,undefined).  Reads a batch dumped by tests/test_oracle_sanitizer.py,
 * matches it with orc_match_batch and prints a digest of the result, so the test can
 * compare it with the regular build's digest.
 *
 * batch file (little endian): i32 n_traces, i32 n_threads, then ORC_MODES orc_params,
 * i64 trace_off[n+1], f64 lat[N], f64 lon[N], i64 time[N], u8 mode[n]
 */
#include <stdio.h>
#include <stdlib.h>

#include "oracle.h"

static unsigned long long fnv(unsigned long long h, const void* p, size_t n) {
  const unsigned char* c = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: oracle_asan graph.otrg batch.bin\n");
    return 2;
  }
  orc_graph* g = orc_graph_load(argv[1]);
  FILE* f = fopen(argv[2], "rb");
  if (!g || !f) return 3;
  int32_t n = 0, threads = 1;
  orc_params p[ORC_MODES];
  if (fread(&n, 4, 1, f) != 1 || fread(&threads, 4, 1, f) != 1 || fread(p, sizeof(p), 1, f) != 1) return 4;
  int64_t* off = (int64_t*)malloc(8 * ((size_t)n + 1));
  if (fread(off, 8, (size_t)n + 1, f) != (size_t)n + 1) return 5;
  const size_t N = (size_t)off[n];
  double* lat = (double*)malloc(8 * N + 8);
  double* lon = (double*)malloc(8 * N + 8);
  int64_t* tm = (int64_t*)malloc(8 * N + 8);
  uint8_t* mode = (uint8_t*)malloc((size_t)n + 1);
  if (fread(lat, 8, N, f) != N || fread(lon, 8, N, f) != N || fread(tm, 8, N, f) != N ||
      fread(mode, 1, (size_t)n, f) != (size_t)n)
    return 6;
  fclose(f);
  orc_result r;
  orc_match_batch(g, p, n, off, lat, lon, tm, NULL, mode, 3u, 3u, threads, &r);
  unsigned long long h = 1469598103934665603ull;
  h = fnv(h, r.winner, 4 * (size_t)r.n_states);
  h = fnv(h, r.route_edge, 4 * (size_t)r.n_route);
  h = fnv(h, r.seg_id, 8 * (size_t)r.n_seg);
  h = fnv(h, r.seg_start, 8 * (size_t)r.n_seg);
  h = fnv(h, r.seg_end, 8 * (size_t)r.n_seg);
  h = fnv(h, r.seg_queue, 4 * (size_t)r.n_seg);
  h = fnv(h, r.rep_id, 8 * (size_t)r.n_rep);
  h = fnv(h, r.rep_t0, 8 * (size_t)r.n_rep);
  printf("states %lld route %lld segments %lld reports %lld digest %016llx\n", (long long)r.n_states,
         (long long)r.n_route, (long long)r.n_seg, (long long)r.n_rep, h);
  orc_result_free(&r);
  orc_graph_free(g);
  free(off);
  free(lat);
  free(lon);
  free(tm);
  free(mode);
  return 0;
}
