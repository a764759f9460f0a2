#!/usr/bin/env python3
"""JSON-inclusive throughput of the drop-in path (not the headline metric).

The headline bench.py line times the hot path with inputs resident in HBM.  This tool
times what a JSON caller sees: POST /report bodies (Batch.java:56-65 layout) in,
report() bodies (reporter_service.py:164-179) out, through
  1. otr_report_batch — one call with every body (host scan, H2D, match, D2H, format);
  2. otr_report from many threads with otr_coalesce on — the Kafka-stream-thread /
     HTTP-server-thread pattern, each caller blocking on its own response.
Workload: C2 traces (metro graph, 100 probes @15 s, sigma 10 m).

  python tools/bench_json.py [--traces 10000] [--threads 64] [--coalesce 4096]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bodies_for(tr):
    """Batch.report's body: lat/lon as Java floats printed with <= 6 decimals (Point.java:59-65)."""
    out = []
    for t in range(tr.n_traces):
        a, b = int(tr.offsets[t]), int(tr.offsets[t + 1])
        pts = ','.join('{"lat":%.6f,"lon":%.6f,"time":%d}' % (tr.lat[i], tr.lon[i], tr.time[i]) for i in range(a, b))
        out.append('{"uuid":"%s","match_options":{"mode":"auto","report_levels":[0,1],'
                   '"transition_levels":[0,1]},"trace":[%s]}' % (tr.uuids[t], pts))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--traces', type=int, default=10000)
    ap.add_argument('--threads', type=int, default=64)
    ap.add_argument('--coalesce', type=int, default=4096)
    ap.add_argument('--wait-us', type=int, default=5000)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime in the process)
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    gpath = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gpath, args.traces, 100, 15, 10.0, 2, t_begin=1483228800, t_spread=1800)
    t0 = time.time()
    bodies = [b.encode() for b in bodies_for(tr)]
    mb = sum(len(b) for b in bodies) / 1e6
    print('bodies: %d (%.1f MB, %.1f s to build)' % (len(bodies), mb, time.time() - t0), file=sys.stderr)
    M.configure(M.default_config(gpath))
    m = M.Matcher()
    m.report_json_batch(bodies[:256])  # warm-up (workspace, code objects)

    # (a) the C call alone, as a C / Java (FFM) caller sees it
    import ctypes
    from reporter_amd import _lib
    L = _lib.lib()
    n = len(bodies)
    arr = (ctypes.c_char_p * n)(*bodies)
    lens = (ctypes.c_size_t * n)(*[len(b) for b in bodies])
    codes = (ctypes.c_int32 * n)()
    outs = (ctypes.c_void_p * n)()
    olens = (ctypes.c_size_t * n)()
    best_c = None
    for _ in range(args.reps):
        t = time.perf_counter()
        L.otr_report_batch(m._h, n, arr, lens, -1, codes, outs, olens)
        dt = time.perf_counter() - t
        best_c = dt if best_c is None else min(best_c, dt)
        out_mb = sum(olens[i] for i in range(n)) / 1e6
        for i in range(n):
            L.otr_free(outs[i])
    # (b) the Python round trip (ctypes marshalling + decoding every body)
    best = None
    for _ in range(args.reps):
        t = time.perf_counter()
        res = m.report_json_batch(bodies)
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    ok = sum(1 for c, _ in res if c == 200)
    batch_rate = tr.n_probes / best

    got = [None] * len(bodies)
    M.coalesce(args.coalesce, args.wait_us)

    def worker(k):
        mk = M.Matcher()
        for i in range(k, len(bodies), args.threads):
            got[i] = mk.report_json(bodies[i])

    th = [threading.Thread(target=worker, args=(k,)) for k in range(args.threads)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt_c = time.perf_counter() - t
    M.coalesce(0)
    same = got == res
    print(json.dumps({
        'metric': 'report() bodies per second, JSON in -> JSON out (drop-in path, not the headline)',
        'workload': 'C2: %d traces x 100 probes, metro graph, %.1f MB of POST bodies' % (tr.n_traces, mb),
        'batch_api_c_call': {'probes_per_s': round(tr.n_probes / best_c, 1),
                             'traces_per_s': round(tr.n_traces / best_c, 1), 'seconds': round(best_c, 4),
                             'MB_in': round(mb, 1), 'MB_out': round(out_mb, 1)},
        'batch_api_python': {'probes_per_s': round(batch_rate, 1), 'traces_per_s': round(tr.n_traces / best, 1),
                             'seconds': round(best, 4), 'ok_200': ok},
        'coalesced_threads': {'threads': args.threads, 'max_traces': args.coalesce, 'max_wait_us': args.wait_us,
                              'probes_per_s': round(tr.n_probes / dt_c, 1), 'seconds': round(dt_c, 4),
                              'identical_to_batch': same},
        'host_threads': int(os.environ.get('OTR_HOST_THREADS', '0')) or min(os.cpu_count() or 1, 16),
    }), flush=True)


if __name__ == '__main__':
    main()
