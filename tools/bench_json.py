#!/usr/bin/env python3
"""JSON-inclusive throughput of the drop-in path (not the headline metric): bench.py's
json_dropin leg (reporter_amd/tools/dropin.py) on its own, at any size.

POST /report bodies (Batch.java:56-65 layout) in, report() bodies out, through one
otr_report_batch call and through coalesced blocking callers (64 / 256 threads), for
whole traces and for BatchingProcessor-sized windows (BatchingProcessor.java:26-29),
each with the host split (scan, SoA, device, format) from otr_service_stats.
Workloads: c2 (generate_test_trace options configured) or c2dep (the deployed defaults).

  python tools/bench_json.py [--workload c2dep] [--traces 10000] [--window 12]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GTT = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000, 'search_radius': 50,
       'gps_accuracy': 16.45}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', choices=['c2', 'c2dep'], default='c2dep')
    ap.add_argument('--traces', type=int, default=10000)
    ap.add_argument('--window', type=int, default=12)
    ap.add_argument('--threads', type=str, default='64,256')
    ap.add_argument('--coalesce', type=int, default=4096)
    ap.add_argument('--wait-us', type=int, default=2000)
    ap.add_argument('--python-callers', action='store_true', help='caller threads in this interpreter')
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime in the process)
    from reporter_amd import matcher as M
    from reporter_amd.tools import dropin, gen
    gpath = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gpath, args.traces, 100, 15, 10.0, 2, t_begin=1483228800, t_spread=1800)
    cfg = M.default_config(gpath, **(GTT if args.workload == 'c2' else {}))
    M.configure(cfg)
    m = M.Matcher()
    m.report_json_batch(dropin.bodies(tr.slice(0, min(256, tr.n_traces)))[0])  # warm-up (workspace, code objects)
    res = dropin.measure(M, m, tr, window=args.window, threads=tuple(int(x) for x in args.threads.split(',')),
                         max_traces=args.coalesce, wait_us=args.wait_us,
                         config=None if args.python_callers else cfg)
    res['workload'] = '%s: %d traces x 100 probes @15 s, metro graph' % (args.workload.upper(), tr.n_traces)
    res['host_threads'] = int(os.environ.get('OTR_HOST_THREADS', '0')) or min(os.cpu_count() or 1, 16)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
