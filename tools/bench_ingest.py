#!/usr/bin/env python3
"""K11 ingest throughput (§8 f rank 4; not the headline metric).

Workload: the C2 traces (metro graph, 10k traces x 100 probes @15 s, sigma 10 m) written
as the shard lines simple_reporter.match() reads ("uuid,time,lat,lon,acc", 30 % of lines
out of order, one pause per trace that splits it into two windows, coordinates in four
number styles) and resident in HBM.  Timed:
  ingest   otr_ingest alone (lines → windowed traces in HBM), wall clock per call
  e2e      text → tiles: otr_ingest + otr_match_batch (tile rows) + otr_tiles_cull
The parse kernel's roofline: algorithmic bytes = text bytes + 8 B newline offset read +
56 B written per line (hash, uuid offset/len, time, lat, lon, accuracy, keep flag),
over its HIP-event duration on the matcher's stream.  CPU baseline: the oracle's
restatement of match()'s reading loop (oracle/ingest.py, Python, 1 core) on a sample.

  python tools/bench_ingest.py [--traces 10000] [--steps 10] [--e2e-steps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--traces', type=int, default=10000)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--e2e-steps', type=int, default=3)
    ap.add_argument('--cpu-lines', type=int, default=100000)
    args = ap.parse_args()
    import numpy as np
    import torch
    from reporter_amd import _lib
    from reporter_amd import matcher as M
    from reporter_amd import simple_reporter as sr
    from reporter_amd.tools import gen
    gpath = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gpath, args.traces, 100, 15, 10.0, 2, t_begin=gen.T_BEGIN, t_spread=3 * 3600)
    t0 = time.time()
    text = gen.probe_text(tr, 'shard', seed=5, shuffle=0.3, split_gap=600)
    sys.stderr.write('text: %d lines, %.1f MB (gen %.1fs)\n' % (tr.n_probes, len(text) / 1e6, time.time() - t0))
    M.configure(M.default_config(gpath))
    m = M.Matcher()
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()

    def ingest():
        return m.ingest(None, rules=_lib.OTR_INGEST_SHARD, inactivity=120, device_ptr=d_text.data_ptr(),
                        nbytes=len(text))

    for _ in range(args.warmup):
        ingest()
    parse_ms, total_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r, b = ingest()
        parse_ms.append(r.parse_ms)
        total_ms.append(r.total_ms)
    wall = (time.perf_counter() - t0) / args.steps
    n_lines = int(r.n_lines)
    parse = float(np.mean(parse_ms))
    alg = len(text) + 64 * n_lines
    # end to end: text → tiles (privacy 2)
    e2e = None
    if args.e2e_steps:
        sr.text_tiles_device(m, text, 2)
        t0 = time.perf_counter()
        for _ in range(args.e2e_steps):
            tiles = sr.text_tiles_device(m, text, 2)
        e2e = (time.perf_counter() - t0) / args.e2e_steps
        sys.stderr.write('e2e from host text: %d tile files\n' % len(tiles))
    # CPU restatement on a sample
    from oracle import ingest as oi
    cut = text.index(b'\n', int(len(text) * args.cpu_lines / max(n_lines, 1))) + 1 if args.cpu_lines < n_lines \
        else len(text)
    sample = text[:cut]
    n_sample = sample.count(b'\n')
    t0 = time.perf_counter()
    oi.shard_traces(sample, 120)
    cpu = n_sample / (time.perf_counter() - t0)
    out = {
        'metric': 'probe lines ingested/s (shard text in HBM -> windowed traces in HBM)',
        'value': round(n_lines / wall, 1), 'unit': 'lines/s', 'n_gpus': 1, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(wall * 1e3, 3), 'higher_is_better': True, 'dtype': 'u8/f64',
        'data': 'synthetic', 'config': {'workload': 'C2 traces as simple_reporter shard lines', 'lines': n_lines,
                                        'bytes': len(text), 'traces_out': int(r.n_traces)},
        'device_ms': {'parse': round(parse, 3), 'ingest_total': round(float(np.mean(total_ms)), 3)},
        'roofline': {'kernel': 'k_ingest_parse', 'bound': 'hbm', 'achieved': round(alg / parse / 1e6, 1),
                     'peak': PEAK_HBM_GBS, 'unit': 'GB/s', 'frac': round(alg / parse / 1e6 / PEAK_HBM_GBS, 4),
                     'traffic': None, 'algorithmic_bytes': alg},
        'e2e_text_to_tiles': None if e2e is None else {'probes_per_s': round(n_lines / e2e, 1),
                                                       'ms': round(e2e * 1e3, 2), 'text_in': 'host'},
        'cpu_baseline': {'value': round(cpu, 1), 'unit': 'lines/s', 'cores': 1, 'kind': 'port',
                         'sample': 'oracle/ingest.shard_traces on the first %d lines' % n_sample},
    }
    print(json.dumps(out))


if __name__ == '__main__':
    main()
