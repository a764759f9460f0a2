#!/usr/bin/env python3
"""GPS probes matched/s (whole node) on the MI355X hot path — BASELINE.json metric.

One step = one pass of the hot path over one batch resident in HBM:
  trace SoA → states → candidates → bounded routing → Viterbi → paths → OSMLR
  segments → report() → simple_reporter hour buckets → [hour][segment][speed-bin]
  histogram, and for N>1 the RCCL reduce-scatter of that histogram over xGMI.

Workload (N=1): SURVEY.md §8d config C2 — synthetic metro graph (1024x1024 street
grid, ~1M nodes, ~3.6M directed edges, seed 2) and 10,000 traces x 100 probes at
15 s sampling with sigma = 10 m noise (seed 2) = 1M probes.  N>1 (config C3 layout):
N x 10,000 traces generated with one seed, sharded by int(sha1(uuid)[:3], 16) % N
(simple_reporter.py:116), graph replicated per GPU, weak scaling.

Launch:  python bench.py [--gpus N --steps K --warmup W]
  N>1:   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
ROUTE_KERNEL = 'k_route<160, 2>'  # first-tier search kernel (rocprofv3 name)
# HBM bytes per ROUTE_KERNEL launch from the FETCH_SIZE / WRITE_SIZE passes of
# tools/profile_gpu.sh (separate --pmc runs of this same command; tools/pmc_summary.py)
PMC_SUMMARY = os.path.join(ROOT, 'profiles', 'r01_v31_pmc.json')
T_BEGIN = 1483228800


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def route_bytes(c):
    """Algorithmic HBM bytes of one first-tier k_route launch, from the
    device work counters: 64 B per task (task record, step metadata, root lookup),
    32 B per settled node (its adjacency record), 16 B per source candidate
    (edge, fraction, length), 20 B per target read (edge, fraction, src, length),
    4 B per transition entry written (route length in mm, u32; v26 — 8 B fp64 costs before)."""
    tasks, settled, trans, targets, sources = c[5], c[3], c[6], c[11], c[12]
    return 64 * tasks + 32 * settled + 16 * sources + 20 * targets + 4 * trans


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--traces-per-gpu', type=int, default=10000)
    ap.add_argument('--cpu-traces', type=int, default=6000, help='bounded oracle sample (0 = skip)')
    ap.add_argument('--cpu-threads', type=int, default=16)
    ap.add_argument('--delta', type=float, default=None, help='routing round width (perf knob, metres)')
    ap.add_argument('--streams', type=int, default=2,
                    help='matchers (one HIP stream + host thread each) sharing the batch')
    ap.add_argument('--workload', choices=['c2', 'c4', 'c5mix'], default='c2',
                    help='c2 (default, the headline): 100 probes @15 s, sigma 10 m; c4: 60 probes @60 s, '
                         'sigma 50 m, accuracy 50 m, search radius 200 m; c5mix: C2 with the C5 mode mix '
                         '(60%% auto / 25%% bicycle / 15%% pedestrian) on the metro graph')
    ap.add_argument('--tiles', type=int, default=0,
                    help='privacy > 0: the step also runs the device tile stage (K9 rows, K10 sort + cull, '
                         'simple_reporter.py:176-239) on each matcher (not part of the headline config)')
    args = ap.parse_args()

    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    import torch
    import torch.distributed as dist
    # OTR_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on one GPU
    # (RCCL refuses two ranks per device); the histogram exchange is then an all-reduce
    # whose owner slice equals the reduce-scatter output
    backend = os.environ.get('OTR_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            if backend == 'nccl':
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()

    from reporter_amd import _lib
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    if not os.path.exists(_lib.LIB_PATH):
        raise SystemExit('libotr.so missing: run python __graft_entry__.py build first')

    gdir = os.path.join(ROOT, 'build', 'graphs')
    if rank == 0:
        gpath = gen.graph_path('metro', gdir)
    barrier()
    gpath = gen.graph_path('metro', gdir)

    # traces: all ranks generate the same global set, keep their uuid-hash shard
    n_global = args.traces_per_gpu * world
    t0 = time.time()
    # match_options as generate_test_trace.py:44-52 sends them (turn_penalty_factor 0,
    # gps_accuracy = the 95th percentile of the noise); max_route_time_factor stays the
    # deployed 2 (Dockerfile:17)
    gtt = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
    W = {'c2': dict(points=100, rate=15, sigma=10.0, seed=2, bike=0.0, ped=0.0, acc=None,
                    meili=dict(gtt, search_radius=50, gps_accuracy=16.45)),
         'c4': dict(points=60, rate=60, sigma=50.0, seed=4, bike=0.0, ped=0.0, acc=50.0,
                    meili=dict(gtt, search_radius=200, max_search_radius=200, gps_accuracy=82.24)),
         'c5mix': dict(points=100, rate=15, sigma=10.0, seed=5, bike=0.25, ped=0.15, acc=None,
                       meili=dict(gtt, search_radius=50, gps_accuracy=16.45))}[args.workload]
    allt = gen.make_traces(gpath, n_global, W['points'], W['rate'], W['sigma'], W['seed'], W['bike'], W['ped'],
                           W['acc'], t_begin=T_BEGIN, t_spread=1800)
    if world > 1:
        shard = np.array([int(hashlib.sha1(u.encode()).hexdigest()[:3], 16) % world for u in allt.uuids])
        mine = allt.subset(np.flatnonzero(shard == rank))
    else:
        mine = allt
    log('rank %d: %d traces, %d probes (gen %.1fs)' % (rank, mine.n_traces, mine.n_probes, time.time() - t0))

    cfg = M.default_config(gpath, device=local, **W['meili'])
    if args.delta is not None:
        cfg['otr']['delta'] = args.delta
    M.configure(cfg)
    n_nodes, n_edges, n_segments = M.graph_info()

    # one matcher per host thread, each on its own HIP stream, each with a contiguous
    # slice of this GPU's traces (reporter_service.py:51-52: one matcher per thread)
    from concurrent.futures import ThreadPoolExecutor
    ns = max(1, args.streams)
    cuts = np.linspace(0, mine.n_traces, ns + 1).astype(np.int64)
    parts = [mine.subset(np.arange(cuts[k], cuts[k + 1])) for k in range(ns)]
    matchers = [M.Matcher() for _ in range(ns)]
    dev = torch.device('cuda', local)
    hours = 3  # traces start within 30 min of T_BEGIN and last 25 min
    hist_len = hours * n_segments * _lib.HIST_BINS
    hist_len += (-hist_len) % world
    keep, darrs, hists = [], [], []
    for part in parts:
        t = [torch.from_numpy(x).to(dev) for x in (part.offsets, part.lat, part.lon, part.time, part.mode)]
        da = {'trace_offsets': t[0].data_ptr(), 'lat': t[1].data_ptr(), 'lon': t[2].data_ptr(),
              'time': t[3].data_ptr(), 'mode': t[4].data_ptr()}
        if part.accuracy is not None:
            t.append(torch.from_numpy(np.ascontiguousarray(part.accuracy, np.float32)).to(dev))
            da['accuracy'] = t[-1].data_ptr()
        keep.append(t)
        darrs.append(da)
        hists.append(torch.zeros(hist_len, dtype=torch.int32, device=dev))
    hist = torch.zeros(hist_len, dtype=torch.int32, device=dev)
    hist_out = torch.zeros(hist_len // world, dtype=torch.int32, device=dev)
    pool = ThreadPoolExecutor(max_workers=ns)
    from reporter_amd import simple_reporter as sr
    tile_stats = []
    torch.cuda.synchronize()

    def run_part(k):
        r = matchers[k].match_batch(parts[k], device_arrays=darrs[k], hist_device=hists[k].data_ptr(),
                                    hist_hours=hours, hist_base_time=T_BEGIN, copy_out=False, timing=True,
                                    tile_rows=args.tiles > 0)
        if r.status != 0:
            raise RuntimeError('batch status %d (%d overflow tasks)' % (r.status, r.n_overflow_traces))
        if args.tiles > 0:
            tc = time.perf_counter()
            kept = sr.cull_rows(matchers[k], None, args.tiles, device_ptr=r.d_rows, n=r.n_rows)
            tile_stats.append((int(r.n_rows), len(kept), time.perf_counter() - tc))
        return r

    def step():
        rs = list(pool.map(run_part, range(ns)))
        torch.sum(torch.stack(hists), dim=0, out=hist)  # combine the per-stream histograms
        if world > 1 and backend == 'nccl':
            dist.reduce_scatter_tensor(hist_out, hist, op=dist.ReduceOp.SUM)
        elif world > 1:
            hc = hist.cpu()
            dist.all_reduce(hc, op=dist.ReduceOp.SUM)
            hist_out.copy_(hc[rank * hist_out.numel():(rank + 1) * hist_out.numel()])
        torch.cuda.current_stream().synchronize()
        return rs

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    t_start = time.perf_counter()
    route_ms, results = [], []
    for _ in range(args.steps):
        rs = step()
        route_ms.extend(r.kernel_ms[_lib.STAGES.index('route')] for r in rs)
        results.append(rs)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    probes = torch.tensor([float(mine.n_probes)], dtype=torch.float64, device=dev)
    if world > 1:
        if backend != 'nccl':
            el, probes = el.cpu(), probes.cpu()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(probes, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_probes = float(probes.item())
    value = total_probes * args.steps / elapsed

    rs = results[-1]
    counters = [sum(int(r.counters[k]) for r in rs) for k in range(len(rs[0].counters))]
    stage_ms = {s: round(float(np.mean([r.kernel_ms[i] for r in rs])), 3) for i, s in enumerate(_lib.STAGES)
                if rs[0].kernel_ms[i] > 0}
    route_avg_ms = float(np.mean(route_ms))
    rbytes = route_bytes(counters) / ns  # per launch (each stream launches once per step)
    achieved = rbytes / (route_avg_ms * 1e-3) / 1e9

    traffic = None
    if os.path.exists(PMC_SUMMARY):
        k = json.load(open(PMC_SUMMARY))['kernels'].get(ROUTE_KERNEL, {})
        if 'fetch_bytes_per_launch' in k and 'write_bytes_per_launch' in k:
            traffic = int(k['fetch_bytes_per_launch'] + k['write_bytes_per_launch'])

    cpu = None
    if rank == 0 and world == 1 and args.cpu_traces > 0:
        from oracle import pyoracle as po
        g = po.Graph(gpath)
        sample = mine.subset(np.arange(min(args.cpu_traces, mine.n_traces)))
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        tc = time.perf_counter()
        po.match_batch(g, sample, po.params(**{k: float(v) for k, v in W['meili'].items()}), threads=threads)
        dt = time.perf_counter() - tc
        cpu = {'value': round(sample.n_probes / dt, 1), 'unit': 'probes/s', 'cores': threads, 'kind': 'port',
               'sample': '%d traces x %d probes of the same %s workload through oracle/liboracle.so '
                         '(scalar C restatement, %d pthreads, %.1f s)' % (sample.n_traces, W['points'],
                                                                          args.workload.upper(), threads, dt)}

    if rank == 0:
        line = {
            'metric': 'GPS probes matched/sec (whole node)',
            'value': round(value, 1),
            'unit': 'probes/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(1e3 * elapsed / args.steps, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic',
            'config': {'workload': '%s: metro street grid (%d nodes, %d directed edges, %d OSMLR segments), '
                                   '%d traces x %d probes per GPU @%d s, sigma %g m%s' % (
                                       args.workload.upper(), n_nodes, n_edges, n_segments, args.traces_per_gpu,
                                       W['points'], W['rate'], W['sigma'],
                                       {'c2': '', 'c4': ', accuracy 50 m, search radius 200 m',
                                        'c5mix': ', modes 60% auto / 25% bicycle / 15% pedestrian'}[args.workload]),
                       'probes_per_step': int(total_probes),
                       'parallelism': ('uuid-sharded dp%d + ' + ('RCCL reduce-scatter' if backend == 'nccl' else 'gloo all-reduce (rehearsal)') + ' of [hour][segment][speed] histogram')
                                      % world if world > 1 else 'single GPU',
                       'streams': ns,
                       'stage_ms_per_stream': stage_ms,
                       'tile_stage': ({'privacy': args.tiles, 'rows': tile_stats[-1][0], 'kept': tile_stats[-1][1],
                                       'ms': round(1e3 * tile_stats[-1][2], 3)} if tile_stats else None),
                       'work': {'states': int(sum(r.n_states for r in rs)), 'grid_cells': int(counters[0]),
                                'shape_segments_tested': int(counters[1]), 'candidates': int(counters[2]),
                                'output_segments': int(counters[7])}},
            'roofline': {'kernel': ROUTE_KERNEL + ' (K3 bounded one-to-many searches, 2 per wave + K4 transition)',
                         'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / PEAK_HBM_GBS, 4), 'traffic': traffic,
                         'traffic_source': os.path.relpath(PMC_SUMMARY, ROOT) if traffic else None,
                         'launch_ms': round(route_avg_ms, 3), 'algorithmic_bytes': int(rbytes),
                         'settled_nodes': int(counters[3]), 'relaxed_edges': int(counters[4]),
                         'tasks': int(counters[5]), 'transition_entries': int(counters[6]),
                         'source_candidates': int(counters[12]),
                         'retry_settled_nodes': int(counters[9]), 'search_rounds': int(counters[13]),
                         'table_keys': int(counters[14]),
                         'tasks_keys_gt': {'64': int(counters[22]), '96': int(counters[15]), '128': int(counters[23])},
                         'phase_cycles': [int(x) for x in counters[16:22]] if ('stamps' in _lib.LIB_PATH or 'cstamp' in _lib.LIB_PATH) else None},
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
