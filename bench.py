#!/usr/bin/env python3
"""GPS probes matched/s (whole node) on the MI355X hot path — BASELINE.json metric.

One step = one pass of the hot path over one batch resident in HBM:
  trace SoA → states → candidates → bounded routing → Viterbi → paths → OSMLR
  segments → report() → simple_reporter hour buckets → [hour][segment][speed-bin]
  histogram, and for N>1 the RCCL reduce-scatter of that histogram over xGMI.

Workload (N=1): SURVEY.md §8d config C2 — synthetic metro graph (1024x1024 street
grid, ~1M nodes, ~3.5M directed edges, seed 2) and 10,000 traces x 100 probes at
15 s sampling with sigma = 10 m noise (seed 2) = 1M probes, matched with the match_options
generate_test_trace.py:44-52 sends (turn_penalty_factor 0) under the deployed
max_route_time_factor 2 (Dockerfile:17).  N>1: BASELINE config 3 (C3) — 1,000,000
"veh%07d" uuids x 100 probes = 100M probes per step node-wide, sharded by
int(sha1(uuid)[:3], 16) % N (simple_reporter.py:116), the graph replicated per GPU, each
GPU matching its ~1M/N traces in device batches of --chunk-traces (strong scaling: the
total is fixed), then the keyed histogram exchange.

Besides the timed device-resident line the bench reports, for rank 0 at N=1:
  * roofline: the dominant route-search kernel of the workload (largest device time):
    SURVEY §8(d) algorithmic bytes (K3: 24 B per settled node + 16 B per relaxed edge;
    K4: 8 B per transition entry) ÷ its HIP-event time on the matcher's stream;
  * parity: the oracle sample matched on the CPU compared bit-exactly with the GPU
    output for the same traces of this batch (the line fails on a mismatch);
  * cpu_baseline: that oracle sample's rate on the host cores the process may use;
  * end_to_end: the SoA input in pinned host memory → H2D → match → reports and the
    histogram back on the host (SURVEY §8(d)'s drop-in definition; PCIe included).

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
T_BEGIN = 1483228800
# HBM bytes per launch of the dominant kernel from separate FETCH_SIZE / WRITE_SIZE
# --pmc passes of this command (tools/profile_gpu.sh, tools/pmc_summary.py), when the
# committed summary holds the kernel
PMC_SUMMARY = os.environ.get('OTR_PMC_SUMMARY', os.path.join(ROOT, 'profiles', 'r04_final_pmc.json'))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def kernel_name(code, turns=False, first=False):
    """rocprofv3 name of a route kernel (otr_batch_result.route_tier_code); turns: kept for
    callers (turn-mode tasks run in the edge-state kernels: code 6,000,000 + CAP * 100 + targets)."""
    if code < 0:  # the global-memory search: -1 on 32K-state slabs, -2 on 1M-state slabs
        return 'k_general' if code == -1 else 'k_general (1M-state slabs)'
    if 6000000 <= code < 7000000:  # the lean edge-state tiers: 6,000,000 + CAP * 100 + targets
        return 'k_route_e1<%d>' % ((code - 6000000) // 100)
    # the timed launches run the LDS route kernels compiled without work counting (the
    # last template argument, CNT = false; the instrumented step runs CNT = true)
    if 900000 <= code < 1000000:  # the 64-bit label tier: 900,000 + CAP
        return 'k_route<%d, 1, true, true, false>' % (code - 900000)
    cap, g = code // 10, code % 10
    return 'k_route<%d, %d, %s, false, false>' % (cap, g, 'false' if first else 'true')


def route_bytes(work):
    """SURVEY.md §8(d) algorithmic bytes of one route-search launch: K3 per source search
    16 B per settled node (row pointer + coordinates) + 8 B per settled node (its label)
    + 16 B per relaxed edge (dst, length, access, osmlr); K4 8 B per transition entry."""
    searches, settled, relaxed, trans = work
    return 24 * settled + 16 * relaxed + 8 * trans


def local_ranks():
    """Ranks of this job on this host (torch.distributed.run sets LOCAL_WORLD_SIZE)."""
    return int(os.environ.get('LOCAL_WORLD_SIZE', os.environ.get('WORLD_SIZE', 1)))


def usable_cores():
    """Host cores this process may use: its CPU affinity, capped by a cgroup CPU quota
    (cpu.max), which a shared GPU box sets below the machine's core count."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    for path in ('/sys/fs/cgroup/cpu.max',):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != 'max':
                n = min(n, max(1, int(int(quota) / int(period))))
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        if q > 0:
            n = min(n, max(1, q // p))
    except (OSError, ValueError):
        pass
    return n


class _DevBytes:
    """A device byte range (library-owned) as a torch tensor view, without a copy."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {'shape': (int(nbytes),), 'typestr': '|u1', 'data': (int(ptr), False),
                                         'version': 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--traces-per-gpu', type=int, default=None,
                    help='default: 10,000 (c2, c5mix), 20,000 (c4: BASELINE C4); c3: every owned uuid')
    ap.add_argument('--cpu-traces', type=int, default=None,
                    help='bounded oracle sample for the CPU baseline and the parity check (0 = skip)')
    ap.add_argument('--delta', type=float, default=None, help='routing round width (perf knob, metres)')
    ap.add_argument('--streams', type=int, default=1,
                    help='matchers (one HIP stream + host thread each) sharing the batch; 2 overlaps one '
                         "stream's host syncs and kernel tails with the other's kernels (+1.6%% at C2) but "
                         'the two route launches then share the GPU, halving the per-launch roofline figure')
    ap.add_argument('--chunk-traces', type=int, default=125000,
                    help='traces per device batch (a shard larger than this is matched in several batches per '
                         'step; 125,000 = the N = 8 share of C3)')
    ap.add_argument('--workload', choices=['c1', 'c2', 'c2dep', 'c3', 'c4', 'c5mix', 'c5'], default=None,
                    help='default: c2 at N = 1, c3 at N > 1.  c1: the city graph, 1,000 traces x 300 probes @1 s, '
                         'sigma 5 m (BASELINE config 1); c2 (the headline): 100 probes @15 s, sigma 10 m; '
                         'c2dep: the same traces '
                         'matched with the deployed configuration only (what Batch.java requests get: mode '
                         'defaults, turn penalties auto 200 / bicycle 140 / pedestrian 100); c3: the C3 shard of '
                         '1M veh%%07d uuids x 100 probes this GPU owns; c4: 60 probes @60 s, sigma 50 m, '
                         'accuracy 50 m, search radius 200 m; c5mix: C2 with the C5 mode mix '
                         '(60%% auto / 25%% bicycle / 15%% pedestrian) on the metro graph; c5: the country graph '
                         '(50M nodes), this GPU\'s N = 8 share (125,000) of 1M vehicles over 24 h, C5 mode mix')
    ap.add_argument('--e2e-steps', type=int, default=3, help='host-to-host drop-in steps (0 = skip)')
    ap.add_argument('--json-traces', type=int, default=2000,
                    help='traces of the JSON drop-in leg (Batch.java bodies; 0 = skip)')
    ap.add_argument('--e2e-streams', type=int, default=2,
                    help='worker threads (matchers, HIP streams, pinned batches) of the host-to-host measurement')
    ap.add_argument('--opt', action='append', default=[],
                    help='A/B only (not the headline config): KEY=VALUE match option override, e.g. '
                         'max_route_time_factor=0')
    ap.add_argument('--hist', choices=['keyed', 'dense'], default='keyed',
                    help='keyed (default, SURVEY 8e): tile rows (K9) sort-reduced per GPU into (hour-tile file, '
                         'segment pair, speed bin) counts, all-to-all to the (hour, tile) owner, owner merge + '
                         'privacy cull; dense: the [hour][segment][speed] K8 histogram reduce-scattered')
    ap.add_argument('--privacy', type=int, default=2,
                    help='owner-side pair cull threshold of the keyed histogram (simple_reporter.py:345 default)')
    ap.add_argument('--tiles', type=int, default=0,
                    help='privacy > 0: the step also runs the device tile stage (K9 rows, K10 sort + cull, '
                         'simple_reporter.py:176-239) on each matcher (not part of the headline config)')
    ap.add_argument('--dist', action='store_true',
                    help='run the N > 1 path (process group, uuid shards, keyed all-to-all exchange to the '
                         '(hour, tile) owner) even at N = 1: RCCL at world size 1 on one GPU')
    args = ap.parse_args()

    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    # the distributed path: every N > 1 run, and N = 1 with --dist (RCCL at world size 1)
    dist_on = world > 1 or args.dist
    if args.workload is None:  # the headline at N = 1; BASELINE config 3 across GPUs
        args.workload = 'c2' if not dist_on else 'c3'
    import torch
    import torch.distributed as dist
    # OTR_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on one GPU
    # (RCCL refuses two ranks per device); the histogram exchange is then an all-reduce
    # whose owner slice equals the reduce-scatter output
    backend = os.environ.get('OTR_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if dist_on:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29531')
        os.environ.setdefault('RANK', str(rank))
        os.environ.setdefault('WORLD_SIZE', str(world))
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)

    def barrier():
        if dist_on:
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
    gname = {'c5': 'country', 'c1': 'city'}.get(args.workload, 'metro')
    if rank == 0:
        tg = time.time()
        gpath = gen.graph_path(gname, gdir)
        log('graph %s ready (%.1fs)' % (gname, time.time() - tg))
    barrier()
    gpath = gen.graph_path(gname, gdir)

    # match_options as generate_test_trace.py:44-52 sends them (turn_penalty_factor 0,
    # gps_accuracy = the 95th percentile of the noise); max_route_time_factor stays the
    # deployed 2 (Dockerfile:17)
    gtt = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000}
    # C1: generate_test_trace.py's 1 Hz traces with 5 m noise on the city graph,
    # gps_accuracy = round(min(100, 1.645 * max(1, 5)), 2) = 8.22
    W = {'c1': dict(points=300, rate=1, sigma=5.0, seed=1, bike=0.0, ped=0.0, acc=None, traces=1000,
                    meili=dict(gtt, search_radius=50, gps_accuracy=8.22)),
         'c2': dict(points=100, rate=15, sigma=10.0, seed=2, bike=0.0, ped=0.0, acc=None, traces=10000,
                    meili=dict(gtt, search_radius=50, gps_accuracy=16.45)),
         # the deployed configuration (Dockerfile:14-17,42-49 + the per-mode defaults): a
         # Batch.java request carries only mode and levels (Batch.java:56-65)
         'c2dep': dict(points=100, rate=15, sigma=10.0, seed=2, bike=0.0, ped=0.0, acc=None, traces=10000,
                       meili={}),
         'c3': dict(points=100, rate=15, sigma=10.0, seed=3, bike=0.0, ped=0.0, acc=None, traces=None,
                    meili=dict(gtt, search_radius=50, gps_accuracy=16.45)),
         'c4': dict(points=60, rate=60, sigma=50.0, seed=4, bike=0.0, ped=0.0, acc=50.0, traces=20000,
                    meili=dict(gtt, search_radius=200, max_search_radius=200, gps_accuracy=82.24)),
         'c5mix': dict(points=100, rate=15, sigma=10.0, seed=5, bike=0.25, ped=0.15, acc=None, traces=10000,
                       meili=dict(gtt, search_radius=50, gps_accuracy=16.45)),
         # C5: the country graph, 1M vehicles' traces over 24 h with the 60/25/15 mode mix,
         # uuid-sharded like C3; per GPU the N = 8 share (125,000 traces, 12.5M probes)
         'c5': dict(points=100, rate=15, sigma=10.0, seed=5, bike=0.25, ped=0.15, acc=None, traces=125000,
                    spread=86400, meili=dict(gtt, search_radius=50, gps_accuracy=16.45))}[args.workload]

    for kv in args.opt:
        k, v = kv.split('=', 1)
        W['meili'][k] = float(v)
    t0 = time.time()
    if args.workload in ('c3', 'c5'):
        # C3 / C5: 1,000,000 uuids "veh%07d" x 100 probes, sharded by
        # int(sha1(uuid)[:3], 16) % N (simple_reporter.py:116); each rank generates only the
        # uuids it owns (a uuid's trace is seeded by its number, so shards are independent).
        # --traces-per-gpu bounds the uuids per rank (C3: a one-GPU rehearsal; C5: the
        # N = 8 share by default).
        n_uuid = 1000000
        owner = np.array([int(hashlib.sha1(('veh%07d' % u).encode()).hexdigest()[:3], 16) % world
                          for u in range(n_uuid)])
        mine_ids = np.flatnonzero(owner == rank)
        cap = args.traces_per_gpu or W['traces']
        if cap:
            mine_ids = mine_ids[:cap]
        mine = gen.make_traces_ids(gpath, mine_ids, W['points'], W['rate'], W['sigma'], W['seed'], W['bike'],
                                   W['ped'], W['acc'], t_begin=T_BEGIN, t_spread=W.get('spread', 1800),
                                   threads=max(1, min(16, usable_cores() // max(1, local_ranks()))))
    else:
        n_per = args.traces_per_gpu or W['traces']
        n_global = n_per * world
        allt = gen.make_traces(gpath, n_global, W['points'], W['rate'], W['sigma'], W['seed'], W['bike'],
                               W['ped'], W['acc'], t_begin=T_BEGIN, t_spread=1800)
        if dist_on:
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
    # device batches: contiguous slices of this GPU's traces, at most --chunk-traces each, at
    # least one per stream; stream k matches batches k, k + ns, ... in turn
    n_parts = max(ns, -(-mine.n_traces // max(1, args.chunk_traces)))
    n_parts += (-n_parts) % ns
    cuts = np.linspace(0, mine.n_traces, n_parts + 1).astype(np.int64)
    parts = [mine.slice(int(cuts[k]), int(cuts[k + 1])) for k in range(n_parts)]
    matchers = [M.Matcher() for _ in range(ns)]
    dev = torch.device('cuda', local)
    # dense histogram hours: traces start within `spread` of T_BEGIN and last <= 100 min
    hours = (W.get('spread', 1800) + W['points'] * W['rate']) // 3600 + 2
    if args.hist == 'dense' and args.workload == 'c5':
        raise SystemExit('bench: the dense [hour][segment][speed] histogram of C5 would take %d GB; use --hist keyed'
                         % (hours * 60 * 8 * 4 // 1000))
    keyed = args.hist == 'keyed'
    if not keyed and n_parts > ns:
        raise SystemExit('bench: the dense histogram takes one device batch per stream; use --hist keyed')
    # the dense histogram's tensors exist only in dense mode (C5's would be 4 x 51 GB)
    hist_len = hours * n_segments * _lib.HIST_BINS if not keyed else world
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

    EW = _lib.HIST_ENTRY.itemsize
    ebufs = [torch.zeros(0, dtype=torch.uint8, device=dev) for _ in range(n_parts)]  # per-batch local entries
    n_local, n_rows, row_views = [0] * n_parts, [0] * n_parts, [None] * n_parts
    hist_stats = {}
    # one batch per stream on one GPU: its single owner reduces the rows themselves
    rows_direct = keyed and not dist_on and n_parts == ns

    def run_one(k, j, route_work):
        r = matchers[k].match_batch(parts[j], device_arrays=darrs[j],
                                    hist_device=None if keyed else hists[k].data_ptr(),
                                    hist_hours=0 if keyed else hours, hist_base_time=T_BEGIN, copy_out=False,
                                    timing=True, tile_rows=keyed or args.tiles > 0, route_work=route_work)
        if r.status != 0:
            raise RuntimeError('batch status %d (%d traces beyond every search tier)' % (r.status,
                                                                                          r.n_overflow_traces))
        n_rows[j] = int(r.n_rows)
        if rows_direct:
            row_views[j] = (torch.as_tensor(_DevBytes(r.d_rows, int(r.n_rows) * _lib.TILE_ROW.itemsize), device=dev)
                            if int(r.n_rows) > 0 else torch.zeros(0, dtype=torch.uint8, device=dev))
        elif keyed:  # this batch's (file, pair, speed bin) counts, on the matcher's stream
            if ebufs[j].numel() < int(r.n_rows) * EW:
                ebufs[j] = torch.empty(int(r.n_rows) * EW * 5 // 4 + EW, dtype=torch.uint8, device=dev)
            n_local[j] = sr.hist_reduce(matchers[k], r.d_rows, r.n_rows, privacy=1, rows_in=True,
                                        out=ebufs[j].data_ptr())
        if args.tiles > 0:
            tc = time.perf_counter()
            kept = sr.cull_rows(matchers[k], None, args.tiles, device_ptr=r.d_rows, n=r.n_rows)
            tile_stats.append((int(r.n_rows), len(kept), time.perf_counter() - tc))
        return r

    def run_part(k, route_work=False):
        # (each result keeps its own counters and times; its rows were consumed in run_one)
        return [run_one(k, j, route_work) for j in range(k, n_parts, ns)]

    owned = {'buf': torch.zeros(0, dtype=torch.uint8, device=dev), 'n': 0}

    def keyed_exchange():
        """§8e: the batches' entries → all-to-all by (hour, tile) owner → the owner's
        merge + privacy cull (one more sort-reduce, on the first matcher's stream)."""
        torch.cuda.synchronize()
        if rows_direct:
            rows = torch.cat(row_views)
            n_in = rows.numel() // _lib.TILE_ROW.itemsize
            if owned['buf'].numel() < max(n_in, 1) * EW:
                owned['buf'] = torch.empty(max(n_in, 1) * EW * 5 // 4, dtype=torch.uint8, device=dev)
            owned['n'] = sr.hist_reduce(matchers[0], rows.data_ptr(), n_in, privacy=args.privacy, rows_in=True,
                                        out=owned['buf'].data_ptr())
            hist_stats.update(rows=int(sum(n_rows)), owned=int(owned['n']))
            return
        local_e = torch.cat([ebufs[j][:n_local[j] * EW] for j in range(n_parts)])
        if dist_on:
            tx = time.perf_counter()
            send = local_e if backend == 'nccl' else local_e.cpu()
            recv = sr.exchange_hist(send, world)
            recv = recv if recv.is_cuda else recv.to(dev)
            torch.cuda.synchronize()
            hist_stats.update(exchange_ms=round(1e3 * (time.perf_counter() - tx), 3),
                              exchange_bytes_sent=int(local_e.numel()), exchange_bytes_received=int(recv.numel()))
        else:
            recv = local_e
        n_in = recv.numel() // EW
        if owned['buf'].numel() < max(n_in, 1) * EW:
            owned['buf'] = torch.empty(max(n_in, 1) * EW * 5 // 4, dtype=torch.uint8, device=dev)
        owned['n'] = sr.hist_reduce(matchers[0], recv.data_ptr(), n_in, privacy=args.privacy,
                                    out=owned['buf'].data_ptr())
        hist_stats.update(rows=int(sum(n_rows)), local_entries=int(sum(n_local)), received=int(n_in),
                          owned=int(owned['n']))

    split = {}

    def step(route_work=False):
        hist_stats.clear()
        t0 = time.perf_counter()
        rs = [r for rk in pool.map(lambda k: run_part(k, route_work), range(ns)) for r in rk]
        t1 = time.perf_counter()
        if keyed:
            keyed_exchange()
            torch.cuda.current_stream().synchronize()
            split.update(match=round(1e3 * (t1 - t0), 3), histogram=round(1e3 * (time.perf_counter() - t1), 3))
            return rs
        torch.sum(torch.stack(hists), dim=0, out=hist)  # combine the per-stream histograms
        if dist_on and backend == 'nccl':
            dist.reduce_scatter_tensor(hist_out, hist, op=dist.ReduceOp.SUM)
        elif dist_on:
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
    results = []
    for _ in range(args.steps):
        results.append(step())
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    timed_split = dict(split)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    probes = torch.tensor([float(mine.n_probes)], dtype=torch.float64, device=dev)
    if dist_on:
        if backend != 'nccl':
            el, probes = el.cpu(), probes.cpu()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(probes, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_probes = float(probes.item())
    value = total_probes * args.steps / elapsed

    # ---- per-kernel device time over the timed steps (every stream, every step); the work
    # each kernel did comes from one more, instrumented step over the same batch (the
    # route kernels count their work only on request, OTR_BATCH_ROUTE_WORK: the counting
    # itself costs ~7% of the first tier).  The path is deterministic, so the counts are
    # those of every timed step (the bench checks the output segment counts agree).
    rs = results[-1]
    work_rs = step(route_work=True)
    barrier()
    counters = [sum(int(r.counters[k]) for r in work_rs) for k in range(len(rs[0].counters))]
    if [int(r.counters[7]) for r in work_rs] != [int(r.counters[7]) for r in rs]:
        raise RuntimeError('instrumented step differs from the timed steps')
    work_of = {}
    for r in work_rs:
        for t in range(len(r.route_tier_code)):
            if int(r.route_tier_code[t]) != 0:
                w = work_of.setdefault(t, np.zeros(4, np.int64))
                w += np.array([int(x) for x in r.route_tier_work[t]], np.int64)
    stage_ms = {s: round(float(np.sum([r.kernel_ms[i] for r in rs])) / ns, 3) for i, s in enumerate(_lib.STAGES)
                if rs[0].kernel_ms[i] > 0}
    tiers = {}
    for step_rs in results:
        for r in step_rs:
            for t in range(len(r.route_tier_code)):
                code = int(r.route_tier_code[t])
                if code == 0:
                    continue
                d = tiers.setdefault(t, {'code': code, 'launches': 0, 'ms': 0.0, 'work': np.zeros(4, np.int64)})
                d['launches'] += 1
                d['ms'] += float(r.route_tier_ms[t])
    for t, d in tiers.items():  # per-launch work of the instrumented step, times the launches
        d['work'] = work_of.get(t, np.zeros(4, np.int64)) * (d['launches'] // max(1, n_parts))
    dom_t = max(tiers, key=lambda t: tiers[t]['ms'])
    dom = tiers[dom_t]
    launch_ms = dom['ms'] / dom['launches']
    dom_bytes = route_bytes(dom['work'] / dom['launches'])
    achieved = dom_bytes / (launch_ms * 1e-3) / 1e9
    # turn-cost modes run the route kernels compiled with the turn walk
    turns = float(W['meili'].get('turn_penalty_factor', 1.0)) > 0.0
    tier_table = {kernel_name(d['code'], turns, t in (0, 12, 13)): {'ms_per_launch': round(d['ms'] / d['launches'], 3),
                                          'searches_per_launch': int(d['work'][0] // d['launches']),
                                          'settled_per_launch': int(d['work'][1] // d['launches']),
                                          'relaxed_per_launch': int(d['work'][2] // d['launches']),
                                          'transitions_per_launch': int(d['work'][3] // d['launches']),
                                          'gbs': round(route_bytes(d['work'] / d['launches']) /
                                                       (max(d['ms'], 1e-9) / d['launches'] * 1e-3) / 1e9, 1)}
                  for t, d in sorted(tiers.items())}
    traffic, traffic_src, l2_hit = None, None, None
    from reporter_amd.build import source_hash
    build_id = '%s:%s' % (source_hash(), os.path.basename(os.environ.get('OTR_LIB') or 'libotr.so'))
    # FETCH_SIZE + WRITE_SIZE of the dominant kernel from the committed PMC summary of this
    # workload's bench command (tools/profile_set.sh + tools/profile_summary.py:
    # profiles/<round>_pmc_<workload>.json; OTR_PMC_SUMMARY overrides)
    psum = PMC_SUMMARY if os.environ.get('OTR_PMC_SUMMARY') else None
    if psum is None:
        import glob
        cands = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_pmc_%s.json' % args.workload)))
        psum = cands[-1] if cands else (PMC_SUMMARY if args.workload == 'c2' else None)
    # (only a summary recorded from this build: same sources, the product library)
    if psum and os.path.exists(psum) and args.streams == 1:
        pj = json.load(open(psum))
        k = pj.get('kernels', {}).get(kernel_name(dom['code'], turns, dom_t in (0, 12, 13)), {})
        if pj.get('build') != build_id:
            k = {}
            traffic_src = 'null: %s was recorded from build %s, this run is %s' % (
                os.path.relpath(psum, ROOT), pj.get('build'), build_id)
        if 'fetch_bytes_per_launch' in k and 'write_bytes_per_launch' in k:
            traffic = int(k['fetch_bytes_per_launch'] + k['write_bytes_per_launch'])
            traffic_src = os.path.relpath(psum, ROOT)
            l2_hit = k.get('l2_hit')

    # ---- rank 0: oracle sample (CPU baseline) and its bit-exact comparison, on rank 0's
    # own shard at every N (after the timed region; the other ranks wait at the closing
    # barrier), so a multi-GPU line carries its own parity evidence
    cpu, parity = None, None
    n_cpu = args.cpu_traces if args.cpu_traces is not None else {'c1': 1000, 'c2': 6000, 'c2dep': 2000, 'c5mix': 6000,
                                                                 'c4': 600,
                                                                 'c5': 3000, 'c3': 6000}[args.workload]
    if rank == 0 and n_cpu > 0:
        from oracle import pyoracle as po
        from oracle.compare import compare, subset
        g = po.Graph(gpath)
        idx = np.arange(min(n_cpu, mine.n_traces))
        sample = mine.subset(idx)
        threads = usable_cores()
        tc = time.perf_counter()
        want = po.match_batch(g, sample, po.params(**W['meili']), threads=threads)
        dt = time.perf_counter() - tc
        cpu = {'value': round(sample.n_probes / dt, 1), 'unit': 'probes/s', 'cores': threads, 'kind': 'port',
               'sample': '%d traces x %d probes of the same %s workload%s through oracle/liboracle.so '
                         '(scalar C restatement, %d pthreads = the cores this process may use: affinity capped by '
                         'the cgroup CPU quota; os.cpu_count() = %d; %.1f s)' % (
                             sample.n_traces, W['points'], args.workload.upper(),
                             (' (rank 0 shard of %d)' % world) if world > 1 else '', threads, os.cpu_count() or 0,
                             dt)}
        # the GPU output of the same traces (copy-out run, untimed): the whole batch when it
        # is one device batch, else the sample's traces alone (traces are matched independently)
        if n_parts == 1:
            got_full = _lib.result_to_numpy(M.Matcher().match_batch(mine, copy_out=True))
            got = subset(got_full, idx, mine.offsets)
        else:
            got = _lib.result_to_numpy(M.Matcher().match_batch(sample, copy_out=True))
        errors, stats = compare(got, want)
        parity = {'traces': int(sample.n_traces), 'probes': int(sample.n_probes), 'ok': not errors,
                  'segments': stats.get('n_seg'), 'reports': stats.get('n_rep'), 'errors': errors[:3],
                  'floats_bitexact': all(v for k, v in stats.items() if k.endswith('_bitexact'))}

    # ---- rank 0, N = 1: the drop-in path host → host (PCIe included; never `value`).
    # E host threads (--e2e-streams), each a worker of the service with its own matcher (own
    # HIP stream, reporter_service.py:51-52: one matcher per thread) and its own pinned copy
    # of the batch, each running the full batch --e2e-steps times back to back: while one
    # worker's kernels run, another's H2D inputs and D2H reports/entries move on the DMA
    # engines.  Rate = E x steps x probes / wall time.
    e2e = None
    if rank == 0 and world == 1 and args.e2e_steps > 0:
        from concurrent.futures import ThreadPoolExecutor as _TPE
        ne = max(1, args.e2e_streams)
        ematchers = [matchers[k] if k < len(matchers) else M.Matcher() for k in range(ne)]
        harrs, pins = [], []
        for k in range(ne):
            pin = {}
            for name, arr in (('offsets', mine.offsets), ('lat', mine.lat), ('lon', mine.lon), ('time', mine.time),
                              ('mode', mine.mode)):
                pin[name] = torch.from_numpy(np.ascontiguousarray(arr)).pin_memory()
            if mine.accuracy is not None:
                pin['accuracy'] = torch.from_numpy(np.ascontiguousarray(mine.accuracy, np.float32)).pin_memory()
            pins.append(pin)
            harrs.append({'trace_offsets': pin['offsets'].data_ptr(), 'lat': pin['lat'].data_ptr(),
                          'lon': pin['lon'].data_ptr(), 'time': pin['time'].data_ptr(),
                          'mode': pin['mode'].data_ptr(),
                          'accuracy': pin['accuracy'].data_ptr() if 'accuracy' in pin else None})
        hist_hosts = [torch.zeros(hist_len, dtype=torch.int32).pin_memory() for _ in range(ne)] if not keyed else None
        ehists = ([hists[0]] + [torch.zeros_like(hists[0]) for _ in range(ne - 1)]) if not keyed else None
        e2e_out = [None] * ne

        def e2e_one(k):
            m = ematchers[k]
            if not keyed:
                r = m.match_batch(mine, host_arrays=harrs[k], hist_device=ehists[k].data_ptr(), hist_hours=hours,
                                  hist_base_time=T_BEGIN, copy_out=False, copy_reports=True)
                hist_hosts[k].copy_(ehists[k], non_blocking=False)
                e2e_out[k] = (int(r.n_rep), None)
                return
            # keyed: the tile rows reduced and culled in HBM, the owned entries to the host
            r = m.match_batch(mine, host_arrays=harrs[k], copy_out=False, copy_reports=True, tile_rows=True)
            ent = sr.hist_reduce(m, r.d_rows, r.n_rows, privacy=args.privacy, rows_in=True)
            e2e_out[k] = (int(r.n_rep), len(ent))

        def e2e_worker(k, steps):
            for _ in range(steps):
                e2e_one(k)

        epool = _TPE(max_workers=ne)
        list(epool.map(e2e_worker, range(ne), [1] * ne))  # warm every worker
        torch.cuda.synchronize()
        te0 = time.perf_counter()
        list(epool.map(e2e_worker, range(ne), [args.e2e_steps] * ne))
        torch.cuda.synchronize()
        tel = time.perf_counter() - te0
        epool.shutdown()
        e2e = {'value': round(ne * mine.n_probes * args.e2e_steps / tel, 1), 'unit': 'probes/s',
               'ms_per_step': round(1e3 * tel / (ne * args.e2e_steps), 3), 'streams': ne, 'reports': e2e_out[0][0],
               'owned_entries': e2e_out[0][1],
               'what': 'SoA input in pinned host memory -> H2D -> match -> reports (dense, host) and the ' +
                       ('keyed (hour-tile, pair, speed) histogram entries after the privacy cull'
                        if keyed else '[hour][segment][speed] histogram') + ' (host); SURVEY 8(d) drop-in definition' +
                       ("; %d worker threads, one matcher / HIP stream / pinned batch each, one batch's copies "
                        "overlapping another's kernels" % ne if ne > 1 else '')}

    # ---- rank 0, N = 1: the JSON drop-in path as its callers use it (never `value`):
    # Batch.java bodies of this workload's traces, whole and in BatchingProcessor-sized
    # windows, through one otr_report_batch call and through coalesced blocking callers
    # (reporter_amd/tools/dropin.py), with the host split of each
    json_dropin = None
    if rank == 0 and world == 1 and args.json_traces > 0:
        from reporter_amd.tools import dropin
        tj = time.perf_counter()
        json_dropin = dropin.measure(M, matchers[0], mine.slice(0, min(args.json_traces, mine.n_traces)), config=cfg)
        json_dropin['vs_value'] = {
            k: round(json_dropin[g][c]['probes_per_s'] / value, 3)
            for k, g, c in (('whole_batch_call', 'whole_traces', 'batch_c_call'),
                            ('whole_coalesced_256', 'whole_traces', 'coalesced_256_threads'),
                            ('windows_coalesced_256', 'streaming_windows', 'coalesced_256_threads'))}
        log('json drop-in leg %.1f s' % (time.perf_counter() - tj))

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
            'scaling': 'strong' if args.workload == 'c3' and not args.traces_per_gpu else 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic',
            'config': {'workload': '%s: %s street grid (%d nodes, %d directed edges, %d OSMLR segments), '
                                   '%d traces x %d probes per GPU @%d s, sigma %g m%s; %s' % (
                                       args.workload.upper(), gname, n_nodes,
                                       n_edges, n_segments, mine.n_traces,
                                       W['points'], W['rate'], W['sigma'],
                                       {'c1': '', 'c2': '', 'c3': ', C3 uuid shard (1M veh%07d uuids, sha1[:3] % N)',
                                        'c4': ', accuracy 50 m, search radius 200 m',
                                        'c5mix': ', modes 60% auto / 25% bicycle / 15% pedestrian',
                                        'c2dep': '',
                                        'c5': ', 1M veh%07d uuids sha1[:3] % 8 share over 24 h, modes 60% auto / '
                                              '25% bicycle / 15% pedestrian'}[
                                           args.workload],
                                       'the deployed configuration (mode defaults: turn_penalty_factor auto 200, '
                                       'max_route_time_factor 2)' if args.workload == 'c2dep' else
                                       'generate_test_trace match_options, max_route_time_factor 2'),
                       'probes_per_step': int(total_probes),
                       'parallelism': ('uuid-sharded dp%d + ' % world + (
                           ('keyed (hour-tile, pair, speed) entries all-to-all to the tile owner over ' +
                            ('RCCL' if backend == 'nccl' else 'gloo (rehearsal)')) if keyed else
                           (('RCCL reduce-scatter' if backend == 'nccl' else 'gloo all-reduce (rehearsal)') +
                            ' of the dense [hour][segment][speed] histogram'))) if dist_on else 'single GPU',
                       'histogram': ({'kind': 'keyed (SURVEY 8e)', 'privacy': args.privacy, **hist_stats}
                                     if keyed else {'kind': 'dense [hour][segment][speed]'}),
                       'streams': ns,
                       'device_batches': n_parts,
                       'stage_ms_per_stream': stage_ms,
                       # host wall time of the last timed step: the matcher calls (kernels, their
                       # host syncs and copies) and the keyed histogram reduce / exchange
                       'step_wall_ms': timed_split,
                       # one stream, one batch: the step = the matcher's timed stages + the
                       # owner's keyed reduce + what neither covers (host syncs, launches)
                       'step_accounting': ({'stage_sum_ms': round(sum(stage_ms.values()), 3),
                                            'owner_reduce_ms': timed_split.get('histogram'),
                                            'unaccounted_ms': round(1e3 * elapsed / args.steps - sum(stage_ms.values())
                                                                    - (timed_split.get('histogram') or 0.0), 3)}
                                           if ns == 1 and n_parts == 1 and world == 1 else None),
                       'route_kernels': tier_table,
                       'tile_stage': ({'privacy': args.tiles, 'rows': tile_stats[-1][0], 'kept': tile_stats[-1][1],
                                       'ms': round(1e3 * tile_stats[-1][2], 3)} if tile_stats else None),
                       'work': {'states': int(sum(r.n_states for r in rs)), 'grid_cells': int(counters[0]),
                                'shape_segments_tested': int(counters[1]), 'candidates': int(counters[2]),
                                'output_segments': int(counters[7]),
                                # edge-state searches that outgrew a table and went on in the next
                                # one from their HBM dump (otr_edge1.h), turn-cost modes only
                                'edge_searches_dumped': int(counters[23]),
                                'edge_searches_resumed': int(counters[22])}},
            'roofline': {'kernel': kernel_name(dom['code'], turns, dom_t in (0, 12, 13)) + ' (dominant route-search kernel of this workload)',
                         'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / PEAK_HBM_GBS, 4), 'traffic': traffic,
                         'traffic_source': traffic_src, 'l2_hit': l2_hit, 'launch_ms': round(launch_ms, 3),
                         'algorithmic_bytes': int(dom_bytes),
                         'bytes_formula': 'SURVEY 8(d): 24 B x settled + 16 B x relaxed + 8 B x transitions',
                         'searches': int(dom['work'][0] // dom['launches']),
                         'settled_nodes': int(dom['work'][1] // dom['launches']),
                         'relaxed_edges': int(dom['work'][2] // dom['launches']),
                         'transition_entries': int(dom['work'][3] // dom['launches']),
                         'search_rounds': int(counters[13]), 'table_keys': int(counters[14]),
                         # diagnostic build only (OTR_STAMPS, OTR_LIB=libotr_stamps.so): shader
                         # clocks of the first tier's search phases, summed over waves
                         'phase_cycles': ({'pending': int(counters[16]), 'resolved': int(counters[17]),
                                           'partition': int(counters[18]), 'relax': int(counters[19]),
                                           'setup': int(counters[20]), 'rows': int(counters[21])}
                                          if counters[19] else None)},
            'build': build_id,
            'cpu_baseline': cpu,
            'parity': parity,
            'end_to_end': e2e,
            'json_dropin': json_dropin,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.barrier()  # rank 0's oracle sample and line come after the timed region
        dist.destroy_process_group()
    # a parity failure ends rank 0 with an error only after the other ranks left the barrier
    if rank == 0 and parity is not None and not parity['ok']:
        raise SystemExit('bench: GPU output differs from the oracle sample: %s' % parity['errors'])


if __name__ == '__main__':
    main()
