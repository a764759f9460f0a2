#!/usr/bin/env python3
"""Summary of one workload of tools/profile_set.sh: per kernel the launches and average
duration (kernel trace; the full-size launches: the kernel's largest grid), FETCH_SIZE and WRITE_SIZE per launch (their own --pmc passes,
KiB counters -> bytes; gfx950: the raw sum, see DESIGN.md §4 on the calibration), the
L2 (TCC) hit rate, and measured HBM GB/s = (fetch + write) / duration against 8 TB/s.

  python tools/profile_summary.py gpurun_out/r05p/c2dep > profiles/r05_pmc_c2dep.json
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

PEAK_GBS = 8000.0


def short(name):
    name = re.sub(r'^void ', '', name)
    name = re.sub(r'\(.*$', '', name)
    return re.sub(r'^otr::', '', name)


def find(d, suffix):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(suffix):
                return os.path.join(root, f)
    return None


def per_dispatch(path, names):
    """{kernel: ({counter: average over the kernel's full-size dispatches}, dispatches)}: one
    row per dispatch and counter (rocprofv3 csv).  Full size: the kernel's largest grid (the
    bench batch; the bench's smaller launches — the JSON drop-in leg, oracle samples — are
    left out so the per-launch figures are the workload's)."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if any(r['Counter_Name'].startswith(n) for n in names):
                rows.append((short(r['Kernel_Name']), int(r['Grid_Size']), r['Counter_Name'], float(r['Counter_Value'])))
    big = defaultdict(int)
    for k, gsz, _, _ in rows:
        big[k] = max(big[k], gsz)
    acc = defaultdict(lambda: defaultdict(list))
    for k, gsz, c, v in rows:
        if gsz == big[k]:
            acc[k][c].append(v)
    return {k: ({c: sum(v) / len(v) for c, v in cs.items()}, max(len(v) for v in cs.values())) for k, cs in acc.items()}


def main(d):
    kt = find(os.path.join(d, 'kt'), 'kernel_trace.csv')
    rows = []
    with open(kt) as f:
        for r in csv.DictReader(f):
            gsz = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
            rows.append((short(r['Kernel_Name']), gsz, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6))
    big = defaultdict(int)
    for k, gsz, _ in rows:
        big[k] = max(big[k], gsz)
    dur = defaultdict(list)  # the full-size launches (the kernel's largest grid), as per_dispatch
    for k, gsz, ms in rows:
        if gsz == big[k]:
            dur[k].append(ms)
    fetch = per_dispatch(find(os.path.join(d, 'FETCH_SIZE'), 'counter_collection.csv'), ['FETCH_SIZE'])
    write = per_dispatch(find(os.path.join(d, 'WRITE_SIZE'), 'counter_collection.csv'), ['WRITE_SIZE'])
    l2 = per_dispatch(find(os.path.join(d, 'TCC_HIT_sum'), 'counter_collection.csv'), ['TCC_HIT', 'TCC_MISS'])
    out = {'source': os.path.relpath(d), 'kernels': {}}
    # the build the profiled bench command ran (bench.py's 'build': sources hash + library):
    # bench.py attaches this summary's traffic only to lines of the same build
    try:
        with open(os.path.join(d, 'bench_kt.json')) as f:
            out['build'] = json.loads(f.read().strip().splitlines()[-1]).get('build')
    except (OSError, ValueError, IndexError):
        out['build'] = None
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if not k.startswith('k_'):
            continue
        e = {'launches': len(dur[k]), 'avg_ms': round(sum(dur[k]) / len(dur[k]), 4),
             'total_ms': round(sum(dur[k]), 3)}
        if k in fetch:
            e['fetch_bytes_per_launch'] = round(sum(fetch[k][0].values()) * 1024.0)
        if k in write:
            e['write_bytes_per_launch'] = round(sum(write[k][0].values()) * 1024.0)
        if k in l2:
            h = sum(v for c, v in l2[k][0].items() if c.startswith('TCC_HIT'))
            m = sum(v for c, v in l2[k][0].items() if c.startswith('TCC_MISS'))
            e['l2_hit'] = round(h / (h + m), 4) if h + m > 0 else None
        if 'fetch_bytes_per_launch' in e and 'write_bytes_per_launch' in e and e['avg_ms'] > 0:
            gbs = (e['fetch_bytes_per_launch'] + e['write_bytes_per_launch']) / (e['avg_ms'] * 1e-3) / 1e9
            e['hbm_gbs'] = round(gbs, 1)
            e['hbm_frac'] = round(gbs / PEAK_GBS, 4)
        out['kernels'][k] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main(sys.argv[1])
