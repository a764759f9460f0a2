#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh run: per-kernel average duration (kernel trace),
per-dispatch FETCH_SIZE / WRITE_SIZE (separate --pmc passes, KiB → bytes), and the
calibration ratios of tools/calib_fetch (counter bytes ÷ known bytes per access shape,
MI355X_MICROARCH.md §HBM).  Output: one JSON document on stdout.

  python tools/pmc_summary.py gpurun_out/prof > profiles/r01_pmc.json
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r'^void ', '', name)
    name = re.sub(r'\(.*$', '', name)
    name = re.sub(r'^otr::', '', name)
    return name


def counters(path):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[short(r['Kernel_Name'])].append(float(r['Counter_Value']) * 1024.0)
    return acc


def durations(path):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[short(r['Kernel_Name'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-6)
    return acc


def main(d):
    out = {'kernels': {}, 'calibration': {}}
    dur = durations(os.path.join(d, 'kt', 'run_kernel_trace.csv'))
    fetch = counters(os.path.join(d, 'FETCH_SIZE', 'run_counter_collection.csv'))
    write = counters(os.path.join(d, 'WRITE_SIZE', 'run_counter_collection.csv'))
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if not (k.startswith('k_') or k.startswith('otr')):
            continue
        e = {'launches': len(dur[k]), 'avg_ms': round(sum(dur[k]) / len(dur[k]), 4)}
        if k in fetch:
            e['fetch_bytes_per_launch'] = round(sum(fetch[k]) / len(fetch[k]))
        if k in write:
            e['write_bytes_per_launch'] = round(sum(write[k]) / len(write[k]))
        out['kernels'][k] = e
    cal_f = counters(os.path.join(d, 'cal_FETCH_SIZE', 'run_counter_collection.csv'))
    cal_w = counters(os.path.join(d, 'cal_WRITE_SIZE', 'run_counter_collection.csv'))
    known = json.load(open(os.path.join(d, 'calib.json')))
    for k, key, src in (('k_stream', 'stream_bytes', cal_f), ('k_gather64', 'gather64_bytes', cal_f),
                        ('k_gather16', 'gather16_bytes', cal_f), ('k_gather4', 'gather4_bytes', cal_f),
                        ('k_write8', 'write8_bytes', cal_w)):
        if k in src:
            v = sum(src[k]) / len(src[k])
            out['calibration'][k] = {'known_bytes': known[key], 'counter_bytes': round(v),
                                     'ratio': round(v / known[key], 4)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof')
