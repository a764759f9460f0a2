#!/usr/bin/env python3
"""Per-kernel L2 (TCC) hit rate from a tools/profile_l2.sh pass, joined with the
FETCH_SIZE/WRITE_SIZE bytes and kernel-trace durations of a tools/pmc_summary.py
document: measured HBM GB/s = (fetch + write bytes per launch) / average launch time,
as a fraction of the 8 TB/s MI355X peak (MI355X_MICROARCH.md).

  python tools/l2_summary.py gpurun_out/l2 profiles/r01_v22_pmc.json > profiles/r01_v23_l2.json
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

PEAK_GBS = 8000.0
KERNELS = ('k_route', 'k_paths', 'k_viterbi', 'k_candidates', 'k_segments', 'k_prep', 'k_tasks', 'k_task_rec')


def short(name):
    name = re.sub(r'^void ', '', name)
    name = re.sub(r'\(.*$', '', name)
    return re.sub(r'^otr::', '', name)


def hits(path):
    acc = defaultdict(lambda: [0.0, 0.0, 0])
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r['Kernel_Name'])
            if r['Counter_Name'].startswith('TCC_HIT'):
                acc[k][0] += float(r['Counter_Value'])
                acc[k][2] += 1
            elif r['Counter_Name'].startswith('TCC_MISS'):
                acc[k][1] += float(r['Counter_Value'])
    return acc


def main():
    d, pmc = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    bytes_ = json.load(open(pmc))['kernels'] if pmc else {}
    out = {'source': {'l2_passes': d, 'fetch_write': pmc}, 'peak_hbm_gbs': PEAK_GBS, 'workloads': {}}
    for sub, wl in (('p1', 'C2'), ('p4', 'C4')):
        p = os.path.join(d, sub, 'run_counter_collection.csv')
        if not os.path.exists(p):
            continue
        rows = {}
        for k, (h, m, n) in sorted(hits(p).items(), key=lambda kv: -(kv[1][0] + kv[1][1])):
            if not k.startswith(KERNELS):
                continue
            e = {'launches': n, 'tcc_hit': int(h), 'tcc_miss': int(m),
                 'l2_hit_rate': round(h / (h + m), 4) if h + m else None}
            b = bytes_.get(k)
            if wl == 'C2' and b and b.get('avg_ms'):
                tot = b['fetch_bytes_per_launch'] + b['write_bytes_per_launch']
                e['hbm_bytes_per_launch'] = tot
                e['avg_ms'] = b['avg_ms']
                e['hbm_gbs'] = round(tot / (b['avg_ms'] * 1e-3) / 1e9, 1)
                e['hbm_frac'] = round(e['hbm_gbs'] / PEAK_GBS, 4)
            rows[k] = e
        out['workloads'][wl] = rows
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
