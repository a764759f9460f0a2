#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes written by tools/profile_sq.sh."""
import collections
import csv
import json
import os
import re
import sys


def main(d):
    out = collections.defaultdict(dict)
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, 'run_counter_collection.csv')
        if not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            k = re.sub(r'\(.*$', '', re.sub(r'^void ', '', r['Kernel_Name'])).replace('otr::', '')
            acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
        for k, cs in acc.items():
            if k.startswith('k_'):
                for c, v in cs.items():
                    out[k][c] = sum(v) / len(v)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/sq')
