#!/usr/bin/env python3
"""Summary of tools/ab.sh lines: per variant, probes/s and the route kernels' ms per launch."""
import collections
import json
import os
import sys


def main(d):
    acc = collections.defaultdict(list)
    for f in sorted(os.listdir(d)):
        if not f.endswith('.json'):
            continue
        try:
            line = json.loads(open(os.path.join(d, f)).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        acc[f.rsplit('_', 1)[0]].append(line)
    for v, lines in acc.items():
        vals = [round(x['value'] / 1e6, 3) for x in lines]
        par = [x['parity']['ok'] for x in lines if x.get('parity')]
        ks = collections.defaultdict(list)
        for x in lines:
            for k, r in x['config']['route_kernels'].items():
                if r['ms_per_launch'] > 0.05:
                    ks[k].append(r['ms_per_launch'])
        print('%-14s Mprobes/s %s parity %s' % (v, vals, par))
        for k, ms in ks.items():
            print('    %-40s %s' % (k, ms))


if __name__ == '__main__':
    main(sys.argv[1])
