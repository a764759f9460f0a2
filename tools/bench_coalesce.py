#!/usr/bin/env python3
"""Concurrent otr_report callers (native threads, reporter_amd/tools/loadgen) with and
without the request coalescer, on C2 bodies.  One JSON line per configuration.

  python tools/bench_coalesce.py [--traces 10000] [--threads 64,256] [--coalesce 0,1024]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--traces', type=int, default=10000)
    ap.add_argument('--threads', default='64,256')
    ap.add_argument('--coalesce', default='0,1024')
    ap.add_argument('--wait-us', type=int, default=2000)
    args = ap.parse_args()
    from bench_json import bodies_for
    from reporter_amd import matcher as M
    from reporter_amd.tools import gen
    gpath = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    tr = gen.make_traces(gpath, args.traces, 100, 15, 10.0, 2, t_begin=1483228800, t_spread=1800)
    d = tempfile.mkdtemp(prefix='otr_load_')
    bodies = os.path.join(d, 'bodies.txt')
    with open(bodies, 'w') as f:
        f.write('\n'.join(bodies_for(tr)) + '\n')
    conf = os.path.join(d, 'valhalla.json')
    with open(conf, 'w') as f:
        json.dump(M.default_config(gpath), f)
    exe = os.path.join(ROOT, 'reporter_amd', 'tools', 'loadgen')
    for th in [int(x) for x in args.threads.split(',')]:
        for c in [int(x) for x in args.coalesce.split(',')]:
            r = subprocess.run([exe, conf, bodies, str(th), str(c), str(args.wait_us)], stdout=subprocess.PIPE,
                               text=True, timeout=600)
            line = json.loads(r.stdout.strip().splitlines()[-1])
            line['probes_per_s'] = round(line['traces_per_s'] * tr.n_probes / tr.n_traces, 1)
            line['exit'] = r.returncode
            print(json.dumps(line), flush=True)
            if r.returncode != 0:
                raise SystemExit(r.returncode)


if __name__ == '__main__':
    main()
