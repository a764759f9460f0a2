#!/usr/bin/env python3
"""N > 1 load balance on the CPU: a sample of C3's fleet (veh%07d uuids,
metro graph, bench.py's c3 options) matched by the CPU oracle (ANALYSIS ONLY), its tile
rows (simple_reporter.py:176-196) and keyed entries, and per rank at N = 2, 4, 8:
  * traces per uuid shard (sha1(uuid)[:3] % N, simple_reporter.py:116),
  * rows / keyed entries / files per (hour, tile) file owner (simple_reporter.file_owner),
  * ranks that own no file.
Prints one JSON document.

  python tools/owner_load.py [n_uuids]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    from oracle import hist, pyoracle as po, tiles
    from reporter_amd import simple_reporter as sr
    from reporter_amd.tools import gen
    gp = gen.graph_path('metro', os.path.join(ROOT, 'build', 'graphs'))
    ids = np.arange(n, dtype=np.int64) * (1000000 // n)  # spread over the 1M uuids
    tr = gen.make_traces_ids(gp, ids, 100, 15, 10.0, 3, t_begin=1483228800, t_spread=1800, threads=8)
    opts = {'turn_penalty_factor': 0, 'beta': 3, 'sigma_z': 4.07, 'breakage_distance': 2000, 'search_radius': 50,
            'gps_accuracy': 16.45}
    res = po.match_batch(po.Graph(gp), tr, po.params(**opts), threads=os.cpu_count() or 8)
    first = tr.time[tr.offsets[:-1]]
    last = tr.time[tr.offsets[1:] - 1]
    rows = tiles.rows_from_reports(res, first, last)
    ent = hist.reduce(hist.entries_from_rows(rows), 1)
    files = np.unique(rows['file'].astype(np.int64))
    out = {'sample': '%d C3 uuids x 100 probes (metro graph, CPU oracle)' % n, 'rows': int(len(rows)),
           'entries': int(len(ent)), 'files': int(len(files)), 'per_world': {}}
    for world in (2, 4, 8):
        shard = np.array([int(hashlib.sha1(u.encode()).hexdigest()[:3], 16) % world for u in tr.uuids])
        ro = sr.file_owner(rows['file'].astype(np.int64), world)
        eo = sr.file_owner(ent['file'].astype(np.int64), world)
        fo = sr.file_owner(files, world)
        tr_per = np.bincount(shard, minlength=world)
        rows_per = np.bincount(ro, minlength=world)
        ent_per = np.bincount(eo, minlength=world)
        out['per_world'][str(world)] = {
            'traces_per_rank': tr_per.tolist(),
            'trace_imbalance': round(float(tr_per.max() / tr_per.mean()), 3),
            'rows_per_owner': rows_per.tolist(), 'entries_per_owner': ent_per.tolist(),
            'files_per_owner': np.bincount(fo, minlength=world).tolist(),
            'entry_imbalance': round(float(ent_per.max() / ent_per.mean()), 3),
            'owners_without_files': int((np.bincount(fo, minlength=world) == 0).sum())}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
