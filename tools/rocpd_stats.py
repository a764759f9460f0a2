#!/usr/bin/env python3
"""Per-kernel stats (calls, average / total ns, % of kernel time) from a rocprofv3
kernel-trace SQLite database (rocpd, the default output format):
    python tools/rocpd_stats.py gpurun_out/.../run_results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    q = ('select s.display_name, count(*), avg(d.end - d.start), sum(d.end - d.start) '
         'from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id '
         'group by s.display_name order by sum(d.end - d.start) desc')
    rows = list(c.execute(q))
    tot = sum(r[3] for r in rows) or 1
    return [{'Name': r[0], 'Calls': r[1], 'AverageNs': round(r[2], 1), 'TotalDurationNs': r[3],
             'Percentage': round(100.0 * r[3] / tot, 3)} for r in rows]


if __name__ == '__main__':
    rows = stats(sys.argv[1])
    out = open(sys.argv[2], 'w', newline='') if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(out, fieldnames=['Name', 'Calls', 'AverageNs', 'TotalDurationNs', 'Percentage'])
    w.writeheader()
    w.writerows(rows)
