#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg ns, %) from a rocprofv3 SQLite (rocpd) output, as
the --stats CSV gives it, with rocPRIM template names shortened.

  python tools/rocpd_stats.py gpurun_out/.../run_results.db > profiles/<name>.csv
"""
import re
import sqlite3
import sys


def short(name):
    if 'rocprim' in name:
        m = re.search(r'detail::(\w+?)_config<[^,]*, ([\w ]+)(?:, ([\w ]+))?>', name)
        kind = re.search(r'wrapped_(\w+?)_config', name)
        return 'rocprim::%s<%s>' % (kind.group(1) if kind else 'kernel', m.group(2) if m else '?') \
            if kind else re.sub(r'<.*', '', name)[:80]
    return name


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute('select name, total_calls, total_duration, average, percentage from top_kernels'))
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage"')
    for name, calls, total, avg, pct in rows:
        # top_kernels reports microseconds; the CSV keeps --stats' nanoseconds
        print('"%s",%d,%d,%.1f,%.2f' % (short(name).replace('"', "'"), calls, round(total * 1e3), avg * 1e3, pct))


if __name__ == '__main__':
    main(sys.argv[1])
