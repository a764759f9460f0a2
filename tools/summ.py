#!/usr/bin/env python3
"""One line per bench JSON file: rate, step ms, route stages, dominant kernel and roofline."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 - a summary tool: report and go on
        print(f, 'unreadable', e)
        continue
    c = d['config']
    st = c.get('stage_ms_per_stream', {})
    r = d['roofline']
    par = d.get('parity') or {}
    print('%-40s %12.0f %8.3f route %7.3f big %7.3f  %-30s %8.3f ms frac %.4f parity %s' % (
        f[-40:], d['value'], d['ms_per_step'], st.get('route', 0), st.get('route_big', 0), r['kernel'][:30],
        r['launch_ms'], r['frac'], par.get('ok')))
