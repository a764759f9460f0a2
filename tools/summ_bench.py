"""Print the headline fields of bench JSON lines (tools/r03_check.sh outputs)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, 'unreadable:', e)
        continue
    c = d['config']
    print(f, d['value'], 'ms/step', d['ms_per_step'], 'e2e', c.get('end_to_end', {}).get('value') if isinstance(c.get('end_to_end'), dict) else c.get('end_to_end'))
    print('  stages', c.get('stage_ms_per_stream'))
    for k, v in c.get('route_kernels', {}).items():
        if v.get('searches_per_launch'):
            print('  ', k, v['ms_per_launch'], 'ms', v['searches_per_launch'], 'searches', v.get('settled_per_launch'), 'settled')
    print('  parity', d.get('parity'))
    print('  roofline', d.get('roofline'))
