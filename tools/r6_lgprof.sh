#!/bin/bash
# kernel trace of small coalesced requests (loadgen, c2dep bodies in 12-point windows)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6lgp}
mkdir -p $O
timeout -k 10 300 python3 -u - <<'PY' > $O/prep.log 2>&1 || exit 1
import json, os, sys
sys.path.insert(0, '.')
from reporter_amd import matcher as M
from reporter_amd.tools import gen, dropin
gp = gen.graph_path('metro', 'build/graphs')
tr = gen.make_traces(gp, 400, 100, 15, 10.0, 2, t_begin=1483228800, t_spread=1800)
json.dump(M.default_config(gp), open('/tmp/lg_cfg.json', 'w'))
open('/tmp/lg_small.txt', 'wb').write(b'\n'.join(dropin.bodies(tr, 12)[0]) + b'\n')
print('prepared')
PY
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o run -- reporter_amd/tools/loadgen /tmp/lg_cfg.json /tmp/lg_small.txt 64 4096 2000 > $O/lg.json 2> $O/lg.err
echo rc=$?
