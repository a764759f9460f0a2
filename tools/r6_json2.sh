#!/bin/bash
# JSON drop-in (c2dep bench_json, native callers) + small-request kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${1:-r6j4}
mkdir -p $O
timeout -k 10 400 python3 -u tools/bench_json.py --workload c2dep --traces 4000 > $O/json_c2dep.json 2> $O/json_c2dep.err || exit 1
timeout -k 10 400 python3 -u tools/bench_json.py --workload c2 --traces 4000 > $O/json_c2.json 2> $O/json_c2.err || exit 1
bash tools/r6_lgprof.sh ${1:-r6j4}/lgp
