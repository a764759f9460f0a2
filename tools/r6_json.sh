#!/bin/bash
# JSON drop-in measurements (one gpurun call): bench lines with the json_dropin leg (c2,
# c2dep) and the coalescer's dispatcher count / quiet gap on c2dep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r6j}
mkdir -p $O
for W in c2 c2dep; do
  timeout -k 10 400 python3 -u bench.py --workload $W --cpu-traces 0 --e2e-steps 0 > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
  echo "$W ok"
done
for V in "1 100" "2 100" "3 100" "2 0" "2 300"; do
  set -- $V
  OTR_COALESCE_DISPATCHERS=$1 OTR_COALESCE_GAP_US=$2 timeout -k 10 400 python3 -u tools/bench_json.py --workload c2dep --traces 4000 > $O/json_c2dep_d$1_g$2.json 2> $O/json_c2dep_d$1_g$2.err || exit 1
  echo "d$1 g$2 ok"
done
