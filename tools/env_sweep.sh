#!/bin/bash
# One workload under several settings of one environment knob (one gpurun call):
#   bash tools/env_sweep.sh TAG WORKLOAD VAR VALUE... -> gpurun_out/TAG/<VAR>_<VALUE>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; WL=$2; VAR=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python3 -u bench.py --workload $WL --e2e-steps 0 --cpu-traces 0 > $O/${VAR}_$v.json 2> $O/${VAR}_$v.err || { echo "$VAR=$v failed"; exit 1; }
  echo "$VAR=$v ok"
done
