#!/bin/bash
# A/B of environment knobs on one library: single-stream bench lines per setting.
# Items may join several assignments with "+" (A=1+B=2).
# Usage: ENVS="OTR_DIRECT_BMM=1900000 OTR_DIRECT_BMM=1500000" BENCH_ARGS="--workload c4" bash tools/ab_env.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abenv
mkdir -p $O
for rep in 1 2; do
  for e in NONE=1 $ENVS; do
    env ${e//+/ } timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --cpu-traces 0 --streams 1 ${BENCH_ARGS} > $O/bench_${e//[\/+,]/_}_$rep.json 2> $O/bench_${e//[\/+,]/_}_$rep.err
  done
done
echo done
