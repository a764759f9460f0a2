#!/bin/bash
# A/B of bench arguments: single-stream bench lines per argument set (';'-separated).
# Usage: ARGSETS="--delta 100;--delta 200" BENCH_ARGS="--workload c4" bash tools/ab_args.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abargs
mkdir -p $O
IFS=';' read -ra SETS <<< "$ARGSETS"
for rep in 1 2; do
  i=0
  for a in "${SETS[@]}"; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --cpu-traces 0 --streams 1 ${BENCH_ARGS} $a > $O/bench_${i}_$rep.json 2> $O/bench_${i}_$rep.err
    i=$((i+1))
  done
done
echo done
