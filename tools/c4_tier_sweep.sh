#!/bin/bash
# C4 retry-tier lists (OTR_TIERS) on one box: bench lines under gpurun_out/c4sweep/tN.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c4sweep; mkdir -p $O
i=0
for T in "${@:-256,448x2,1024,2048}"; do
  i=$((i+1))
  OTR_TIERS=$T timeout -k 10 200 python3 -u bench.py --workload c4 --e2e-steps 0 --cpu-traces 0 > $O/t$i.json 2> $O/t$i.err || { echo "t$i failed"; exit 1; }
  echo "t$i $T ok"
done
