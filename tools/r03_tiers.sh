#!/bin/bash
# Retry-tier lists on C4 (OTR_TIERS A/B).  Usage: bash tools/r03_tiers.sh TAG list1 list2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-tiers}; shift
mkdir -p $O
for t in "$@"; do
  OTR_TIERS=$t timeout -k 10 600 python3 -u bench.py --workload c4 --e2e-steps 0 --cpu-traces 0 --steps 3 --warmup 1 > $O/c4_$t.json 2> $O/c4_$t.err; echo c4 $t $?
done
