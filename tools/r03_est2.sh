#!/bin/bash
# First-tier size estimate scale A/B on C4 and C2.  Usage: bash tools/r03_est2.sh TAG k1 k2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-est2}; shift
mkdir -p $O
for k in "$@"; do
  OTR_EST_K=$k timeout -k 10 600 python3 -u bench.py --workload c4 --e2e-steps 0 --cpu-traces 0 --steps 3 --warmup 1 > $O/c4_$k.json 2> $O/c4_$k.err; echo c4 $k $?
  OTR_EST_K=$k timeout -k 10 300 python3 -u bench.py --e2e-steps 0 --cpu-traces 0 > $O/c2_$k.json 2> $O/c2_$k.err; echo c2 $k $?
done
