#!/bin/bash
# Profiles of one or more bench workloads (run through gpurun from the repo root), each
# command in its own rocprofv3 runs:
#   kt      --kernel-trace --stats (per-kernel durations; the stats CSV is the summary)
#   FETCH   --pmc FETCH_SIZE      (3 of the 4 TCC slots: a pass of its own)
#   WRITE   --pmc WRITE_SIZE
#   L2      --pmc TCC_HIT_sum TCC_MISS_sum
# Summary per workload: python tools/profile_summary.py gpurun_out/TAG/W > profiles/<round>_pmc_W.json
# Usage: bash tools/profile_set.sh TAG W [W...]   (W: c2 c2dep c4 c1 c5mix)
# A pass that fails or times out ends the call.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
for W in "$@"; do
  O=gpurun_out/$TAG/$W
  mkdir -p $O
  ARGS="--workload $W --cpu-traces 0 --e2e-steps 0 --json-traces 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 bench.py $ARGS --steps 5 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err
  for P in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    N=${P%% *}
    timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/$N -o run -- \
      python3 bench.py $ARGS --steps 2 --warmup 1 > $O/bench_$N.json 2> $O/bench_$N.err
  done
  echo "$W done"
done
echo done
