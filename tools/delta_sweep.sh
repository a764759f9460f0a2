#!/bin/bash
# Route round width (Δ, metres: search order only) sweep on C2 and C4, bench lines under
# gpurun_out/dsweep.  Usage: bash tools/delta_sweep.sh "C2 deltas" "C4 deltas"
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dsweep
for d in ${1:-60 75 90}; do
  timeout -k 10 240 python3 -u bench.py --steps 5 --cpu-traces 0 --e2e-steps 0 --delta $d > gpurun_out/dsweep/c2_$d.json 2> gpurun_out/dsweep/c2_$d.err
done
for d in ${2:-60 75}; do
  timeout -k 10 240 python3 -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 --delta $d > gpurun_out/dsweep/c4_$d.json 2> gpurun_out/dsweep/c4_$d.err
done
