#!/bin/bash
# Routing round width sweep (perf knob only: labels are order-independent).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep
mkdir -p $O
for d in ${DELTAS:-60 80 100 130 170}; do
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --cpu-traces 0 --delta $d > $O/delta_$d.json 2> $O/delta_$d.err
done
echo done
