#!/bin/bash
# One-GPU A/B of the bench's matcher streams (1 vs 2) and the deployed turn-penalty config
# (turn_penalty_factor 200: every search in the global-memory edge-based kernel).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ms}
mkdir -p $O
for s in 1 2; do
  timeout -k 10 300 python3 bench.py --streams $s --cpu-traces 0 --e2e-steps 0 > $O/s$s.json 2> $O/s$s.err
done
timeout -k 10 400 python3 bench.py --cpu-traces 0 --e2e-steps 0 --opt turn_penalty_factor=200 > $O/turn.json 2> $O/turn.err
echo done
