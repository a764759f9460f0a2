#!/bin/bash
# C2 single-stream kernel traces under the generate_test_trace options (turn penalty 0)
# and under the deployed turn penalties (turn_penalty_factor 200): per-kernel costs of
# both route-search modes.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abt}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gtt -o run -- python3 bench.py --streams 1 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/gtt.json 2> $O/gtt.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/turn -o run -- python3 bench.py --streams 1 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 --opt turn_penalty_factor=200 > $O/turn.json 2> $O/turn.err
echo done
