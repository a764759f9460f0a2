#!/bin/bash
# A/B on one GPU: single-stream kernel traces of the C2 bench with the route-time bound
# on (deployed) and off (max_route_time_factor=0), for per-kernel costs.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/on -o run -- python3 bench.py --streams 1 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/on.json 2> $O/on.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/off -o run -- python3 bench.py --streams 1 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 --opt max_route_time_factor=0 > $O/off.json 2> $O/off.err
echo done
