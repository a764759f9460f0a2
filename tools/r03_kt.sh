#!/bin/bash
# Kernel-trace + stats of the default C2 bench (one rocprofv3 pass), for A/B of a change.
# Usage: bash tools/r03_kt.sh TAG
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-kt}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-traces 0 > $O/bench_kt.json 2> $O/bench_kt.err
timeout -k 10 240 python3 bench.py --cpu-traces 0 > $O/bench2.json 2> $O/bench2.err
echo done
