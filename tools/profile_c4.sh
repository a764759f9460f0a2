#!/bin/bash
# Kernel-trace stats of the C4 workload (sparse 60 s probes, 200 m radius), one stream.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --workload c4 --steps 2 --warmup 1 --streams 1 --cpu-traces 0 --e2e-steps 0 > $O/bench.json 2> $O/err
echo done
