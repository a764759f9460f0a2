#!/bin/bash
# Round-3 profiles of the default C2 bench command: kernel trace + stats, FETCH_SIZE and
# WRITE_SIZE passes (+ calibration), L2 hits/misses, and the SQ issue/wait passes.
# Summaries: tools/pmc_summary.py, tools/l2_summary.py, tools/sq_summary.py.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/profile_gpu.sh
O=gpurun_out/l2
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p1 -o run -- \
  python3 bench.py --steps 2 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/bench_p1.json 2> $O/bench_p1.err
bash tools/profile_sq.sh sq
echo done
