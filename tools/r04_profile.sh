#!/bin/bash
# Round-4 profiles: kernel trace + stats of the default C2 bench command and of the deployed
# configuration, FETCH_SIZE / WRITE_SIZE passes (tools/profile_gpu.sh), L2 hits/misses, and
# the SQ issue/wait passes of both.  Summaries: tools/pmc_summary.py, tools/l2_summary.py,
# tools/sq_summary.py, tools/rocpd_stats.py.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/profile_gpu.sh
O=gpurun_out/kt_c2dep
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --workload c2dep --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/bench.json 2> $O/bench.err
O=gpurun_out/l2
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p1 -o run -- \
  python3 bench.py --steps 2 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/bench_p1.json 2> $O/bench_p1.err
bash tools/profile_sq.sh sq
bash tools/profile_sq.sh sq_c2dep --workload c2dep
echo done
