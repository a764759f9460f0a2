#!/bin/bash
# L2 (TCC) hit rate per kernel of the default bench command: one --pmc pass
# (TCC_HIT_sum + TCC_MISS_sum, 2 of the 4 TCC slots), kernel trace only.
# Summary: python tools/l2_summary.py gpurun_out/l2 profiles/<round>_pmc.json > profiles/<round>_l2.json
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/l2
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p1 -o run -- \
  python3 bench.py --steps 2 --warmup 1 --cpu-traces 0 > $O/bench_p1.json 2> $O/bench_p1.err
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p4 -o run -- \
  python3 bench.py --workload c4 --steps 1 --warmup 1 --cpu-traces 0 > $O/bench_p4.json 2> $O/bench_p4.err
echo done
