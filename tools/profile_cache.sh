#!/bin/bash
# L2 hit rate pass + a diagnostic stamps-build bench (per-phase search cycles).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/cache
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/p1 -o run -- \
  python3 bench.py --steps 1 --warmup 1 --cpu-traces 0 > $O/bench_p1.json 2> $O/bench_p1.err
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $O/p2 -o run -- \
  python3 bench.py --steps 1 --warmup 1 --cpu-traces 0 > $O/bench_p2.json 2> $O/bench_p2.err
OTR_LIB=$PWD/reporter_amd/libotr_stamps.so timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-traces 0 > $O/bench_stamps.json 2> $O/bench_stamps.err
echo done
