#!/bin/bash
# One GPU call: the GPU test suite, then the bench lines (C2 headline with the CPU
# baseline, parity sample and end-to-end leg; C4 at BASELINE size; a C3 shard
# rehearsal), then a kernel-trace profile of the C2 command.
# Usage (from the repo root, through gpurun):  bash tools/gpu_check.sh [tag] [skip_tests]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-check}
O=gpurun_out/$T
mkdir -p $O
if [ "${2:-}" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --workload c4 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --workload c3 --traces-per-gpu 10000 --cpu-traces 0 --e2e-steps 0 > $O/bench_c3.json 2> $O/bench_c3.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --cpu-traces 0 --e2e-steps 0 > $O/bench_under_rocprof.json 2> $O/rocprof.err
echo done
