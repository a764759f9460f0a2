#!/bin/bash
# One GPU call: GPU parity tests, the default bench line, then the C4 and C5-mix lines.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u bench.py --workload c4 --cpu-traces 0 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --workload c5mix --cpu-traces 0 > $O/bench_c5mix.json 2> $O/bench_c5mix.err
echo done
