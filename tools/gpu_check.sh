#!/bin/bash
# One GPU call: GPU parity tests, then the default bench line (with CPU baseline).
# Usage (from the repo root, through gpurun):  bash tools/gpu_check.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
