#!/bin/bash
# GPU tile-stage tests first (each pytest step under its own time limit), then the rest.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tiles
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_tiles.py -x -v --timeout 60 --timeout-method thread > $O/pytest_tiles.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo done
