#!/bin/bash
# the whole GPU test suite (one gpurun call), log under gpurun_out/TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r6t}
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
exit $rc
