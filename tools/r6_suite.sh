#!/bin/bash
# GPU suite subset + determinism diagnostics (one gpurun call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r6b}
mkdir -p $O
shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
exit $rc
