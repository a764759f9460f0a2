#!/bin/bash
# GPU test suite, then the deployed-config bench (c2dep) for the default build and A/B
# libraries.  Usage: bash tools/r03_edge.sh TAG lib1 lib2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-edge}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 900 --timeout-method thread > $O/pytest.log 2>&1
tail -4 $O/pytest.log
bash tools/r03_ab.sh $T c2dep "" "$@"
