#!/bin/bash
# Round-3 check in one GPU call: the GPU test suite, the C2 headline bench and the
# deployed-configuration bench (c2dep).  Usage: bash tools/r03_check.sh TAG [notests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r3}
O=gpurun_out/$T
mkdir -p $O
if [ "${2:-}" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  tail -25 $O/pytest.log
fi
timeout -k 10 240 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -2 $O/bench.err
timeout -k 10 300 python -u bench.py --workload c2dep > $O/bench_dep.json 2> $O/bench_dep.err
tail -2 $O/bench_dep.err
