#!/bin/bash
# Small-search tier check + A/B (one gpurun call): its GPU test and the parity suite, then
# bench lines with the tier off / default / a larger size limit (tools/ab.sh)
# Usage: bash tools/r6_small.sh TAG "W:ROUNDS ..." VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; WS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
fi
for wr in $WS; do
  w=${wr%%:*}; r=${wr#*:}
  bash tools/ab.sh ${TAG}_$w $w $r "$@" -- --json-traces 0 || exit 1
done
echo done
