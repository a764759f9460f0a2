#!/bin/bash
# A/B of library variants over several workloads (one gpurun call): tools/ab.sh per workload
# Usage: bash tools/r6_ab.sh TAG "W:ROUNDS W:ROUNDS" VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; WS=$2; shift 2
for wr in $WS; do
  w=${wr%%:*}; r=${wr#*:}
  bash tools/ab.sh ${TAG}_$w $w $r "$@" -- --json-traces 0 || exit 1
done
