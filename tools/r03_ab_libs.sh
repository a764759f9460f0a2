#!/bin/bash
# A/B of several library variants on one workload, in the order given, then the default
# library again (box drift).  Usage: bash tools/r03_ab_libs.sh TAG libA.so libB.so ... [-- bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
O=gpurun_out/$T
mkdir -p $O
i=0
for V in "${LIBS[@]}" reporter_amd/libotr.so; do
  i=$((i+1))
  OTR_LIB=$V timeout -k 10 300 python -u bench.py --cpu-traces 0 --e2e-steps 0 "$@" > $O/r$i.json 2> $O/r$i.err || exit 1
  echo "$i $V" >> $O/order.txt
done
echo done
