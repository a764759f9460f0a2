#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of the default C2 bench for each library
# variant given.  Usage: bash tools/r03_kt_libs.sh TAG libA.so libB.so ...
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
i=0
for V in "$@"; do
  i=$((i+1))
  echo "$i $V" >> $O/order.txt
  OTR_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$i -o run -- \
    python3 bench.py --steps 5 --warmup 2 --cpu-traces 0 --e2e-steps 0 > $O/b$i.json 2> $O/b$i.err
done
echo done
