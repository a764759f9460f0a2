#!/bin/bash
# A/B of library builds on the C2 headline (and optionally c2dep): bench lines per build.
# Usage: bash tools/r03_ab.sh TAG WORKLOAD lib1 lib2 ...   (lib "" = reporter_amd/libotr.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; W=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for L in "$@"; do
  n=$(basename "${L:-default}" .so)
  if [ -n "$L" ]; then export OTR_LIB=$PWD/$L; else unset OTR_LIB; fi
  timeout -k 10 300 python -u bench.py --workload $W --cpu-traces 0 --e2e-steps 0 > $O/bench_${W}_$n.json 2> $O/bench_${W}_$n.err || exit 1
  tail -1 $O/bench_${W}_$n.err
done
