#!/bin/bash
# A/B of libotr builds on one GPU: for each NAME, a single-stream C2 bench under a kernel
# trace with OTR_LIB=reporter_amd/libotr_NAME.so ("main" = reporter_amd/libotr.so).
#   tools/ab_libs.sh OUTDIR main A nocnt [-- extra bench args]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p $O
for n in "${names[@]}"; do
  if [ "$n" == "main" ]; then lib=reporter_amd/libotr.so; else lib=reporter_amd/libotr_$n.so; fi
  OTR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- \
    python3 bench.py --streams 1 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 "$@" > $O/$n.json 2> $O/$n.err
  echo "$n done"
done
