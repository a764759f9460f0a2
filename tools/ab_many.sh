#!/bin/bash
# A/B of several libotr builds on one GPU, plain bench lines (no profiler), in order and
# then once more in reverse order (drift check):
#   tools/ab_many.sh OUTDIR main prev variantA ... [-- extra bench args]
# "main" = reporter_amd/libotr.so, NAME = reporter_amd/libotr_NAME.so
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
shift
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ "${1:-}" == "--" ] && shift
mkdir -p $O
run() {
  local n=$1 tag=$2
  if [ "$n" == "main" ]; then lib=reporter_amd/libotr.so; else lib=reporter_amd/libotr_$n.so; fi
  OTR_LIB=$lib timeout -k 10 240 python3 -u bench.py --cpu-traces 0 --e2e-steps 0 "${@:3}" > $O/${n}_$tag.json 2> $O/${n}_$tag.err
  echo "$n $tag done"
}
for n in "${names[@]}"; do run $n a "$@"; done
for ((k=${#names[@]}-1; k>=0; k--)); do run ${names[$k]} b "$@"; done
