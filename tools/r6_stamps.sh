#!/bin/bash
# per-phase shader-clock stamps of the first route tier (libotr_stamps.so) on c2 and c5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r6st}
mkdir -p $O
shift
for W in "$@"; do
  OTR_LIB=$PWD/reporter_amd/libotr_stamps.so timeout -k 10 400 python3 -u bench.py --workload $W --cpu-traces 0 --e2e-steps 0 --json-traces 0 > $O/$W.json 2> $O/$W.err || exit 1
  echo "$W ok"
done
