#!/bin/bash
# route-stage A/B: per-root first tier (OTR_ROUTE_STEP=0) vs the multi-root step kernel
# and its variants, one bench line each (no CPU sample).  Results under gpurun_out/$1.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-abstep}; mkdir -p $O
B="python -u bench.py --cpu-traces 0 --e2e-steps 0"
OTR_ROUTE_STEP=0 timeout -k 10 200 $B > $O/perroot.json 2> $O/perroot.err
timeout -k 10 200 $B > $O/step.json 2> $O/step.err
[ -f reporter_amd/libotr_stamps.so ] && OTR_ROUTE_STEP=0 OTR_LIB=reporter_amd/libotr_stamps.so timeout -k 10 200 $B > $O/perroot_stamps.json 2> $O/perroot_stamps.err
for v in "$@"; do
  [ -f reporter_amd/libotr_$v.so ] || continue
  OTR_LIB=reporter_amd/libotr_$v.so timeout -k 10 200 $B > $O/step_$v.json 2> $O/step_$v.err
done
echo ok
