#!/bin/bash
# A/B of a library variant on one workload: the default libotr.so, then OTR_LIB=$2, then
# the default again (box drift).  Usage: bash tools/r03_ab_lib.sh TAG reporter_amd/libotr_X.so [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-ab}; V=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --cpu-traces 0 --e2e-steps 0 "$@" > $O/a1.json 2> $O/a1.err || exit 1
OTR_LIB=$V timeout -k 10 300 python -u bench.py --cpu-traces 0 --e2e-steps 0 "$@" > $O/b.json 2> $O/b.err || exit 1
timeout -k 10 300 python -u bench.py --cpu-traces 0 --e2e-steps 0 "$@" > $O/a2.json 2> $O/a2.err || exit 1
echo done
