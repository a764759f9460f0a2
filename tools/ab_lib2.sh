#!/bin/bash
# A/B of the product library against one variant build (OTR_LIB) on C2 and C4, one GPU call.
# Usage: bash tools/ab_lib2.sh TAG VARIANT [tests]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ab2}; V=${2:-nosink}; mkdir -p $O
if [ "${3:-}" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_known_answers.py tests/test_semantics_kat.py tests/test_gpu_tiers.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
fi
B="python -u bench.py --cpu-traces 0 --e2e-steps 0"
timeout -k 10 200 $B > $O/c2.json 2> $O/c2.err
OTR_LIB=reporter_amd/libotr_$V.so timeout -k 10 200 $B > $O/c2_$V.json 2> $O/c2_$V.err
timeout -k 10 300 $B --workload c4 > $O/c4.json 2> $O/c4.err
OTR_LIB=reporter_amd/libotr_$V.so timeout -k 10 300 $B --workload c4 > $O/c4_$V.json 2> $O/c4_$V.err
echo ok
