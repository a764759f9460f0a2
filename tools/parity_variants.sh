#!/bin/bash
# GPU parity of library variants (reporter_amd/libotr_<name>.so) — each in its own process.
# Usage: VARIANTS="h24 fretry" bash tools/parity_variants.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pv
mkdir -p $O
for v in $VARIANTS; do
  OTR_LIB=reporter_amd/libotr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_known_answers.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
