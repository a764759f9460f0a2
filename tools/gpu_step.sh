#!/bin/bash
# A/B of the route stage on one GPU call: the parity subset, the default bench line, and
# optionally the SQ counter passes (tools/profile_sq.sh).  Usage: bash tools/gpu_step.sh TAG [sq]
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-step}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_known_answers.py tests/test_semantics_kat.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-traces 2000 --e2e-steps 0 > $O/bench.json 2> $O/bench.err
if [ "${2:-}" = "sq" ]; then bash tools/profile_sq.sh ${1:-step}/sq; fi
echo ok
