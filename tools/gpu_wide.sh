#!/bin/bash
# The route-tier test subset, then the C2 and C4 bench lines (no CPU sample).  Usage: bash tools/gpu_wide.sh TAG
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-wide}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_known_answers.py tests/test_semantics_kat.py tests/test_gpu_tiers.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
B="python -u bench.py --cpu-traces 0 --e2e-steps 0"
timeout -k 10 200 $B > $O/c2.json 2> $O/c2.err
timeout -k 10 300 $B --workload c4 > $O/c4.json 2> $O/c4.err
echo ok
