#!/bin/bash
# Round-4 check on one MI355X (one gpurun call): the deployed-configuration bench (C2 traces,
# turn penalties on), the C2 headline, then optionally the GPU test suite.  Every bench line
# carries its oracle sample; a mismatch ends the call.  Results under gpurun_out/$1.
# Usage: bash tools/r04_check.sh TAG [tests] [extra bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04}
mkdir -p $O
shift
T=${1:-}
shift
timeout -k 10 300 python3 -u bench.py --workload c2dep --e2e-steps 0 "$@" > $O/c2dep.json 2> $O/c2dep.err || { echo c2dep failed; tail -30 $O/c2dep.err; exit 1; }
echo c2dep ok
timeout -k 10 300 python3 -u bench.py --e2e-steps 0 "$@" > $O/c2.json 2> $O/c2.err || { echo c2 failed; tail -30 $O/c2.err; exit 1; }
echo c2 ok
if [ "$T" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  echo tests $?
  tail -5 $O/pytest.log
fi
if [ "$T" = n2 ] || [ "$T" = tests ]; then
  OTR_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 > $O/c3_n2_gloo.json 2> $O/c3_n2_gloo.err
  echo c3_n2 $?
fi
