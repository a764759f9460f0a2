#!/bin/bash
# One GPU measurement set (run through gpurun from the repo root): the GPU tests selected
# by $TESTS (default: the whole -m gpu suite; "none" skips them), then the bench workloads
# given, each under its own time limit.  Results under gpurun_out/TAG.
# A step that times out, aborts or faults ends the call (nothing more runs on the GPU).
# Usage: TESTS="tests/test_gpu_tiers.py -k edge" bash tools/run_set.sh TAG [WORKLOAD...]
#   workloads: c2 c1 c2dep c4 c5mix c5 c3n2 c2dep_noresume c3w1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-set}
mkdir -p $O
shift
W=("$@")
fatal() {  # time limit, abort, segfault, signal: stop here
  case $1 in 124|134|137|139) return 0 ;; esac
  [ "$1" -gt 128 ] && return 0
  return 1
}
step() {  # step NAME SECONDS CMD...: run, report, stop the call on a fatal status
  local name=$1 secs=$2
  shift 2
  timeout -k 10 $secs "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "$name $rc"
  if fatal $rc; then echo "$name: fatal status $rc, stopping"; tail -20 $O/$name.err; exit $rc; fi
}
T=${TESTS:-tests}
if [ "$T" != none ]; then
  timeout -k 10 ${TEST_SECS:-900} python3 -u -m pytest $T -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  echo "tests $rc"; tail -3 $O/pytest_gpu.log
  if fatal $rc; then exit $rc; fi
fi
for w in "${W[@]}"; do
  case $w in
    c2) step c2 300 python3 -u bench.py ;;
    c1) step c1 300 python3 -u bench.py --workload c1 --e2e-steps 0 ;;
    c2dep) step c2dep 300 python3 -u bench.py --workload c2dep --e2e-steps 0 ;;
    c2dep_noresume) OTR_E1RESUME=0 step c2dep_noresume 300 python3 -u bench.py --workload c2dep --e2e-steps 0 ;;
    c4) step c4 300 python3 -u bench.py --workload c4 --e2e-steps 0 ;;
    c5mix) step c5mix 200 python3 -u bench.py --workload c5mix --e2e-steps 0 ;;
    c5) step c5 400 python3 -u bench.py --workload c5 --e2e-steps 0 ;;
    c3w1) step c3_w1_rccl 600 python3 -u bench.py --dist --workload c3 --e2e-steps 0 ;;
    c3n2) OTR_BENCH_BACKEND=gloo step c3_n2_gloo 600 python3 -u -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 ;;
  esac
done
echo done
