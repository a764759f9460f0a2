#!/bin/bash
# Round-6 measurement set on one MI355X (one gpurun call): the GPU test suite, then every
# bench workload (C2 headline with CPU baseline, parity sample and host-to-host leg; C1;
# the deployed configuration; C4; C5 mode mix; C5 country; the C3 N = 2 gloo rehearsal with
# BASELINE config 3's default 1M uuids; the RCCL branch at world size 1, bench --dist).  Results under gpurun_out/$1.  Profiles: tools/profile_set.sh, tools/profile_sq.sh.
# A step that times out, aborts or faults ends the call (nothing more runs on the GPU).
# Usage: bash tools/r06_final.sh TAG [notests] [WORKLOAD...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r06f}
mkdir -p $O
shift
T=${1:-}
[ $# -gt 0 ] && shift
W=("$@")
[ ${#W[@]} -eq 0 ] && W=(c2 c1 c2dep c4 c5mix c5 c3n2 c3w1)
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
if [ "$T" != notests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  echo "tests $rc"; tail -2 $O/pytest_gpu.log
  if fatal $rc; then exit $rc; fi
fi
for w in "${W[@]}"; do
  case $w in
    c2) step c2 300 python3 -u bench.py ;;
    c1) step c1 300 python3 -u bench.py --workload c1 --e2e-steps 0 ;;
    c2dep) step c2dep 300 python3 -u bench.py --workload c2dep --e2e-steps 0 ;;
    c4) step c4 300 python3 -u bench.py --workload c4 --e2e-steps 0 ;;
    c5mix) step c5mix 200 python3 -u bench.py --workload c5mix --e2e-steps 0 ;;
    c5) step c5 400 python3 -u bench.py --workload c5 --e2e-steps 0 ;;
    c3n2) OTR_BENCH_BACKEND=gloo step c3_n2_gloo 600 python3 -u -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 ;;
    c3w1) MASTER_ADDR=127.0.0.1 MASTER_PORT=29543 step c3_w1_rccl 300 python3 -u bench.py --dist --e2e-steps 0 ;;
  esac
done
echo done
