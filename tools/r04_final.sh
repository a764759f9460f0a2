#!/bin/bash
# Round-4 measurement set on one MI355X (one gpurun call): the GPU test suite, then every
# bench workload (C2 headline with CPU baseline, parity sample and host-to-host leg; C1;
# the deployed configuration; C4; C5 mode mix; C5 country; the C3 N = 2 gloo rehearsal with
# BASELINE config 3's default 1M uuids).  Results under gpurun_out/$1.  Profiles: tools/r04_profile.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04f}
mkdir -p $O
if [ "${2:-}" != notests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1
  echo tests $?; tail -2 $O/pytest_gpu.log
fi
timeout -k 10 300 python3 -u bench.py > $O/c2.json 2> $O/c2.err || { echo c2 failed; tail -20 $O/c2.err; exit 1; }
echo c2 done
timeout -k 10 300 python3 -u bench.py --workload c1 --e2e-steps 0 > $O/c1.json 2> $O/c1.err; echo c1 $?
timeout -k 10 300 python3 -u bench.py --workload c2dep --e2e-steps 0 > $O/c2dep.json 2> $O/c2dep.err; echo c2dep $?
timeout -k 10 300 python3 -u bench.py --workload c4 --e2e-steps 0 > $O/c4.json 2> $O/c4.err; echo c4 $?
timeout -k 10 200 python3 -u bench.py --workload c5mix --e2e-steps 0 > $O/c5mix.json 2> $O/c5mix.err; echo c5mix $?
timeout -k 10 400 python3 -u bench.py --workload c5 --e2e-steps 0 > $O/c5.json 2> $O/c5.err; echo c5 $?
OTR_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 > $O/c3_n2_gloo.json 2> $O/c3_n2_gloo.err; echo c3 $?
