#!/bin/bash
# Round-2 closing measurement set on one MI355X (one gpurun call): the GPU test suite,
# every bench workload (C2 headline with CPU baseline, parity sample and end-to-end leg;
# C4 at BASELINE size; C5 mode mix; the deployed turn penalties; the C3 N = 2 gloo
# rehearsal), then tools/profile_gpu.sh (kernel trace + FETCH/WRITE passes).
# Results under gpurun_out/$1 and gpurun_out/prof.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r02f}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo tests done
timeout -k 10 400 python3 -u bench.py > $O/c2.json 2> $O/c2.err
timeout -k 10 600 python3 -u bench.py --workload c4 > $O/c4.json 2> $O/c4.err
timeout -k 10 400 python3 -u bench.py --workload c5mix > $O/c5mix.json 2> $O/c5mix.err
timeout -k 10 400 python3 -u bench.py --cpu-traces 2000 --opt turn_penalty_factor=200 > $O/turn.json 2> $O/turn.err
OTR_BENCH_BACKEND=gloo timeout -k 10 500 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --workload c3 --traces-per-gpu 10000 \
  > $O/c3_n2_gloo.json 2> $O/c3_n2_gloo.err
echo benches done
bash tools/profile_gpu.sh
echo done
