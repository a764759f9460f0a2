#!/bin/bash
# The other BASELINE workloads on one MI355X: C4, C5 mix (metro), C5 country, C3 N = 2 gloo
# rehearsal.  Usage: bash tools/r03_wl.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-wl}
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --workload c4 --e2e-steps 0 > $O/c4.json 2> $O/c4.err; echo c4 $?
timeout -k 10 400 python3 -u bench.py --workload c5mix --e2e-steps 0 > $O/c5mix.json 2> $O/c5mix.err; echo c5mix $?
timeout -k 10 700 python3 -u bench.py --workload c5 --e2e-steps 0 > $O/c5.json 2> $O/c5.err; echo c5 $?
OTR_BENCH_BACKEND=gloo timeout -k 10 500 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --workload c3 --traces-per-gpu 10000 \
  > $O/c3_n2_gloo.json 2> $O/c3_n2_gloo.err; echo c3 $?
timeout -k 10 400 python3 -u bench.py --cpu-traces 0 > $O/c2_e2e.json 2> $O/c2_e2e.err; echo c2 $?
