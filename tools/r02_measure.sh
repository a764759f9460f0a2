#!/bin/bash
# Round-2 measurement set on one MI355X: every bench workload, the deployed turn-penalty
# configuration, the N = 2 gloo rehearsal of C3, and the FETCH/WRITE profile of the
# default bench (tools/profile_gpu.sh).  Results under gpurun_out/$1.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r02m}
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/c2.json 2> $O/c2.err
timeout -k 10 400 python3 bench.py --streams 1 --cpu-traces 0 --e2e-steps 0 > $O/c2_s1.json 2> $O/c2_s1.err
timeout -k 10 600 python3 bench.py --workload c4 > $O/c4.json 2> $O/c4.err
timeout -k 10 400 python3 bench.py --workload c5mix > $O/c5mix.json 2> $O/c5mix.err
timeout -k 10 400 python3 bench.py --cpu-traces 2000 --opt turn_penalty_factor=200 > $O/turn.json 2> $O/turn.err
OTR_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --workload c3 --traces-per-gpu 10000 \
  > $O/c3_n2_gloo.json 2> $O/c3_n2_gloo.err
echo benches done
bash tools/profile_gpu.sh
echo done
