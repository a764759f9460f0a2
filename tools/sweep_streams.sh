#!/bin/bash
# Matchers (HIP streams + host threads) sharing one GPU's batch.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/streams
mkdir -p $O
for n in ${STREAMS:-1 2 3 4}; do
  timeout -k 10 150 python -u bench.py --steps 4 --warmup 2 --cpu-traces 0 --streams $n > $O/streams_$n.json 2> $O/streams_$n.err
done
echo done
