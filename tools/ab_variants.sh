#!/bin/bash
# A/B of library variants (reporter_amd/libotr_<name>.so, built with
# python -m reporter_amd.build --variant <name> DEFS...): GPU parity of each variant,
# then single-stream bench lines, alternating base and variants twice.
# Usage: VARIANTS="h24 adjb" bash tools/ab_variants.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab
mkdir -p $O
for v in $VARIANTS; do
  OTR_LIB=reporter_amd/libotr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_known_answers.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
done
for rep in 1 2; do
  for v in base $VARIANTS; do
    lib=reporter_amd/libotr_$v.so
    [ "$v" = base ] && lib=reporter_amd/libotr.so
    OTR_LIB=$lib timeout -k 10 150 python -u bench.py --steps 5 --warmup 2 --cpu-traces 0 --streams 1 ${BENCH_ARGS} > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
  done
done
echo done
