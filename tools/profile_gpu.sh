#!/bin/bash
# Round profile on a GPU box (run through gpurun from the repo root):
#   1. kernel-trace + stats of the default bench command
#   2./3. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (TCC slots: they do not fit one pass)
#   4./5. the same counters on tools/calib_fetch (known byte counts per access shape)
# Summaries: python tools/pmc_summary.py gpurun_out/prof > profiles/<round>_pmc.json
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
STEPS=${STEPS:-5}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --steps $STEPS --warmup 2 --cpu-traces 0 --e2e-steps 0 > $O/bench_kt.json 2> $O/bench_kt.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-traces 0 --e2e-steps 0 > $O/bench_$c.json 2> $O/bench_$c.err
  timeout -k 10 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/cal_$c -o run -- \
    ./reporter_amd/tools/calib_fetch > $O/calib.json 2> $O/calib_$c.err
done
echo done
