#!/bin/bash
# A/B runner (one gpurun call): bench.py lines for library builds in alternating order.
# Usage: bash tools/ab.sh TAG WORKLOAD ROUNDS VARIANT... [-- extra bench args]
#   VARIANT = name (reporter_amd/libotr_<name>.so; "base" = reporter_amd/libotr.so), optionally
#   name:VAR=VAL[+VAR=VAL...] to run that library with those environment settings (A/B knobs)
# Each variant runs ROUNDS times, the order reversed every round (A B C, C B A, ...); the
# first line of every variant carries the oracle parity sample, the rest skip it.
# Lines: gpurun_out/TAG/<name>_<round>.json; summary: python tools/ab_summary.py gpurun_out/TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; WL=$2; ROUNDS=$3; shift 3
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
O=gpurun_out/$TAG
mkdir -p $O
for ((r = 0; r < ROUNDS; r++)); do
  if ((r % 2 == 0)); then ORD=("${V[@]}"); else ORD=(); for ((k = ${#V[@]} - 1; k >= 0; k--)); do ORD+=("${V[$k]}"); done; fi
  for v in "${ORD[@]}"; do
    n=${v%%:*}; EV=(); [ "$n" != "$v" ] && IFS=+ read -ra EV <<< "${v#*:}"
    tag=$(echo "$v" | tr ':=,+' '____')
    LIB=reporter_amd/libotr.so; [ "$n" != base ] && LIB=reporter_amd/libotr_$n.so
    CPU="--cpu-traces 0"; [ $r = 0 ] && CPU=""
    env "${EV[@]}" OTR_LIB=$PWD/$LIB timeout -k 10 300 python3 -u bench.py --workload $WL --e2e-steps 0 $CPU "$@" \
      > $O/${tag}_$r.json 2> $O/${tag}_$r.err || { echo "$v round $r failed"; tail -20 $O/${tag}_$r.err; exit 1; }
    echo "$v $r ok"
  done
done
