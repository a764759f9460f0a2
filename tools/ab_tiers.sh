#!/bin/bash
# Retry-tier lists (OTR_TIERS) on C4 and C2, one bench line each.  Usage: bash tools/ab_tiers.sh TAG LIST...
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-abtiers}; shift; mkdir -p $O
B="python -u bench.py --cpu-traces 0 --e2e-steps 0"
for t in "$@"; do
  n=$(echo "$t" | tr ',' '_')
  OTR_TIERS=$t timeout -k 10 300 $B --workload c4 > $O/c4_$n.json 2> $O/c4_$n.err
done
for t in "$@"; do
  n=$(echo "$t" | tr ',' '_')
  OTR_TIERS=$t timeout -k 10 200 $B > $O/c2_$n.json 2> $O/c2_$n.err
done
echo ok
