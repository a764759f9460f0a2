#!/bin/bash
# Runs a command with a heartbeat file under gpurun_out/ (a line every 20 s), so a long
# silent stretch (the country graph's generation) is not taken for a hang; the heartbeat
# stops with the command and the command's exit status is returned.
# Usage: bash tools/heartbeat_run.sh TAG CMD...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$1
HBF=gpurun_out/$1/heartbeat.txt
shift
(while sleep 20; do date +%T >> $HBF; done) &
HB=$!
"$@"
rc=$?
kill $HB 2>/dev/null
wait $HB 2>/dev/null
exit $rc
