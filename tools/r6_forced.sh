set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6f
OTR_LIB=$PWD/reporter_amd/libotr_unfixed.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k forced > gpurun_out/r6f/unfixed.log 2>&1; echo "unfixed rc=$?"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r6f/fixed.log 2>&1; echo "fixed rc=$?"
