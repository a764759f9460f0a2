set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6a
timeout -k 10 240 env OTR_LIB=reporter_amd/libotr_ndall.so OTR_TIERS=256,448x2,768,2048 OTR_EST_K=0.7 python tools/determinism.py --workload c4 --runs 8 > gpurun_out/r6a/ndall_est07.json 2> gpurun_out/r6a/ndall_est07.err && \
timeout -k 10 240 env OTR_LIB=reporter_amd/libotr_ndall.so OTR_TIERS=256,448x2,768,2048 OTR_EST_K=0.7 OTR_NDUMP_GB=0.05 python tools/determinism.py --workload c4 --runs 6 > gpurun_out/r6a/ndall_est07_small.json 2> gpurun_out/r6a/ndall_est07_small.err && \
timeout -k 10 240 python tools/determinism.py --workload c4 --runs 6 > gpurun_out/r6a/base.json 2> gpurun_out/r6a/base.err
echo rc=$?
