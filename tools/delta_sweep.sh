set -e -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/dsweep
for d in 40 80 120; do
  timeout -k 10 240 python3 -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-traces 0 --e2e-steps 0 --delta $d > gpurun_out/dsweep/c4_$d.json 2> gpurun_out/dsweep/c4_$d.err
done
for d in 45 75; do
  timeout -k 10 240 python3 -u bench.py --steps 5 --cpu-traces 0 --e2e-steps 0 --delta $d > gpurun_out/dsweep/c2_$d.json 2> gpurun_out/dsweep/c2_$d.err
done
timeout -k 10 240 python3 -u bench.py --steps 5 --cpu-traces 0 --e2e-steps 0 > gpurun_out/dsweep/c2_60.json 2> gpurun_out/dsweep/c2_60.err
