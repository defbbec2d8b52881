# round 4, end: 150-step full-size convergence of the engine (3 seeds) after the session-2 changes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for seed in 1234 1 2; do
  timeout -k 10 300 python -u tools/converge.py --steps 150 --seed $seed > gpurun_out/conv2_engine_$seed.log 2>&1 || { tail -20 gpurun_out/conv2_engine_$seed.log; exit 1; }
  tail -1 gpurun_out/conv2_engine_$seed.log
done
