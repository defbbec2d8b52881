# round 5: 150-step full-size convergence of the engine in bf16 / fp16 / fp32 on the same
# data and init (tools/converge.py), loss every 10 steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for p in bf16 fp16 fp32; do
  timeout -k 10 300 python -u tools/converge.py --steps 150 --precision $p > gpurun_out/conv_$p.log 2>&1 || { tail -20 gpurun_out/conv_$p.log; exit 1; }
  tail -1 gpurun_out/conv_$p.log
done
