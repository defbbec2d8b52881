# round 4, final tree: hardware counters (rocprofv3 --pmc, 3 passes each) for the attention
# kernels at the fused-chain shape and for a whole bench.py step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/ab/pmc.sh r4attn tools/bench_attn.py --packed --B 16 --iters 3 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r4attn 6 > gpurun_out/pmc_r4attn.md || exit 1
bash tools/ab/pmc.sh r4step bench.py --steps 2 --warmup 1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r4step 24 > gpurun_out/pmc_r4step.md || exit 1
cat gpurun_out/pmc_r4attn.md gpurun_out/pmc_r4step.md
