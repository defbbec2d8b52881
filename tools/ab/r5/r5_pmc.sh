# round 5: hardware counters of the attention kernels (B16 packed) and of a whole step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab/pmc.sh r5attn tools/bench_attn.py --packed --B 16 --iters 3 && python tools/pmc_summary.py gpurun_out/pmc_r5attn 8 \
  > gpurun_out/r5_pmc_attn.md || exit 1
bash tools/ab/pmc.sh r5step bench.py --steps 2 --warmup 1 && python tools/pmc_summary.py gpurun_out/pmc_r5step 24 \
  > gpurun_out/r5_pmc_step.md || exit 1
cat gpurun_out/r5_pmc_attn.md gpurun_out/r5_pmc_step.md
