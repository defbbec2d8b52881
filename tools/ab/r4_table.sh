# round 4: bench.py table over the model / parallelism configurations (1 GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/bench_table.py --gpus 1 --configs ddp_small,ddp_small_lean,ddp_small_fp16,fsdp_small,ddp_medium,fsdp_medium,fsdp_xl \
  --out gpurun_out/${TAG:-r4}_bench_table.md > gpurun_out/r4_table.log 2>&1 || { tail -30 gpurun_out/r4_table.log; exit 1; }
cat gpurun_out/${TAG:-r4}_bench_table.md
