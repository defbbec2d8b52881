# round 5: bench.py table over the model / parallelism / precision configurations (1 GPU),
# then the 150-step convergence run, engine vs eager
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/bench_table.py --gpus 1 --steps 10 \
  --configs ddp_small,ddp_small_lean,ddp_small_fp16,ddp_small_fp32,ddp_small_hd128,fsdp_small,ddp_medium,fsdp_medium,fsdp_xl \
  --out gpurun_out/r5_bench_table.md > gpurun_out/r5_table.log 2>&1 || { tail -30 gpurun_out/r5_table.log; exit 1; }
cat gpurun_out/r5_bench_table.md
timeout -k 10 300 python -u tools/converge.py --steps 150 > gpurun_out/r5_conv_engine.log 2>&1 || { tail -20 gpurun_out/r5_conv_engine.log; exit 1; }
timeout -k 10 300 python -u tools/converge.py --steps 150 --eager > gpurun_out/r5_conv_eager.log 2>&1 || { tail -20 gpurun_out/r5_conv_eager.log; exit 1; }
tail -4 gpurun_out/r5_conv_engine.log; tail -4 gpurun_out/r5_conv_eager.log
