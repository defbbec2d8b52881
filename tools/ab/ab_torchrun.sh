#!/bin/bash
# Same-box A/B of the single-GPU bench under different launch modes (what does the
# distributed setup itself cost at world size 1?).
mkdir -p gpurun_out
m() { grep -o '"ms_per_step": [0-9.]*' "$1" | cut -d' ' -f2; }
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1"
b() { timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3; }
b > gpurun_out/v_plain.log 2>&1 || exit 1; echo "plain python            $(m gpurun_out/v_plain.log)"
b $R MASTER_PORT=29541 > gpurun_out/v_envnccl.log 2>&1 || exit 1; echo "env rank, nccl          $(m gpurun_out/v_envnccl.log)"
b $R MASTER_PORT=29542 DLT_BACKEND=gloo > gpurun_out/v_envgloo.log 2>&1 || exit 1; echo "env rank, gloo          $(m gpurun_out/v_envgloo.log)"
b $R MASTER_PORT=29543 TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 > gpurun_out/v_envnccl_nowd.log 2>&1 || exit 1
echo "env rank, nccl, no monitor $(m gpurun_out/v_envnccl_nowd.log)"
timeout -k 10 300 env DLT_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/v_trgloo.log 2>&1 || exit 1
echo "torchrun gloo           $(m gpurun_out/v_trgloo.log)"
b > gpurun_out/v_plain2.log 2>&1 || exit 1; echo "plain python            $(m gpurun_out/v_plain2.log)"
