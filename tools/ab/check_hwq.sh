#!/bin/bash
# The package raises GPU_MAX_HW_QUEUES itself: bench.py alone and with an RCCL communicator.
mkdir -p gpurun_out
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
m() { grep -o '"ms_per_step": [0-9.]*' "$1" | cut -d' ' -f2; }
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1"
b() { timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3; }
b > gpurun_out/h_plain.log 2>&1 || exit 1; echo "plain          $(m gpurun_out/h_plain.log)"
b $R MASTER_PORT=29571 > gpurun_out/h_nccl.log 2>&1 || exit 1; echo "nccl           $(m gpurun_out/h_nccl.log)"
b $R MASTER_PORT=29572 DLT_FORCE_COLLECTIVES=1 > gpurun_out/h_forced.log 2>&1 || exit 1; echo "nccl forced    $(m gpurun_out/h_forced.log)"
b $R MASTER_PORT=29573 DLT_HW_QUEUES=0 > gpurun_out/h_nccl4.log 2>&1 || exit 1; echo "nccl, 4 queues $(m gpurun_out/h_nccl4.log)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29574 bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/h_tr.log 2>&1 || exit 1
echo "torchrun       $(m gpurun_out/h_tr.log)"
