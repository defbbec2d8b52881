#!/bin/bash
# bench.py's multi-rank paths rehearsed on ONE GPU (ranks share it over gloo).
mkdir -p gpurun_out
set -o pipefail
export DLT_BACKEND=gloo DLT_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 1 > gpurun_out/mr_ddp.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --mode fsdp > gpurun_out/mr_fsdp.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 2 --warmup 1 > gpurun_out/mr_ddp4.log 2>&1
rc=$?
for f in mr_ddp mr_fsdp mr_ddp4; do echo "$f: $(tail -1 gpurun_out/$f.log | cut -c1-260)"; done
exit $rc
