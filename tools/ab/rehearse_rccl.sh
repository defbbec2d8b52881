#!/bin/bash
# bench.py's DDP path over RCCL on ONE GPU: torch.distributed.run with one rank and the
# nccl (RCCL) backend, with and without DLT_FORCE_COLLECTIVES=1 (every gradient bucket
# all-reduced through RCCL from the weight-gradient stream, as on a multi-GPU node; a
# 1-rank all-reduce moves no link traffic, so the difference is the schedule's own cost:
# RCCL kernel launches, their CU occupancy next to the backward, stream waits).
mkdir -p gpurun_out
set -o pipefail
run() {  # $1 = tag, $2 = port, rest = env
  local tag=$1 port=$2; shift 2
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus 1 --steps 20 --warmup 3 > "gpurun_out/rccl_$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(grep '"metric"' "gpurun_out/rccl_$tag.log" | cut -c1-170)"
  return $rc
}
run plain 29521 DLT_FORCE_COLLECTIVES=0 && run forced 29522 DLT_FORCE_COLLECTIVES=1 && \
run plain2 29523 DLT_FORCE_COLLECTIVES=0 && run forced2 29524 DLT_FORCE_COLLECTIVES=1
