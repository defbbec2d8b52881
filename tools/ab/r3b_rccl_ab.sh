#!/bin/bash
# One RCCL rank with every gradient bucket forced through RCCL: window-schedule variants (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
port=29531
for rep in 1 2; do
  for spec in ${VARIANTS:-ffbb:DLT_WINDOW_SCHED=ffbb fb:DLT_WINDOW_SCHED=fb ov0:DLT_WINDOW_SCHED=fb,DLT_BWD_OVERLAP=0}; do
    name=${spec%%:*}; kv=${spec#*:}
    port=$((port + 1))
    env DLT_FORCE_COLLECTIVES=1 $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 20 --warmup 3 $BENCH_ARGS > gpurun_out/rab_$name.$rep.log 2>&1 || { tail -20 gpurun_out/rab_$name.$rep.log; exit 1; }
    echo "$name $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/rab_$name.$rep.log | tr '\n' ' ')"
  done
done
