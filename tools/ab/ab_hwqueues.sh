#!/bin/bash
# HIP hardware queues vs an RCCL communicator (world size 1): RCCL's own streams take
# hardware queues, so the engine's two compute streams can land on one queue and run
# serialised.  Same-box A/B over GPU_MAX_HW_QUEUES.
mkdir -p gpurun_out
m() { grep -o '"ms_per_step": [0-9.]*' "$1" | cut -d' ' -f2; }
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1"
b() { timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3; }
i=0
for q in "" 8 16; do
  for mode in plain nccl forced; do
    i=$((i+1))
    case $mode in
      plain) args="";;
      nccl) args="$R MASTER_PORT=2956$i";;
      forced) args="$R MASTER_PORT=2956$i DLT_FORCE_COLLECTIVES=1";;
    esac
    qa=""; [ -n "$q" ] && qa="GPU_MAX_HW_QUEUES=$q"
    b $args $qa > gpurun_out/q_${mode}_$q.log 2>&1 || exit 1
    echo "queues=${q:-default} $mode: $(m gpurun_out/q_${mode}_$q.log)"
  done
done
