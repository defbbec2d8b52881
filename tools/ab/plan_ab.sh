#!/bin/bash
# Same-box A/B of two GEMM plan files over the bench-table configurations (alternating).
# usage: bash tools/ab/ab_plan.sh PLAN_A PLAN_B
set -u
mkdir -p gpurun_out
A=$1; B=$2
for cfg in "ddp small 8 4" "fsdp small 8 4" "ddp medium 4 8" "fsdp medium 4 8" "ddp xl 4 8"; do
  set -- $cfg
  for p in "$A" "$B" "$A" "$B"; do
    DLT_GEMM_PLAN=$p timeout -k 10 300 python -u bench.py --mode $1 --model_size $2 --batch_size $3 --grad_accum $4 --steps 6 --warmup 2 > gpurun_out/abp.log 2>&1 || { echo "fail $cfg $p"; tail -5 gpurun_out/abp.log; exit 1; }
    echo "$1 $2 [$(basename $p)]: $(tail -1 gpurun_out/abp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
