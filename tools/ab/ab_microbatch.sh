#!/bin/bash
set -u
mkdir -p gpurun_out
for cfg in "8 4" "16 2" "32 1" "8 4"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --steps 15 --warmup 3 --batch_size $1 --grad_accum $2 > gpurun_out/mb_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/mb_$1_$2.log; exit 1; }
  echo "B$1 GA$2: $(tail -1 gpurun_out/mb_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_gb_per_gpu"])')"
done
timeout -k 10 240 env DLT_PIPELINE=0 python -u bench.py --steps 15 --warmup 3 > gpurun_out/mb_seq.log 2>&1 && echo "B8 GA4 seq: $(tail -1 gpurun_out/mb_seq.log | cut -c1-120)"
