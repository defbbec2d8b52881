#!/bin/bash
# A/B of one env knob on one box: bench.py for each value, two alternating rounds.
# usage: VAR=DLT_CE_CHUNKS VALUES="1 4 8" bash tools/ab/ab_env.sh
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_${VAR}_${v}_$r.log 2>&1 || { tail -5 gpurun_out/ab_${VAR}_${v}_$r.log; exit 1; }
    echo "$VAR=$v round $r: $(grep '"metric"' gpurun_out/ab_${VAR}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
  done
done
