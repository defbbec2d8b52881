#!/bin/bash
# Same-box A/B of environment knobs on the default bench (alternating, 2 rounds).
# usage: bash tools/ab/ab_knobs.sh "NAME=VAL ..." "NAME=VAL ..." ...   ("" = defaults)
set -u
mkdir -p gpurun_out
for r in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/abn_${i}_${r}.log 2>&1 || { echo "fail [$cfg]"; tail -5 gpurun_out/abn_${i}_${r}.log; exit 1; }
    echo "[$cfg] #$r: $(tail -1 gpurun_out/abn_${i}_${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
