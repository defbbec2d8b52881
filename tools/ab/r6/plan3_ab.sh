#!/bin/bash
# Three-way in-step A/B of the lm_head forward pin: shipped vs two variants (plan files
# written by tools/ab/plan_variant.py), interleaved.  usage: plan3_ab.sh PIN_B PIN_C [rounds]
set -u
mkdir -p gpurun_out
B=$1; C=$2; R=${3:-3}
python tools/ab/plan_variant.py gpurun_out/plan_b.json tn:16384x50304x768=$B || exit 1
python tools/ab/plan_variant.py gpurun_out/plan_c.json tn:16384x50304x768=$C || exit 1
for r in $(seq 1 $R); do
  for v in a b c; do
    if [ $v = a ]; then unset DLT_GEMM_PLAN; else export DLT_GEMM_PLAN=gpurun_out/plan_$v.json; fi
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/p3_$v$r.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/p3_$v$r.log; exit 1; }
    echo "$v#$r: $(tail -1 gpurun_out/p3_$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
