#!/bin/bash
# AdamW with nontemporal loads/stores (default) vs plain (DLT_ADAMW_NT=0), same box.
mkdir -p gpurun_out
m() { grep -o '"ms_per_step": [0-9.]*' "$1" | cut -d' ' -f2; }
for nt in 0 1; do
  DLT_ADAMW_NT=$nt timeout -k 10 200 python tools/bench_ops.py > gpurun_out/ops_nt$nt.md 2>&1 || exit 1
  echo "NT=$nt $(grep -E 'adamw|sumsq' gpurun_out/ops_nt$nt.md | tr '\n' ' ')"
done
for r in 1 2; do for nt in 0 1; do
  DLT_ADAMW_NT=$nt timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_nt$nt.log 2>&1 || exit 1
  echo "bench NT=$nt: $(m gpurun_out/b_nt$nt.log)"
done; done
