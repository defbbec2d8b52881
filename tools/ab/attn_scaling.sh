#!/bin/bash
# Attention kernel time vs batch (S = 1024): tail / per-item overhead diagnosis.
set -u
mkdir -p gpurun_out
for b in 4 8 16 32 64; do
  for p in 0.0 0.1; do
    timeout -k 10 120 python -u tools/bench_attn.py --packed --S 1024 --B $b --p $p > gpurun_out/ascale_${b}_${p}.log 2>&1
    rc=$?; echo "B$b p$p rc=$rc: $(grep -v amdgpu.ids gpurun_out/ascale_${b}_${p}.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  done
done
