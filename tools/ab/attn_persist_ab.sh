#!/bin/bash
# dK/dV: persistent walk vs one item per workgroup, across batch sizes (S = 1024).
set -u
mkdir -p gpurun_out
for b in 8 16 64; do
  for per in 0 1; do
    DLT_ATTN_PERSIST=$per timeout -k 10 120 python -u tools/bench_attn.py --packed --S 1024 --B $b --p 0.1 > gpurun_out/ap_${b}_${per}.log 2>&1
    rc=$?; echo "B$b persist=$per rc=$rc: $(grep -v amdgpu.ids gpurun_out/ap_${b}_${per}.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  done
done
for per in 0 1; do
  DLT_ATTN_PERSIST=$per timeout -k 10 120 python -u tools/bench_attn.py --packed --S 4096 --B 4 --p 0.1 > gpurun_out/ap_s4k_${per}.log 2>&1
  echo "S4096 B4 persist=$per: $(grep -v amdgpu.ids gpurun_out/ap_s4k_${per}.log | tr '\n' ' ')"
done
