#!/bin/bash
# Attention timings split into keep-bit kernel / forward kernel / backward, with and without dropout.
set -u
mkdir -p gpurun_out
for s in "1024 8" "1024 16" "4096 2" "16384 1"; do
  set -- $s
  for p in 0.1 0.0; do
    timeout -k 10 120 python -u tools/bench_attn.py --packed --S $1 --B $2 --p $p > gpurun_out/asplit_$1_$2_$p.log 2>&1
    rc=$?; echo "S$1 B$2 p$p rc=$rc: $(grep -v amdgpu.ids gpurun_out/asplit_$1_$2_$p.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  done
done
