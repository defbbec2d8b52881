#!/bin/bash
# Cross-entropy: 1024-thread rows (7 chunks/thread, 64 VGPRs, 2 blocks/CU) vs 512-thread rows (13 chunks, 94 VGPRs).
mkdir -p gpurun_out
DLT_CE_THREADS=1024 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -q -k cross_entropy --timeout 120 > gpurun_out/ce_t.log 2>&1 || { tail -20 gpurun_out/ce_t.log; exit 1; }
tail -1 gpurun_out/ce_t.log
for t in 512 1024; do
  DLT_CE_THREADS=$t timeout -k 10 200 python tools/bench_ops.py > gpurun_out/ce_ops_$t.md 2>&1 || exit 1
  echo "threads=$t $(grep cross gpurun_out/ce_ops_$t.md)"
done
for r in 1 2; do for t in 512 1024; do
  DLT_CE_THREADS=$t timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ce_b.log 2>&1 || exit 1
  echo "bench threads=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ce_b.log)"
done; done
