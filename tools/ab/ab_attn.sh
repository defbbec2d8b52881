#!/bin/bash
# Attention kernel change: GPU numerics tests, standalone kernel timings (base vs new lib),
# then an alternating bench.py A/B.  usage: bash tools/ab/ab_attn.sh [rounds]
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attn or attention or dropout" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/attn_tests.log)"; [ $rc -eq 0 ] || exit $rc
for v in base new; do
  lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
  for b in 8 16; do
    DLT_KERNEL_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py --packed --B $b > gpurun_out/attn_$v$b.log 2>&1 || { echo "attn bench fail"; tail -5 gpurun_out/attn_$v$b.log; exit 1; }
    echo "$v B$b: $(tail -3 gpurun_out/attn_$v$b.log | tr '\n' ' ')"
  done
done
bash tools/ab/ab_kernels.sh ${1:-2}
