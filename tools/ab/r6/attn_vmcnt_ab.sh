#!/bin/bash
# Attention DMA-overlap fix: GPU attention tests, isolated kernels (B16 packed, the step's
# shape) and the step, base (_dlt_kernels_base.so = HEAD) vs new, alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or dropout" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "attn tests rc=$rc: $(tail -1 gpurun_out/attn_tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base new; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    DLT_KERNEL_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py --B 16 --packed --iters 50 > gpurun_out/attn_$v$r.log 2>&1 || { echo "attn bench fail $v"; tail -5 gpurun_out/attn_$v$r.log; exit 1; }
    echo "$v#$r attn: $(tr '\n' ' ' < gpurun_out/attn_$v$r.log | tail -c 300)"
  done
done
bash tools/ab/kernels_ab.sh 3
