# round 5: wave-per-row softmax / dsoftmax row kernels (attn_gemm.hip) -- tests, isolated
# timing, fp32 step A/B vs the block-per-row kernels (DLT_ATTN_ROW_WAVE=0), hd96 GEMM route
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/rw_tests.log 2>&1 || { tail -40 gpurun_out/rw_tests.log; exit 1; }
tail -1 gpurun_out/rw_tests.log
DLT_ATTN_ROW_WAVE=0 timeout -k 10 300 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "attention or attn_gemm" > gpurun_out/rw_tests0.log 2>&1 || { tail -40 gpurun_out/rw_tests0.log; exit 1; }
tail -1 gpurun_out/rw_tests0.log
for w in 0 1; do
  echo "row wave $w: $(DLT_ATTN_ROW_WAVE=$w timeout -k 10 200 python tools/bench_f32_ops.py 2>/dev/null | grep 'attn ' | tr -s ' ' | tr '\n' ';')"
done
for r in 1 2; do
  for w in 0 1; do
    DLT_ATTN_ROW_WAVE=$w timeout -k 10 300 python bench.py --precision fp32 --steps 6 --warmup 3 > gpurun_out/rw.log 2>&1 || { tail -20 gpurun_out/rw.log; exit 1; }
    echo "$r fp32 wave=$w: $(grep '"metric"' gpurun_out/rw.log | cut -c1-100)"
  done
done
