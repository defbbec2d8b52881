# round 5: blocked causal GEMMs for the GEMM-formulated attention (DLT_ATTN_BLOCKS=1 dense /
# 2 / 4) -- tests, fp32 step A/B, head_dim-160 route timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py "tests/test_model_gpu.py::test_head_dim_128_trains_on_gpu" \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/bl_tests.log 2>&1 || { tail -40 gpurun_out/bl_tests.log; exit 1; }
tail -1 gpurun_out/bl_tests.log
DLT_ATTN_BLOCKS=1 timeout -k 10 300 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/bl_tests1.log 2>&1 || { tail -40 gpurun_out/bl_tests1.log; exit 1; }
tail -1 gpurun_out/bl_tests1.log
for T in 1 4; do
  echo "T=$T hd160: $(DLT_ATTN_BLOCKS=$T timeout -k 10 200 python tools/bench_attn_gemm.py --hd 160 --nh 8 2>/dev/null | grep '^hd' | cut -c1-120)"
done
for r in 1 2; do
  for T in 1 2 4; do
    DLT_ATTN_BLOCKS=$T timeout -k 10 300 python bench.py --precision fp32 --steps 6 --warmup 3 > gpurun_out/bl.log 2>&1 || { tail -20 gpurun_out/bl.log; exit 1; }
    echo "$r fp32 T=$T: $(grep '"metric"' gpurun_out/bl.log | cut -c1-100)"
  done
done
