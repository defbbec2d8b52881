# round 5: 16-bit GEMM-formulated attention for head_dims without a flash kernel -- tests
# (kernel + engine), then the route timing (tools/bench_attn_gemm.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py "tests/test_model_gpu.py::test_head_dim_128_trains_on_gpu" \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/a16_tests.log 2>&1 || { tail -40 gpurun_out/a16_tests.log; exit 1; }
tail -1 gpurun_out/a16_tests.log
timeout -k 10 300 python tools/bench_attn_gemm.py > gpurun_out/a16_bench.log 2>&1 || { tail -20 gpurun_out/a16_bench.log; exit 1; }
cat gpurun_out/a16_bench.log
timeout -k 10 300 python tools/bench_attn_gemm.py --hd 80 --nh 8 | head -1
