# round 5: head_dims without a flash kernel on zero-padded flash kernels -- tests, route
# timing, and the head_dim-96 model row
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py "tests/test_model_gpu.py::test_head_dim_128_trains_on_gpu" \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/ap_tests.log 2>&1 || { tail -40 gpurun_out/ap_tests.log; exit 1; }
tail -1 gpurun_out/ap_tests.log
timeout -k 10 300 python tools/bench_attn_gemm.py 2>/dev/null | grep -v GPU_MAX
timeout -k 10 300 python tools/bench_attn_gemm.py --hd 80 2>/dev/null | grep "^hd"
timeout -k 10 300 python tools/bench_table.py --gpus 1 --steps 10 --configs ddp_small,ddp_small_hd96 --out gpurun_out/ap_table.md > gpurun_out/ap_table.log 2>&1 \
  || { tail -20 gpurun_out/ap_table.log; exit 1; }
tail -2 gpurun_out/ap_table.md
