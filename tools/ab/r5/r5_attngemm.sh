# round 5: odd head_dim attention through the fp32 GEMM formulation (ops/attn_gemm.py) --
# kernel + engine tests, then the medium plan-pin A/B (r5_plan_medium.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py "tests/test_model_gpu.py::test_head_dim_128_trains_on_gpu" \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/ag_tests.log 2>&1 || { tail -40 gpurun_out/ag_tests.log; exit 1; }
tail -1 gpurun_out/ag_tests.log
bash tools/ab/r5/r5_plan_medium.sh
