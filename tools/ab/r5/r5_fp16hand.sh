# round 5: fp16 activations on the hand-written forward GEMM and the fused down-dgrad +
# SwiGLU-backward kernel (HK = 1 instances): GEMM / model tests, then a same-box
# --precision fp16 step A/B against DLT_GEMM_FP16_HAND=0 (hipBLASLt + unfused)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_bf16 or down_swiglu or planner or fp16" > gpurun_out/f16h_tests.log 2>&1 || { tail -30 gpurun_out/f16h_tests.log; exit 1; }
tail -2 gpurun_out/f16h_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "fp16" \
  > gpurun_out/f16h_model.log 2>&1 || { tail -30 gpurun_out/f16h_model.log; exit 1; }
tail -2 gpurun_out/f16h_model.log
REPS=3 BENCH_ARGS="--precision fp16" VARIANTS="${VARIANTS:-hand:DLT_GEMM_FP16_HAND=1 lib:DLT_GEMM_FP16_HAND=0}" bash tools/ab/env_ab.sh
