# round 5: RMSNorm backward with the dw column sum folded into the kernel (no k_colsum_acc
# launch): norm / model tests, then a same-box step A/B against DLT_NORM_FOLD=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "norm" \
  > gpurun_out/nf_tests.log 2>&1 || { tail -30 gpurun_out/nf_tests.log; exit 1; }
tail -2 gpurun_out/nf_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  -k "matches_sequential or bitwise or repro or fp32_eager" > gpurun_out/nf_model.log 2>&1 || { tail -30 gpurun_out/nf_model.log; exit 1; }
tail -2 gpurun_out/nf_model.log
REPS=3 VARIANTS="fold:DLT_NORM_FOLD=1 sep:DLT_NORM_FOLD=0" bash tools/ab/env_ab.sh
