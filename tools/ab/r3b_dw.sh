#!/bin/bash
# Norm-weight column sums on an ordered side stream: bitwise tests, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "pipelined or bitwise or memory_lean or deferred or resume or forced or collectives or precision or rmsnorm or norm" > gpurun_out/dw_tests.log 2>&1 || { tail -30 gpurun_out/dw_tests.log; exit 1; }
tail -2 gpurun_out/dw_tests.log
VARIANTS='dw1:DLT_DW_STREAM=1 dw0:DLT_DW_STREAM=0' bash tools/ab/r3b_env_ab.sh
