#!/bin/bash
# Overlapped backwards under FSDP: bitwise tests, then A/B small and xl (AC on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_cli_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "fsdp" > gpurun_out/fov_tests.log 2>&1 || { tail -30 gpurun_out/fov_tests.log; exit 1; }
tail -2 gpurun_out/fov_tests.log
BENCH_ARGS='--mode fsdp' VARIANTS='s_ov1:DLT_BWD_OVERLAP=1 s_ov0:DLT_BWD_OVERLAP=0' bash tools/ab/r3b_env_ab.sh || exit 1
STEPS=3 BENCH_ARGS='--mode fsdp --model_size xl --batch_size 4 --grad_accum 8' VARIANTS='xl_ov1:DLT_BWD_OVERLAP=1 xl_ov0:DLT_BWD_OVERLAP=0' bash tools/ab/r3b_env_ab.sh
