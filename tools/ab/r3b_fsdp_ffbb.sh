#!/bin/bash
# FSDP two-chain window ffbb vs fb: FSDP GPU tests, then A/B small and xl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py tests/test_cli_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "fsdp or ffbb or pipelined" > gpurun_out/fffbb_tests.log 2>&1 || { tail -30 gpurun_out/fffbb_tests.log; exit 1; }
tail -2 gpurun_out/fffbb_tests.log
BENCH_ARGS='--mode fsdp' VARIANTS='s_ffbb:DLT_WINDOW_SCHED=ffbb s_fb:DLT_WINDOW_SCHED=fb' bash tools/ab/r3b_env_ab.sh || exit 1
STEPS=3 BENCH_ARGS='--mode fsdp --model_size xl --batch_size 4 --grad_accum 8' VARIANTS='xl_ffbb:DLT_WINDOW_SCHED=ffbb xl_fb:DLT_WINDOW_SCHED=fb' bash tools/ab/r3b_env_ab.sh
