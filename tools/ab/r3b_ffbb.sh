#!/bin/bash
# ffbb two-chain window: bitwise tests, then A/B against the fb schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "pipelined or ffbb or bitwise or memory_lean or deferred or resume or forced or collectives or precision" > gpurun_out/ffbb_tests.log 2>&1 || { tail -30 gpurun_out/ffbb_tests.log; exit 1; }
tail -2 gpurun_out/ffbb_tests.log
VARIANTS='ffbb:DLT_WINDOW_SCHED=ffbb fb:DLT_WINDOW_SCHED=fb' bash tools/ab/r3b_env_ab.sh
