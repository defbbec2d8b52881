#!/bin/bash
# Stream-K weight gradient: kernel + planner GPU tests, then the step A/B against split-K.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "wgrad or planner or stream" > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
PLANS='sk: prev:splitk/32768x6144x768=-8,splitk/32768x50304x768=-2' bash tools/ab/r3b_plan_ab.sh
