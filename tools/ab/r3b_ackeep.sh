#!/bin/bash
# Activation checkpointing that keeps the normed inputs and the SwiGLU output too (within the budget):
# recompute GPU tests, then FSDP small / medium / xl A/B against DLT_AC_KEEP_REST=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "recompute or fsdp or ac or checkpoint" > gpurun_out/ack_tests.log 2>&1 || { tail -30 gpurun_out/ack_tests.log; exit 1; }
tail -2 gpurun_out/ack_tests.log
BENCH_ARGS='--mode fsdp' VARIANTS='s_keep:DLT_AC_KEEP_REST=1 s_rec:DLT_AC_KEEP_REST=0' bash tools/ab/r3b_env_ab.sh || exit 1
STEPS=5 BENCH_ARGS='--mode fsdp --model_size medium --batch_size 4 --grad_accum 8' VARIANTS='m_keep:DLT_AC_KEEP_REST=1 m_rec:DLT_AC_KEEP_REST=0' bash tools/ab/r3b_env_ab.sh || exit 1
STEPS=3 BENCH_ARGS='--mode fsdp --model_size xl --batch_size 4 --grad_accum 8' VARIANTS='xl_keep:DLT_AC_KEEP_REST=1 xl_rec:DLT_AC_KEEP_REST=0' bash tools/ab/r3b_env_ab.sh
