#!/bin/bash
# --memory_first, shipped tree vs the QKV forward unfused from RoPE (fw4 + k_rope_qk_inplace)
# and the fused down-dgrad + SwiGLU backward pinned at M = 8192.
set -u
mkdir -p gpurun_out
python tools/ab/plan_variant.py gpurun_out/plan_rp.json fused:rope:8192x2304x768=false || exit 1
python tools/ab/plan_variant.py gpurun_out/plan_dsw.json fused:dswiglu:8192x3072x768=true || exit 1
python tools/ab/plan_variant.py gpurun_out/plan_rpdsw.json fused:rope:8192x2304x768=false fused:dswiglu:8192x3072x768=true || exit 1
VARIANTS="base:X=0 rp:DLT_GEMM_PLAN=gpurun_out/plan_rp.json dsw:DLT_GEMM_PLAN=gpurun_out/plan_dsw.json rpdsw:DLT_GEMM_PLAN=gpurun_out/plan_rpdsw.json" \
  REPS=${REPS:-2} BENCH_ARGS="--memory_first" bash tools/ab/env_ab.sh
