#!/bin/bash
# --memory_first on the shipped tree (one head chunk, M = 8192 forward pins) vs pins for
# its other M = 8192 / T = 8192 GEMMs: hand data gradients, stream-K weight gradients,
# fw4 lm_head forward.  The base run prints the planner's race picks (stderr).
set -u
mkdir -p gpurun_out
python tools/ab/plan_variant.py gpurun_out/plan_dg8.json fused:dgrad:8192x768x2304=true fused:dgrad:8192x768x768=true \
  fused:dgrad:8192x768x6144=true || exit 1
python tools/ab/plan_variant.py gpurun_out/plan_sk8.json splitk:8192x2304x768=-1024 splitk:8192x768x768=-1024 \
  splitk:8192x6144x768=-1024 splitk:8192x768x3072=-1024 || exit 1
python tools/ab/plan_variant.py gpurun_out/plan_lm8.json tn:8192x50304x768=fw4:4100 || exit 1
VARIANTS="base:DLT_GEMM_REPORT=1 dg8:DLT_GEMM_PLAN=gpurun_out/plan_dg8.json sk8:DLT_GEMM_PLAN=gpurun_out/plan_sk8.json lm8:DLT_GEMM_PLAN=gpurun_out/plan_lm8.json" \
  REPS=${REPS:-2} BENCH_ARGS="--memory_first" bash tools/ab/env_ab.sh
