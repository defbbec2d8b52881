#!/bin/bash
# --memory_first: stream-K for ONE T = 8192 weight gradient at a time vs the raced picks.
set -u
mkdir -p gpurun_out
for r in 2304x768 768x768 6144x768 768x3072; do
  python tools/ab/plan_variant.py gpurun_out/plan_sk_$r.json splitk:8192x$r=-1024 || exit 1
done
VARIANTS="base:X=0 skqkv:DLT_GEMM_PLAN=gpurun_out/plan_sk_2304x768.json sko:DLT_GEMM_PLAN=gpurun_out/plan_sk_768x768.json skgu:DLT_GEMM_PLAN=gpurun_out/plan_sk_6144x768.json skdn:DLT_GEMM_PLAN=gpurun_out/plan_sk_768x3072.json" \
  REPS=${REPS:-2} BENCH_ARGS="--memory_first" bash tools/ab/env_ab.sh
