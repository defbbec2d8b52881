#!/bin/bash
# --memory_first (M = 8192 GEMMs, chunked head): M = 8192 forward pins and one head chunk
# per micro-step, interleaved (tok/s, ms, peak GB).
set -u
mkdir -p gpurun_out
python tools/ab/plan_variant.py gpurun_out/plan_m8.json fused:swiglu4:8192x6144x768=148 \
  tn:8192x2304x768=fw4:144 tn:8192x768x768=fw4:144 tn:8192x768x3072=fw4:144 || exit 1
VARIANTS="base:X=0 ch1:DLT_HEAD_CHUNKS=1 m8:DLT_GEMM_PLAN=gpurun_out/plan_m8.json m8ch1:DLT_GEMM_PLAN=gpurun_out/plan_m8.json,DLT_HEAD_CHUNKS=1" \
  REPS=${REPS:-2} BENCH_ARGS="--memory_first" bash tools/ab/env_ab.sh
