#!/bin/bash
# Deferred-store GEMM epilogue: bitwise vs the immediate-store kernel, timings vs hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 tools/cpp/gemm_bench blas,bf16,imm 16384 2304 768 16384 768 768 16384 6144 768 16384 768 3072 \
  16384 768 2304 16384 768 6144 16384 3072 768 16384 50304 768 > gpurun_out/defer_gemm.log 2>&1 || { cat gpurun_out/defer_gemm.log; exit 1; }
cat gpurun_out/defer_gemm.log
timeout -k 10 200 tools/cpp/gemm_bench epi > gpurun_out/defer_epi.log 2>&1 || { cat gpurun_out/defer_epi.log; exit 1; }
cat gpurun_out/defer_epi.log
