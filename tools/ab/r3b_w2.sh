#!/bin/bash
# 128-row-tile / two-workgroups-per-CU projection GEMM (flags 1024) vs the 256-row kernel and hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 tools/cpp/gemm_bench blas,bf16,w2,nostore,w2nost 16384 2304 768 16384 768 768 16384 6144 768 16384 768 3072 \
  16384 3072 768 16384 50304 768 > gpurun_out/w2_gemm.log 2>&1 || { cat gpurun_out/w2_gemm.log; exit 1; }
cat gpurun_out/w2_gemm.log
timeout -k 10 200 tools/cpp/gemm_bench epi > gpurun_out/w2_epi.log 2>&1 || { cat gpurun_out/w2_epi.log; exit 1; }
cat gpurun_out/w2_epi.log
