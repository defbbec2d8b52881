#!/bin/bash
# Deferred-store variants (stores per interval x VGPR slots): GEMM shapes + fused epilogues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in g1r3 g3r3 g3r0 g1r0; do
  echo "== $v"
  timeout -k 10 200 tools/cpp/gemm_bench_$v blas,bf16,imm 16384 2304 768 16384 6144 768 16384 3072 768 16384 50304 768 > gpurun_out/d2_$v.log 2>&1 || { cat gpurun_out/d2_$v.log; exit 1; }
  cat gpurun_out/d2_$v.log
  timeout -k 10 200 tools/cpp/gemm_bench_$v epi > gpurun_out/d2e_$v.log 2>&1 || { cat gpurun_out/d2e_$v.log; exit 1; }
  cat gpurun_out/d2e_$v.log
done
