#!/bin/bash
# Round-3 GPU check: whole GPU suite, headline bench (+ plan save), memory-lean bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${SUITE:-tests} -m gpu --maxfail 5 -q -rf --timeout 240 --timeout-method thread \
  > gpurun_out/r3_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r3_gpu_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r3_gpu_suite.log | head -20; exit $rc; }
DLT_GEMM_PLAN_OUT=gpurun_out/plan_r3.json DLT_GEMM_REPORT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 \
  > gpurun_out/r3_bench.log 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --memory_lean > gpurun_out/r3_bench_lean.log \
  2> gpurun_out/r3_bench_lean.err || { tail -20 gpurun_out/r3_bench_lean.err; exit 1; }
cat gpurun_out/r3_bench_lean.log
