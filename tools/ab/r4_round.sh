#!/bin/bash
# Round-4 GPU check: whole GPU suite, headline bench (+ GEMM report / plan save), memory-lean bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
T=${TAG:-r4}
if [ -z "$NOSUITE" ]; then
timeout -k 10 1000 python -u -m pytest ${SUITE:-tests} -m gpu --maxfail 5 -q -rf --timeout 240 --timeout-method thread \
  > gpurun_out/${T}_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_gpu_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${T}_gpu_suite.log | head -20; exit $rc; }
fi
DLT_GEMM_PLAN_OUT=gpurun_out/plan_${T}.json DLT_GEMM_REPORT=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
  > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --memory_lean > gpurun_out/${T}_bench_lean.log \
  2> gpurun_out/${T}_bench_lean.err || { tail -20 gpurun_out/${T}_bench_lean.err; exit 1; }
cat gpurun_out/${T}_bench_lean.log
if [ -n "$PROF" ]; then
  DLT_GEMM_REPORT=1 bash tools/ab/prof_step.sh ${T} > gpurun_out/step_${T}_full.md 2>&1 || { tail -20 gpurun_out/step_${T}_full.md; exit 1; }
  f=$(find gpurun_out/prof_${T} -name '*kernel_trace.csv' | head -1)
  python tools/concurrency.py "$f" 40 > gpurun_out/conc_${T}.md 2>&1
  head -60 gpurun_out/step_${T}_full.md
fi
