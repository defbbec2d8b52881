# round 4: step profile of the current tree (kernel trace + concurrency) with the GEMM race report
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
DLT_GEMM_REPORT=1 bash tools/ab/prof_step.sh r4 > gpurun_out/step_r4_full.md 2>&1 || { tail -20 gpurun_out/step_r4_full.md; exit 1; }
f=$(find gpurun_out/prof_r4 -name '*kernel_trace.csv' | head -1)
python tools/concurrency.py "$f" 40 > gpurun_out/conc_r4.md 2>&1
head -60 gpurun_out/step_r4_full.md; cat gpurun_out/conc_r4.md | head -50
grep -A40 'hand-written\|"dgrad' gpurun_out/prof_r4.log | head -60
