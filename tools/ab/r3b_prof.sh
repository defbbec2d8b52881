#!/bin/bash
# Step profile of the current tree + concurrency view (tools/concurrency.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab/prof_step.sh cur > gpurun_out/step_cur_full.md 2>&1 || { tail -20 gpurun_out/step_cur_full.md; exit 1; }
f=$(find gpurun_out/prof_cur -name '*kernel_trace.csv' | head -1)
python tools/concurrency.py "$f" 30 > gpurun_out/conc_cur.md 2>&1
head -30 gpurun_out/step_cur_full.md; cat gpurun_out/conc_cur.md
rm -rf gpurun_out/prof_cur/*/*/*.csv.bak 2>/dev/null; true
