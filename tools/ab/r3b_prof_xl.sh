#!/bin/bash
# Step profiles of the FSDP xl and DDP medium configurations (tools/step_profile.py + concurrency).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for cfg in "xl:--mode fsdp --model_size xl --batch_size 4 --grad_accum 8" "med:--model_size medium --batch_size 4 --grad_accum 8"; do
  n=${cfg%%:*}; a=${cfg#*:}
  bash tools/ab/prof_step.sh $n $a > gpurun_out/step_${n}_full.md 2>&1 || { tail -20 gpurun_out/step_${n}_full.md; exit 1; }
  f=$(find gpurun_out/prof_$n -name '*kernel_trace.csv' | head -1)
  python tools/concurrency.py "$f" 25 > gpurun_out/conc_$n.md 2>&1
  head -45 gpurun_out/step_${n}_full.md; head -20 gpurun_out/conc_$n.md
done
