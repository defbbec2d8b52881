#!/bin/bash
# --memory_first: the o weight gradient deferred to the window (--defer_roles o) and/or the
# lm_head weight gradient on the library (no stream-K scratch), tok/s and peak GB.
set -u
mkdir -p gpurun_out
python tools/ab/plan_variant.py gpurun_out/plan_hl.json splitk:8192x50304x768=1 || exit 1
REPS=${REPS:-2} bash tools/ab/r6/mem_ab.sh "mf:--memory_first;fo:--memory_first --defer_roles o" && \
DLT_GEMM_PLAN=gpurun_out/plan_hl.json REPS=${REPS:-2} bash tools/ab/r6/mem_ab.sh "hl:--memory_first;fohl:--memory_first --defer_roles o"
