#!/bin/bash
# --memory_first --defer_roles o with the o weight gradient deferred for the first N layers
# only (DLT_DEFER_LAYERS=N): tok/s and peak GB against memory_first and all 12 layers.
set -u
for rep in $(seq 1 ${REPS:-2}); do
  REPS=1 bash tools/ab/r6/mem_ab.sh "mf:--memory_first;fo:--memory_first --defer_roles o" || exit 1
  for n in 4 6 8; do
    DLT_DEFER_LAYERS=$n REPS=1 bash tools/ab/r6/mem_ab.sh "fo$n:--memory_first --defer_roles o" || exit 1
  done
done
