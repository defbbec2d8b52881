#!/bin/bash
# Kernel traces of bench.py under GEMM plan variants (same box): for each "name:edit,edit"
# in VARIANTS, write the variant plan (tools/ab/plan_variant.py) and run prof_step.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  name=${v%%:*}; edits=${v#*:}
  python tools/ab/plan_variant.py /tmp/plan_$name.json ${edits//,/ } || exit 1
  DLT_GEMM_PLAN=/tmp/plan_$name.json bash tools/ab/prof_step.sh "$name" || exit 1
done
