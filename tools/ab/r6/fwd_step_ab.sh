#!/bin/bash
# In-step A/B of forward-GEMM plans (same box, interleaved): the shipped plan vs the four
# plain forward roles (o, gate/up, down, lm_head) on k_gemm_fw4 (and variants).
# usage: REPS=2 FW4_FLAGS=129 bash tools/ab/r6/fwd_step_ab.sh "name:plan-edits;name2:..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
IFS=';' read -ra V <<< "$1"; shift
for spec in "${V[@]}"; do
  name=${spec%%:*}; edits=${spec#*:}
  python tools/ab/plan_variant.py gpurun_out/plan_$name.json $edits || exit 1
done
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "${V[@]}"; do
    name=${spec%%:*}
    DLT_GEMM_PLAN=gpurun_out/plan_$name.json DLT_GEMM_FW4_FLAGS=${FW4_FLAGS:-129} timeout -k 10 300 \
      python bench.py --steps ${STEPS:-20} --warmup 3 "$@" > gpurun_out/fs_$name.$rep.log 2>&1 || { tail -5 gpurun_out/fs_$name.$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" gpurun_out/fs_$name.$rep.log $name
  done
done
