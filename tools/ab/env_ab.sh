#!/bin/bash
# Interleaved bench.py A/B of environment-knob variants: VARIANTS="name:K=V,K=V name2:..." (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $VARIANTS; do
    name=${spec%%:*}; kv=${spec#*:}
    env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 $BENCH_ARGS \
      > gpurun_out/env_$name.$rep.log 2> gpurun_out/env_$name.$rep.err || { tail -20 gpurun_out/env_$name.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" gpurun_out/env_$name.$rep.log $name
  done
done
