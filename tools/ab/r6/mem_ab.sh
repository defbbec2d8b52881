#!/bin/bash
# Interleaved bench.py runs of memory configurations (same box): tok/s and peak GB.
# usage: REPS=2 bash tools/ab/r6/mem_ab.sh "name:args;name2:args" (args space-separated)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
IFS=';' read -ra V <<< "$1"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "${V[@]}"; do
    name=${spec%%:*}; a=${spec#*:}
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 $a > gpurun_out/m_$name.$rep.log 2>&1 || { tail -5 gpurun_out/m_$name.$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" gpurun_out/m_$name.$rep.log $name
  done
done
