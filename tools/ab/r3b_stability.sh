#!/bin/bash
# Long run of the headline config with the new window schedule: throughput and memory stay flat.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for n in 50 200; do
  timeout -k 10 400 python -u bench.py --steps $n --warmup 3 > gpurun_out/stab_$n.log 2> gpurun_out/stab_$n.err || { tail -20 gpurun_out/stab_$n.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'steps', d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" gpurun_out/stab_$n.log $n
done
