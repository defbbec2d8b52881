#!/bin/bash
# A/B of GEMM plan variants (same box, interleaved): PLANS="name:key=val,key=val ..." (splitk keys)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/plans
python - <<'PY'
import json, os
base = json.load(open("configs/gemm_plan_mi355x.json"))
for spec in os.environ["PLANS"].split():
    name, _, kv = spec.partition(":")
    p = json.loads(json.dumps(base))
    for item in filter(None, kv.split(",")):
        sec, _, rest = item.partition("/")
        k, _, v = rest.partition("=")
        p[sec][k] = json.loads(v)
    json.dump(p, open(f"gpurun_out/plans/{name}.json", "w"), indent=1)
PY
for rep in 1 2; do
  for spec in $PLANS; do
    name=${spec%%:*}
    DLT_GEMM_PLAN=gpurun_out/plans/$name.json timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 $BENCH_ARGS \
      > gpurun_out/ab_$name.$rep.log 2> gpurun_out/ab_$name.$rep.err || { tail -20 gpurun_out/ab_$name.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" gpurun_out/ab_$name.$rep.log $name
  done
done
