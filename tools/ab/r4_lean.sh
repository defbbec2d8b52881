# round 4: memory-lean variants -- qkv/o deferred (the --memory_lean default) vs nothing deferred
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/ln_$n.log 2> gpurun_out/ln_$n.err || { tail -20 gpurun_out/ln_$n.err; exit 1; }; }
for rep in 1 2; do
  run lean.$rep --memory_lean && run none.$rep --memory_lean --defer_roles none && run o.$rep --memory_lean --defer_roles o || exit 1
done
for f in gpurun_out/ln_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
