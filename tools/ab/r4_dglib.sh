# round 4: data-gradient GEMMs pinned hand-written vs hipBLASLt, in the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/g_$n.log 2> gpurun_out/g_$n.err || { tail -20 gpurun_out/g_$n.err; exit 1; }; }
for rep in 1 2; do
  run hand.$rep DLT_GEMM_PLAN=tools/ab/plan_dghand.json && run lib.$rep DLT_GEMM_PLAN=tools/ab/plan_dglib.json || exit 1
done
for f in gpurun_out/g_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
