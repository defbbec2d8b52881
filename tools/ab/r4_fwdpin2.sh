# round 4: ffbb GEMM grid cap (DLT_FFBB_GEMM_GRID) with the shipped plan and with o + down forward pinned hand
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/fq_$n.log 2> gpurun_out/fq_$n.err || { tail -20 gpurun_out/fq_$n.err; exit 1; }; }
for rep in 1 2; do
  run def.$rep DLT_X=0 && run g256.$rep DLT_FFBB_GEMM_GRID=0 && run g160.$rep DLT_FFBB_GEMM_GRID=160 &&
  run od256.$rep DLT_FFBB_GEMM_GRID=0 DLT_GEMM_PLAN=tools/ab/plan_fwd_od.json || exit 1
done
for f in gpurun_out/fq_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
