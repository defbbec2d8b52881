# round 4: weight-gradient split depths in the step (plan variants): qkv x7, + o x16, qkv stream-K
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/ws_$n.log 2> gpurun_out/ws_$n.err || { tail -20 gpurun_out/ws_$n.err; exit 1; }; }
for rep in 1 2; do
  run def.$rep DLT_X=0 && run q7.$rep DLT_GEMM_PLAN=tools/ab/plan_wq7.json && run q7o16.$rep DLT_GEMM_PLAN=tools/ab/plan_wq7o16.json &&
  run qsk.$rep DLT_GEMM_PLAN=tools/ab/plan_wqsk.json || exit 1
done
for f in gpurun_out/ws_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
