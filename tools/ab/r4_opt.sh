# round 4: overlapped optimizer (bitwise test + in-step A/B) and forward-role plan pins
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -k "overlapped_optimizer or bitwise_reproducible" \
  --timeout 240 --timeout-method thread > gpurun_out/r4_opt_t.log 2>&1 || { tail -40 gpurun_out/r4_opt_t.log; exit 1; }
tail -2 gpurun_out/r4_opt_t.log
run() { n=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/o_$n.log 2> gpurun_out/o_$n.err || { tail -20 gpurun_out/o_$n.err; exit 1; }; }
for rep in 1 2; do
  run ov.$rep && run noov.$rep --no_overlap_optimizer &&
  DLT_GEMM_PLAN=tools/ab/plan_fwd_od.json run od.$rep && DLT_GEMM_PLAN=tools/ab/plan_fwd_all.json run all.$rep || exit 1
done
for f in gpurun_out/o_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
