# round 5 batch 9: four-wave forward GEMM (k_gemm_tn4): numerics, isolated timing, in-step
# plans (all five forward roles / four without lm_head / o + down) vs the shipped plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_tn4" \
  > gpurun_out/e9_tests.log 2>&1 || { tail -40 gpurun_out/e9_tests.log; exit 1; }
tail -2 gpurun_out/e9_tests.log
timeout -k 10 300 python -u tools/bench_gemm_fwd.py > gpurun_out/e9_iso.log 2>&1 || { tail -20 gpurun_out/e9_iso.log; exit 1; }
cat gpurun_out/e9_iso.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" "$1" "$2"; }
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e9_$n.log 2> gpurun_out/e9_$n.err || { tail -20 gpurun_out/e9_$n.err; exit 1; }; show gpurun_out/e9_$n.log $n; }
for rep in 1 2; do
  run lib.$rep DLT_X=0 && run all.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_tn4all.json && \
    run noh.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_tn4noh.json && run od.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_tn4od.json || exit 1
done
