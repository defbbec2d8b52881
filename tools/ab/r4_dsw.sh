# round 4: down dgrad + SwiGLU backward fused kernel now also writes s (the ring operand): tests, isolated, in-step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "swiglu or dgrad or rope or gemm" --timeout 200 --timeout-method thread \
  > gpurun_out/d_t.log 2>&1 || { tail -40 gpurun_out/d_t.log; exit 1; }
tail -1 gpurun_out/d_t.log
timeout -k 10 200 tools/cpp/gemm_bench dgrad 16384 3072 768 > gpurun_out/d_dg.log 2>&1 || { cat gpurun_out/d_dg.log; exit 1; }
cat gpurun_out/d_dg.log
EPI_FLAGS=3084 timeout -k 10 200 tools/cpp/gemm_bench epi > gpurun_out/d_epi.log 2>&1 || { cat gpurun_out/d_epi.log; exit 1; }
cat gpurun_out/d_epi.log
DLT_GEMM_PLAN=tools/ab/plan_dsw.json timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "ffbb or window or reproducible or full_gpt2" > gpurun_out/d_m.log 2>&1 || { tail -40 gpurun_out/d_m.log; exit 1; }
tail -1 gpurun_out/d_m.log
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/d_$n.log 2> gpurun_out/d_$n.err || { tail -20 gpurun_out/d_$n.err; exit 1; }; }
for rep in 1 2; do
  run def.$rep DLT_X=0 && run dsw.$rep DLT_GEMM_PLAN=tools/ab/plan_dsw.json &&
  run dswsw.$rep DLT_GEMM_PLAN=tools/ab/plan_dsw_sw.json || exit 1
done
for f in gpurun_out/d_def*.log gpurun_out/d_dsw*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
