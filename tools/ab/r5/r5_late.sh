# round 5: epilogue-first staging (flags 4096) of the RoPE / SwiGLU-backward GEMM epilogues --
# numerics (both schedules), isolated timings, then the step with / without it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "qkv_rope or down_swiglu or gemm_dgrad or planner" > gpurun_out/lt_tests.log 2>&1 || { tail -40 gpurun_out/lt_tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/lt_tests.log
timeout -k 10 120 tools/cpp/gemm_bench dgrad 16384 3072 768 > gpurun_out/lt_dgrad.log 2>&1 || { cat gpurun_out/lt_dgrad.log; exit 1; }
cat gpurun_out/lt_dgrad.log
for f in 3084 7180; do EPI_FLAGS=$f timeout -k 10 120 tools/cpp/gemm_bench epi > gpurun_out/lt_epi_$f.log 2>&1 || { cat gpurun_out/lt_epi_$f.log; exit 1; }; echo "EPI_FLAGS=$f"; cat gpurun_out/lt_epi_$f.log; done
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/lt_$n.log 2> gpurun_out/lt_$n.err || { tail -20 gpurun_out/lt_$n.err; exit 1; }; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" gpurun_out/lt_$n.log $n; }
for rep in 1 2 3; do
  run base.$rep DLT_X=0 && run late.$rep DLT_GEMM_FLAGS=7180 && run laterope.$rep DLT_GEMM_FLAGS=7180 DLT_GEMM_PLAN=tools/ab/r5/plan_r5_rope.json || exit 1
done
