# round 4: precision tests after the seed fix, GEMM tests with the new default flags, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "precision or grads_vs_fp32 or fp16 or gemm or planner" > gpurun_out/r4_t5.log 2>&1 || { tail -60 gpurun_out/r4_t5.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_t5.log | tail -70 | grep -v PASSED; tail -2 gpurun_out/r4_t5.log
REPS=2 STEPS=20 VARIANTS="new:DLT_SLOT_RING=3 oldflags:DLT_GEMM_FLAGS=0 noring:DLT_SLOT_RING=0" bash tools/ab/r3b_env_ab.sh
