# round 4: SwiGLU output in the dY slot ring (DLT_S_RING): correctness + memory / throughput A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "ffbb or test_swiglu or precision or dswiglu" > gpurun_out/r4_sring_t.log 2>&1 || { tail -60 gpurun_out/r4_sring_t.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_sring_t.log | grep -v PASSED | tail; tail -2 gpurun_out/r4_sring_t.log
REPS=2 STEPS=20 VARIANTS="sring:DLT_S_RING=1 nosring:DLT_S_RING=0 ring2:DLT_SLOT_RING=2" bash tools/ab/r3b_env_ab.sh
