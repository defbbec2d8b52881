# round 4: serial-ffbb first step + dY ring: tests and bench memory / speed A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "ffbb or reproducible or resume_is_exact" > gpurun_out/r4_t6.log 2>&1 || { tail -60 gpurun_out/r4_t6.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_t6.log | grep -v PASSED; tail -2 gpurun_out/r4_t6.log
REPS=2 STEPS=20 VARIANTS="ring3:DLT_SLOT_RING=3 ring0:DLT_SLOT_RING=0" bash tools/ab/r3b_env_ab.sh
