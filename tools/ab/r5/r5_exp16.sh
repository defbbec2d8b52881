# round 5 batch 16: ffbb forward phase offset (chain 1 starts after chain 0's first attention)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
DLT_FFBB_PHASE=1 timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "window_ffbb" > gpurun_out/e16_tests.log 2>&1 || { tail -30 gpurun_out/e16_tests.log; exit 1; }
tail -1 gpurun_out/e16_tests.log
VARIANTS="def:DLT_X=0 phase:DLT_FFBB_PHASE=1" REPS=3 bash tools/ab/env_ab.sh
