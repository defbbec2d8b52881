# round 5 batch 19: backward lag of half a block (DLT_BWD_LAG=half) vs a whole block
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
DLT_BWD_LAG=half timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "window or pipelined" > gpurun_out/e19_tests.log 2>&1 || { tail -30 gpurun_out/e19_tests.log; exit 1; }
tail -1 gpurun_out/e19_tests.log
VARIANTS="block:DLT_X=0 half:DLT_BWD_LAG=half" REPS=3 bash tools/ab/env_ab.sh
