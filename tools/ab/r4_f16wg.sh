# round 4, end: fp16 weight gradients on the hand-written kernels (HK = 1) -- tests, then
# bench.py --precision fp16 with the hand kernels vs the library (DLT_WGRAD_HAND=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "wgrad or planner or fp16 or precision or f16" > gpurun_out/f16wg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f16wg_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/f16wg_tests.log | head; exit $rc; }
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 --precision fp16 > gpurun_out/fw_$n.log 2> gpurun_out/fw_$n.err || { tail -20 gpurun_out/fw_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/fw_$n.log)"; }
for rep in 1 2 3; do
  run hand.$rep DLT_X=0 && run lib.$rep DLT_WGRAD_HAND=0 || exit 1
done
