# round 4, end: fp16 data gradients on the hand-written kernel (HK = 1) -- tests, fp16
# bench with the hand dgrads vs the library (DLT_GEMM_DGRAD=0), bf16 bench alongside
# (the bf16 kernels' ISA is unchanged by the HK template: diffed instruction streams)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
[ -n "$NOTESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "dgrad or wgrad or planner or fp16 or precision or f16 or swiglu" > gpurun_out/f16dg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f16dg_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/f16dg_tests.log | head; exit $rc; }
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 $ARGS > gpurun_out/fd_$n.log 2> gpurun_out/fd_$n.err || { tail -20 gpurun_out/fd_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*\|"final_loss": [0-9.]*' gpurun_out/fd_$n.log | tr '\n' ' ')"; }
for rep in 1 2 3; do
  ARGS="--precision fp16" run f16hand.$rep DLT_X=0 && ARGS="--precision fp16" run f16lib.$rep DLT_GEMM_DGRAD=0 || exit 1
  ARGS="" run bf16.$rep DLT_X=0 || exit 1
done
