# round 5: dK/dV LDS reads through asm (no compiler vmcnt(0) on the next tile's DMA):
# attention tests, isolated B16 timing vs HEAD's kernels, then a step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/ba_tests.log 2>&1 || { tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
for r in 1 2; do
  for v in new base; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    echo "== $v#$r isolated"
    DLT_KERNEL_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py --packed --B 16 --iters 50 || exit 1
  done
done
[ "${1:-}" = "step" ] && { bash tools/ab/kernels_ab.sh 3 || exit 1; }
exit 0
