# round 5: keep-bit kernel rewrite (carry-chain bit packing, branch-free transpose):
# bitwise mask tests, isolated attention timing and a same-box step A/B vs HEAD's kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/kb_tests.log 2>&1 || { tail -30 gpurun_out/kb_tests.log; exit 1; }
tail -2 gpurun_out/kb_tests.log
for r in 1 2; do
  for v in new base; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    echo "== $v#$r isolated"
    DLT_KERNEL_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py --packed --B 16 --iters 50 || exit 1
  done
done
bash tools/ab/kernels_ab.sh 3 || exit 1
