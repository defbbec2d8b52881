# round 5: upper bound of a cheaper dropout select -- attention kernels with the select
# removed (DLT_ATTN_NOSEL, _dlt_kernels_base.so) vs the shipped kernels, isolated and in the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2; do
  for v in new base; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    echo "== $v#$r isolated"
    DLT_KERNEL_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py --packed --B 16 --iters 50 || exit 1
  done
done
bash tools/ab/kernels_ab.sh 2 || exit 1
