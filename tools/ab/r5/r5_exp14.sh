# round 5 batch 14: attention kernels of the head-dim-templated tree vs the round-4 ones
# (ops/_dlt_kernels_base.so: current sources with attention.hip of a780aa1), isolated and in the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2; do
  for v in base new; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    DLT_KERNEL_LIB=$lib timeout -k 10 200 python -u tools/bench_attn.py --packed --B 16 --iters 20 > gpurun_out/e14_attn_$v$r.log 2>&1 \
      || { tail -10 gpurun_out/e14_attn_$v$r.log; exit 1; }
    echo "== $v$r"; grep -v "amdgpu.ids\|HW_QUEUES" gpurun_out/e14_attn_$v$r.log | tail -4
  done
done
bash tools/ab/kernels_ab.sh 2
