# round 5 batch 15: dK/dV with the dropout scale folded into the epilogues (mask applied
# once) vs HEAD's attention (_dlt_kernels_base.so): attention tests, isolated, in the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "attention or head_dim or engine_hip_vs_reference or gpt2_small" > gpurun_out/e15_tests.log 2>&1 || { tail -30 gpurun_out/e15_tests.log; exit 1; }
tail -1 gpurun_out/e15_tests.log
for r in 1 2; do
  for v in base new; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    DLT_KERNEL_LIB=$lib timeout -k 10 200 python -u tools/bench_attn.py --packed --B 16 --iters 20 > gpurun_out/e15_attn_$v$r.log 2>&1 \
      || { tail -10 gpurun_out/e15_attn_$v$r.log; exit 1; }
    echo "== $v$r $(grep -v 'amdgpu.ids\|HW_QUEUES' gpurun_out/e15_attn_$v$r.log | tail -1)"
  done
done
bash tools/ab/kernels_ab.sh 3
