# round 5: fp32 attention through hipBLASLt fp32 GEMMs (DLT_F32_ATTN=gemm) vs the flash VALU
# kernels: fp32 kernel tests, the fp32 bench both ways, a kernel trace of the gemm step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/f32g_tests.log 2>&1 || { tail -40 gpurun_out/f32g_tests.log; exit 1; }
tail -3 gpurun_out/f32g_tests.log
for impl in flash gemm; do
  DLT_F32_ATTN=$impl timeout -k 10 300 python bench.py --precision fp32 --steps 4 --warmup 2 > gpurun_out/f32g_$impl.log 2>&1 \
    || { tail -20 gpurun_out/f32g_$impl.log; exit 1; }
  echo "$impl: $(grep '"metric"' gpurun_out/f32g_$impl.log | cut -c1-200)"
done
DLT_F32_ATTN=gemm bash tools/ab/prof_step.sh r5f32g --precision fp32 > gpurun_out/f32g_prof.txt 2>&1 || { tail -20 gpurun_out/f32g_prof.txt; exit 1; }
head -40 gpurun_out/f32g_prof.txt
