# round 4: XCD row-band tile walk + LDS-transposed stores; fp16 precision tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
B=tools/cpp/gemm_bench
timeout -k 10 300 $B blas,bf16,lt,xb,xblt 16384 50304 768 16384 6144 768 16384 2304 768 16384 768 3072 16384 768 768 > gpurun_out/r4_xb.log 2>&1 || { cat gpurun_out/r4_xb.log; exit 1; }
cat gpurun_out/r4_xb.log
timeout -k 10 120 tools/cpp/gemm_stamps 16384 50304 768 1036 12 > gpurun_out/r4_xb_stamps.log 2>&1 || { cat gpurun_out/r4_xb_stamps.log; exit 1; }
cat gpurun_out/r4_xb_stamps.log
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "precision or grads_vs_fp32 or fp16" > gpurun_out/r4_t4.log 2>&1 || { tail -60 gpurun_out/r4_t4.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_t4.log | tail -20
