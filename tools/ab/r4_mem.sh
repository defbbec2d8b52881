# round 4: memory -- SwiGLU output in the dY ring (DLT_S_RING), chunked lm_head run in the
# window's forwards (DLT_HEAD_CHUNKS); correctness, then throughput / peak A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py::test_swiglu tests/test_kernels_gpu.py::test_gemm_down_swiglu_bwd_vs_fp32 -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4_mem_t.log 2>&1 || { tail -60 gpurun_out/r4_mem_t.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_mem_t.log | grep -v PASSED | tail; tail -2 gpurun_out/r4_mem_t.log
REPS=2 STEPS=20 VARIANTS="c1share:DLT_HEAD_CHUNKS=1 c2share:DLT_HEAD_CHUNKS=2 c2noshare:DLT_HEAD_SHARE=0 sringonly:DLT_HEAD_CHUNKS=0" bash tools/ab/r3b_env_ab.sh
