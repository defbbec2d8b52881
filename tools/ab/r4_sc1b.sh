# round 4: LDS-transposed + write-through stores on the RoPE / SwiGLU epilogues
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
B=tools/cpp/gemm_bench
for f in 0 1036 3084; do
  EPI_FLAGS=$f timeout -k 10 200 $B epi > gpurun_out/r4_epi_$f.log 2>&1 || { cat gpurun_out/r4_epi_$f.log; exit 1; }
  echo "== EPI_FLAGS=$f"; cat gpurun_out/r4_epi_$f.log
done
DLT_GEMM_FLAGS=3084 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "gemm or rope or swiglu or planner" > gpurun_out/r4_sc1_t.log 2>&1 || { tail -60 gpurun_out/r4_sc1_t.log; exit 1; }
tail -2 gpurun_out/r4_sc1_t.log
