# round 4: staged SwiGLU s stores; per-phase cycles of the RoPE / SwiGLU epilogues
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
B=tools/cpp/gemm_bench
S=tools/cpp/gemm_stamps
EPI_FLAGS=3084 timeout -k 10 200 $B epi > gpurun_out/r4_epi2.log 2>&1 || { cat gpurun_out/r4_epi2.log; exit 1; }
cat gpurun_out/r4_epi2.log
timeout -k 10 100 $S 16384 2304 768 3084 > gpurun_out/r4_epi2_st.log 2>&1 &&
EPI=rope timeout -k 10 100 $S 16384 2304 768 3084 >> gpurun_out/r4_epi2_st.log 2>&1 &&
timeout -k 10 100 $S 16384 6144 768 3084 >> gpurun_out/r4_epi2_st.log 2>&1 &&
EPI=swiglu timeout -k 10 100 $S 16384 6144 768 3084 >> gpurun_out/r4_epi2_st.log 2>&1 || { cat gpurun_out/r4_epi2_st.log; exit 1; }
cat gpurun_out/r4_epi2_st.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "gemm or rope or swiglu or planner" > gpurun_out/r4_epi2_t.log 2>&1 || { tail -60 gpurun_out/r4_epi2_t.log; exit 1; }
tail -2 gpurun_out/r4_epi2_t.log
