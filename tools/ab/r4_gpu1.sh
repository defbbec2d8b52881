# round 4, first GPU pass: GEMM epilogue diagnostics, dgrad kernels (bench + tests), bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/ab/r4_gemm_diag.sh > gpurun_out/r4_diag_all.log 2>&1 || { tail -30 gpurun_out/r4_diag_all.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or planner" > gpurun_out/r4_t1.log 2>&1 || { tail -40 gpurun_out/r4_t1.log; exit 1; }
tail -3 gpurun_out/r4_t1.log
DLT_GEMM_REPORT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r4_b1.log 2> gpurun_out/r4_b1.err || { tail -30 gpurun_out/r4_b1.err; exit 1; }
cat gpurun_out/r4_b1.log
