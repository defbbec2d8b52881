# round 4: where the persistent forward GEMM's epilogue time goes (stamps + desync ablation)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S=tools/cpp/gemm_stamps
B=tools/cpp/gemm_bench
timeout -k 10 120 $S 16384 6144 768 0 1 32 16 $((512 | (13 << 24))) > gpurun_out/r4_stamps.log 2>&1 || { cat gpurun_out/r4_stamps.log; exit 1; }
timeout -k 10 120 $S 16384 2304 768 0 1 >> gpurun_out/r4_stamps.log 2>&1 || { cat gpurun_out/r4_stamps.log; exit 1; }
timeout -k 10 120 $S 16384 768 3072 0 1 >> gpurun_out/r4_stamps.log 2>&1 || { cat gpurun_out/r4_stamps.log; exit 1; }
timeout -k 10 200 $S 16384 50304 768 0 1 >> gpurun_out/r4_stamps.log 2>&1 || { cat gpurun_out/r4_stamps.log; exit 1; }
cat gpurun_out/r4_stamps.log
timeout -k 10 300 $B blas,bf16,nostore,d4,d8,d13,d20 16384 6144 768 16384 2304 768 16384 768 3072 16384 768 768 16384 50304 768 > gpurun_out/r4_desync.log 2>&1 || { cat gpurun_out/r4_desync.log; exit 1; }
cat gpurun_out/r4_desync.log
timeout -k 10 300 $B dgrad > gpurun_out/r4_dgrad.log 2>&1 || { cat gpurun_out/r4_dgrad.log; exit 1; }
cat gpurun_out/r4_dgrad.log
