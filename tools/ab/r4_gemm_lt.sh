# round 4: LDS-transposed C stores (flags 1024) vs the permlane16 row-per-lane stores
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
S=tools/cpp/gemm_stamps
B=tools/cpp/gemm_bench
timeout -k 10 120 $S 16384 6144 768 0 1024 1 > gpurun_out/r4_lt_stamps.log 2>&1 || { cat gpurun_out/r4_lt_stamps.log; exit 1; }
timeout -k 10 200 $S 16384 50304 768 0 1024 >> gpurun_out/r4_lt_stamps.log 2>&1 || { cat gpurun_out/r4_lt_stamps.log; exit 1; }
cat gpurun_out/r4_lt_stamps.log
timeout -k 10 300 $B blas,bf16,lt,nostore 16384 6144 768 16384 2304 768 16384 768 3072 16384 768 768 16384 50304 768 > gpurun_out/r4_lt.log 2>&1 || { cat gpurun_out/r4_lt.log; exit 1; }
cat gpurun_out/r4_lt.log
