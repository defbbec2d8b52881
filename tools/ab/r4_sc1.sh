# round 4: write-through (sc1) C stores vs L2-retained stores; race regression tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
B=tools/cpp/gemm_bench
timeout -k 10 300 $B lt,sc1,xblt,xbsc1,blas 16384 50304 768 16384 6144 768 16384 2304 768 16384 768 3072 16384 768 768 > gpurun_out/r4_sc1.log 2>&1 || { cat gpurun_out/r4_sc1.log; exit 1; }
cat gpurun_out/r4_sc1.log
timeout -k 10 120 tools/cpp/gemm_stamps 16384 6144 768 1 1036 3084 > gpurun_out/r4_sc1_stamps.log 2>&1 || { cat gpurun_out/r4_sc1_stamps.log; exit 1; }
timeout -k 10 120 tools/cpp/gemm_stamps 16384 50304 768 1 1036 3084 >> gpurun_out/r4_sc1_stamps.log 2>&1 || { cat gpurun_out/r4_sc1_stamps.log; exit 1; }
cat gpurun_out/r4_sc1_stamps.log
timeout -k 10 900 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "ffbb_hand or forced_collectives_with_hand" > gpurun_out/r4_race.log 2>&1 || { tail -60 gpurun_out/r4_race.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_race.log | tail -20; tail -2 gpurun_out/r4_race.log
REPS=2 STEPS=20 VARIANTS="new:DLT_GEMM_FLAGS=1036 sc1:DLT_GEMM_FLAGS=3084" bash tools/ab/r3b_env_ab.sh
