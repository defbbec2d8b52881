#!/bin/bash
# A/B of the split-K weight-gradient GEMMs on one box: kernel tests, GEMM roles, bench with/without.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "splitk or planner" -x -q --timeout 120 --timeout-method thread > gpurun_out/splitk_tests.log 2>&1 || { tail -30 gpurun_out/splitk_tests.log; exit 1; }
tail -2 gpurun_out/splitk_tests.log
timeout -k 10 300 python tools/gemm_roles.py > gpurun_out/gemm_roles_splitk.log 2>&1 || { tail -20 gpurun_out/gemm_roles_splitk.log; exit 1; }
head -10 gpurun_out/gemm_roles_splitk.log
for i in 1 2; do
  DLT_WGRAD_SPLITK=0 timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_nosplit_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_nosplit_$i.log | cut -c1-140
  DLT_GEMM_REPORT=1 timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_split_$i.log 2>&1 || exit 1
  grep '"metric"' gpurun_out/bench_split_$i.log | cut -c1-140
done
