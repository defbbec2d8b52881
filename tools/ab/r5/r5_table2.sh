# round 5 (late): fp32 kernel tests, then the bench.py table over every configuration on the
# final tree (fp32 row on the GEMM-formulated attention)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/t2_tests.log 2>&1 || { tail -40 gpurun_out/t2_tests.log; exit 1; }
tail -1 gpurun_out/t2_tests.log
timeout -k 10 1000 python -u tools/bench_table.py --gpus 1 --steps 10 \
  --configs ddp_small,ddp_small_lean,ddp_small_fp16,ddp_small_fp32,ddp_small_hd128,ddp_small_hd96,fsdp_small,ddp_medium,fsdp_medium,fsdp_xl \
  --out gpurun_out/r5_bench_table2.md > gpurun_out/r5_table2.log 2>&1 || { tail -30 gpurun_out/r5_table2.log; exit 1; }
cat gpurun_out/r5_bench_table2.md
