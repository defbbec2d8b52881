# round 4: fp16 through the pipelined window + micro-step fusion: tests and bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "fp16 or precision" > gpurun_out/f16b_t.log 2>&1 || { tail -40 gpurun_out/f16b_t.log; exit 1; }
tail -1 gpurun_out/f16b_t.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --precision fp16 > gpurun_out/f16b_bench.$rep.log 2> gpurun_out/f16b_bench.$rep.err || { tail -20 gpurun_out/f16b_bench.$rep.err; exit 1; }
tail -1 gpurun_out/f16b_bench.$rep.log | cut -c1-220
done
