# round 4: the new --memory_lean (nothing deferred): GPU tests touching it + bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "lean or forced" > gpurun_out/ln2_t.log 2>&1 || { tail -40 gpurun_out/ln2_t.log; exit 1; }
tail -1 gpurun_out/ln2_t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --memory_lean > gpurun_out/ln2.log 2> gpurun_out/ln2.err || { tail -20 gpurun_out/ln2.err; exit 1; }
tail -1 gpurun_out/ln2.log | cut -c1-200; grep -o '"peak_gb_per_gpu": [0-9.]*' gpurun_out/ln2.log
