#!/bin/bash
# End-of-round check: smoke(), the whole GPU suite, the headline bench (3 runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/end_smoke.log 2>&1 \
  || { tail -20 gpurun_out/end_smoke.log; exit 1; }
tail -1 gpurun_out/end_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail 5 -q -rf --timeout 240 --timeout-method thread \
  > gpurun_out/end_gpu_suite.log 2>&1 || { tail -30 gpurun_out/end_gpu_suite.log; exit 1; }
tail -2 gpurun_out/end_gpu_suite.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/end_bench.$rep.log 2> gpurun_out/end_bench.$rep.err \
    || { tail -20 gpurun_out/end_bench.$rep.err; exit 1; }
  tail -1 gpurun_out/end_bench.$rep.log
done
