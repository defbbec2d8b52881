#!/bin/bash
# Overlapped backwards: bitwise / determinism GPU tests, then the step A/B (same box, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "pipelined or bitwise or memory_lean or deferred or resume or forced or collectives or precision" > gpurun_out/ov_tests.log 2>&1 || { tail -30 gpurun_out/ov_tests.log; exit 1; }
tail -2 gpurun_out/ov_tests.log
for rep in 1 2; do
  for ov in 1 0; do
    DLT_BWD_OVERLAP=$ov timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ov_$ov.$rep.log 2> gpurun_out/ov_$ov.$rep.err || { tail -20 gpurun_out/ov_$ov.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('overlap', sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" gpurun_out/ov_$ov.$rep.log $ov
  done
done
DLT_BWD_OVERLAP=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --memory_lean > gpurun_out/ov_lean.log 2>&1 && grep -o '"value": [0-9.]*\|"peak_gb_per_gpu": [0-9.]*' gpurun_out/ov_lean.log
