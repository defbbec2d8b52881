#!/bin/bash
# A/B of planner knobs on one box: candidate count and workspace size.
set -u
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/knob_$name.log 2>&1 || { tail -5 gpurun_out/knob_$name.log; exit 1; }
  echo "$name: $(grep '"metric"' gpurun_out/knob_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run default DLT_X=0
run cand64 DLT_GEMM_CANDIDATES=64
run cand128 DLT_GEMM_CANDIDATES=128
run ws256 DLT_GEMM_WORKSPACE_MB=256
run default2 DLT_X=0
