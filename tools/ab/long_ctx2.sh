#!/bin/bash
# Long context beyond the keep-bit mask budget: GPU tests of the regeneration path, then
# seq 32768 (masks regenerated in the backward) next to 16384 (masks kept).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu -k "budget or recompute" --timeout 120 --timeout-method thread > gpurun_out/lc2_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/lc2_tests.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/lc2_tests.log; exit $rc; }
for cfg in "16384 1 2" "32768 1 1"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --seq_len $1 --batch_size $2 --grad_accum $3 --steps 4 --warmup 2 \
    --model_override max_seq_len=$1 > gpurun_out/lc2_$1.log 2>&1
  rc=$?; echo "seq $1 rc=$rc: $(tail -1 gpurun_out/lc2_$1.log | cut -c1-160) peak=$(tail -1 gpurun_out/lc2_$1.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read()).get("peak_gb_per_gpu"))' 2>/dev/null)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lc2_$1.log; exit $rc; }
done
