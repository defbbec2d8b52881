#!/bin/bash
# Selective vs whole-block activation recompute (DLT_AC_SELECTIVE), FSDP + AC configs.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ac_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/ac_tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for sel in 0 1; do
    for cfg in "medium 4 8" "small 8 4"; do
      set -- $cfg
      DLT_AC_SELECTIVE=$sel timeout -k 10 300 python -u bench.py --mode fsdp --model_size $1 --batch_size $2 --grad_accum $3 --steps 6 --warmup 2 > gpurun_out/ac_${1}_${sel}_$r.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "fail $1 $sel"; tail -5 gpurun_out/ac_${1}_${sel}_$r.log; exit $rc; }
      echo "fsdp $1 sel=$sel #$r: $(tail -1 gpurun_out/ac_${1}_${sel}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("peak_gb_per_gpu"))')"
    done
  done
done
