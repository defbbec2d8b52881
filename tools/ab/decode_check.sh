#!/bin/bash
# Decode kernels: GPU tests + decode throughput (fused step vs ATen step).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu -k "decode or generate or sample" --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/dec_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/dec_tests.log; exit $rc; }
for f in 1 0; do
  for b in 1 8; do
    DLT_DECODE_FUSED=$f timeout -k 10 180 python -u tools/bench_decode.py small $b 200 > gpurun_out/dec_${f}_$b.log 2>&1
    rc=$?; echo "fused=$f B$b rc=$rc: $(grep -v amdgpu.ids gpurun_out/dec_${f}_$b.log | tr '\n' '|')"; [ $rc -eq 0 ] || exit $rc
  done
done
