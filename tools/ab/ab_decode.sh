#!/bin/bash
# Same-box A/B of the decode kernels: ops/_dlt_kernels_base.so (tools/ab/build_base_lib.sh)
# against the current ops/_dlt_kernels.so, tools/bench_decode.py, alternating.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu -k "decode or generate or sample or recompute" --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/dec_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/dec_tests.log; exit $rc; }
for r in 1 2; do
  for v in base new; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    for b in 1 8; do
      DLT_KERNEL_LIB=$lib timeout -k 10 180 python -u tools/bench_decode.py small $b 200 > gpurun_out/abd_${v}_${b}_$r.log 2>&1
      rc=$?; echo "$v B$b #$r rc=$rc: $(grep -v amdgpu.ids gpurun_out/abd_${v}_${b}_$r.log | tr '\n' '|')"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
