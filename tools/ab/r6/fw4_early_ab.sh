#!/bin/bash
# fw4 two-tile lm_head: next tile's stages before (flags 8192) vs after the epilogue:
# kernel tests, isolated lm_head, then the step with the lm_head pin 4100 vs 12292.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_fw4" --timeout 120 --timeout-method thread > gpurun_out/fw4e_tests.log 2>&1
rc=$?; echo "fw4 tests rc=$rc: $(tail -1 gpurun_out/fw4e_tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_gemm_fwd.py --shapes lm_head --impls fw4x2,fw4x2e,fw4s5x2,fw4s5x2e,lib --iters 30 > gpurun_out/fw4e_iso.log 2>&1 || { tail -5 gpurun_out/fw4e_iso.log; exit 1; }
grep lm_head gpurun_out/fw4e_iso.log
timeout -k 10 200 python -u tools/bench_gemm_fwd.py --shapes lm_head --impls fw4x2,fw4x2e,fw4s5x2,fw4s5x2e --iters 30 > gpurun_out/fw4e_iso2.log 2>&1 && grep lm_head gpurun_out/fw4e_iso2.log
python tools/ab/plan_variant.py gpurun_out/plan_e.json tn:16384x50304x768=fw4:12292 || exit 1
for r in 1 2 3; do
  for v in base e; do
    if [ $v = base ]; then unset DLT_GEMM_PLAN; else export DLT_GEMM_PLAN=gpurun_out/plan_e.json; fi
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/fw4e_$v$r.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/fw4e_$v$r.log; exit 1; }
    echo "$v#$r: $(tail -1 gpurun_out/fw4e_$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
