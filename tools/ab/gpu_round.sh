#!/bin/bash
# One GPU session: kernel/model tests, then a short bench.  Stops at the first
# fault / abort / timeout (exit codes other than 0 = pass, 1 = test failures).
set -u
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_model_gpu.py"}
timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest $TESTS -x -q -m gpu > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} > gpurun_out/bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"
  tail -5 gpurun_out/bench.log
  exit $brc
fi
exit $rc
