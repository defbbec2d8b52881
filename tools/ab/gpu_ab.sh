#!/bin/bash
# GPU session: full -m gpu suite, then bench A/B over env toggles.  Stops at the first
# fault / abort / timeout.  Usage: VARIANTS="DLT_PIPELINE=0 DLT_PACKED_QKV=0" bash tools/ab/gpu_ab.sh
set -u
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/tests.log
  if [ $rc -ne 0 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
i=0
for v in base ${VARIANTS:-}; do
  i=$((i+1))
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS:-} \
    > gpurun_out/bench_$i.log 2>&1
  brc=$?
  echo "bench[$v] rc=$brc: $(tail -1 gpurun_out/bench_$i.log)"
  if [ $brc -ne 0 ]; then exit $brc; fi
done
