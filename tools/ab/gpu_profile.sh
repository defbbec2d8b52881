#!/bin/bash
# GPU tests + bench + rocprofv3 kernel trace of the bench, summarised into gpurun_out/.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc: $(tail -1 gpurun_out/bench.log | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_profile.md 2>&1; echo "step_profile rc=$?"; head -30 gpurun_out/step_profile.md
