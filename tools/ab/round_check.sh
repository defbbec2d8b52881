#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke(), bench.py (default contract), kernel-trace profile.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc: $(tail -1 gpurun_out/bench_default.log | cut -c1-400)"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_profile.md 2>&1; echo "step_profile rc=$?"; head -24 gpurun_out/step_profile.md
