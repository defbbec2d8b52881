#!/bin/bash
# Kernel trace of the bench with the sequential schedule (no micro-step pipelining), so the
# per-kernel times are the kernels' own; summarised into gpurun_out/step_profile_seq.md.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export DLT_PIPELINE=0
rm -rf gpurun_out/prof_seq
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_seq.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_seq.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_seq -name "*kernel_trace.csv" | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_profile_seq.md 2>&1; echo "step_profile rc=$?"; head -45 gpurun_out/step_profile_seq.md
