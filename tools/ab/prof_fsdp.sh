#!/bin/bash
# Kernel-trace step breakdown of the FSDP path (small, B8 x GA4, AC on) on one GPU.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_fsdp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fsdp -o run --output-format csv -- python3 bench.py --mode fsdp --steps 3 --warmup 2 > gpurun_out/prof_fsdp.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_fsdp.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_fsdp -name "*kernel_trace.csv" | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_profile_fsdp.md 2>&1; echo "step_profile rc=$?"; head -50 gpurun_out/step_profile_fsdp.md
