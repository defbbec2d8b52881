#!/bin/bash
# rocprofv3 kernel trace of bench.py + the last-step breakdown (tools/step_profile.py).
# usage: [env knobs] bash tools/ab/prof_step.sh NAME [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD
name=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$name" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 2 "$@" > "$R/gpurun_out/prof_$name.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_$name.log"; exit 1; }
cd "$R"
grep '"metric"' gpurun_out/prof_$name.log
f=$(find gpurun_out/prof_$name -name '*kernel_trace.csv' | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_$name.md && cat gpurun_out/step_$name.md
