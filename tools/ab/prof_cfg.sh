#!/bin/bash
# rocprofv3 kernel trace of bench.py for one (micro-batch, grad-accum) config, summarised
# by tools/step_profile.py into gpurun_out/step_profile_B<b>_GA<g>.md
#   usage: bash tools/ab/prof_cfg.sh B GA [extra bench args]
set -u
B=$1; GA=$2; shift 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
d=gpurun_out/prof_B${B}_GA${GA}
rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --batch_size $B --grad_accum $GA "$@" > $d.log 2>&1
rc=$?; echo "rocprof B$B GA$GA rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
f=$(find $d -name "*kernel_trace.csv" | head -1)
python tools/step_profile.py "$f" > gpurun_out/step_profile_B${B}_GA${GA}.md 2>&1
head -45 gpurun_out/step_profile_B${B}_GA${GA}.md
