# round 4: kernel-trace step profile of bench.py with extra bench args (NAME ARGS...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
n=$1; shift
bash tools/ab/prof_step.sh $n "$@" > gpurun_out/step_${n}_full.md 2>&1 || { tail -20 gpurun_out/step_${n}_full.md; exit 1; }
f=$(find gpurun_out/prof_$n -name '*kernel_trace.csv' | head -1)
python tools/concurrency.py "$f" 30 > gpurun_out/conc_$n.md 2>&1
head -30 gpurun_out/step_${n}_full.md; head -12 gpurun_out/conc_$n.md
