# round 5: kernel trace of the --precision fp16 step (for the bf16 vs fp16 gap)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab/prof_step.sh r5f16 --precision fp16 > gpurun_out/f16_prof.txt 2>&1 || { tail -20 gpurun_out/f16_prof.txt; exit 1; }
head -60 gpurun_out/f16_prof.txt
