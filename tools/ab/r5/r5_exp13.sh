# round 5 batch 13: kernel traces of the default step and of an fp32 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab/prof_step.sh r5def > gpurun_out/e13_def.txt 2>&1 || { tail -20 gpurun_out/e13_def.txt; exit 1; }
head -60 gpurun_out/e13_def.txt
bash tools/ab/prof_step.sh r5f32 --precision fp32 > gpurun_out/e13_f32.txt 2>&1 || { tail -20 gpurun_out/e13_f32.txt; exit 1; }
head -45 gpurun_out/e13_f32.txt
