# round 5: kernel trace of the ddp_medium step (batch 4 x GA 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab/prof_step.sh r5med --model_size medium --batch_size 4 --grad_accum 8 > gpurun_out/med_prof.txt 2>&1 || { tail -20 gpurun_out/med_prof.txt; exit 1; }
head -45 gpurun_out/med_prof.txt
