# round 5: kernel trace of the fsdp_xl step (batch 4 x GA 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/ab/prof_step.sh r5xl --mode fsdp --model_size xl --batch_size 4 --grad_accum 8 > gpurun_out/xl_prof.txt 2>&1 || { tail -20 gpurun_out/xl_prof.txt; exit 1; }
head -50 gpurun_out/xl_prof.txt
