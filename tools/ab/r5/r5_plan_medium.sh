# round 5: are the shipped plan's medium pins (exhaustive) better than per-process races?
# ddp_medium / fsdp_medium with the shipped plan vs DLT_GEMM_PLAN=none, two interleaved reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2; do
  for plan in shipped none; do
    if [ $plan = none ]; then export DLT_GEMM_PLAN=none; else unset DLT_GEMM_PLAN; fi
    for mode in ddp fsdp; do
      timeout -k 10 300 python bench.py --mode $mode --model_size medium --batch_size 4 --grad_accum 8 --steps 6 --warmup 3 \
        > gpurun_out/pm_${mode}_$plan.log 2>&1 || { tail -20 gpurun_out/pm_${mode}_$plan.log; exit 1; }
      echo "$r $mode $plan: $(grep '"metric"' gpurun_out/pm_${mode}_$plan.log | cut -c1-120)"
    done
  done
done
