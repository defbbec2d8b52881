# round 5: exhaustive hipBLASLt tuning of the fp32 step's GEMM keys, merged into the shipped
# plan (its bf16 pins replayed, not re-tuned), then fp32 bench A/B: shipped vs merged plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
DLT_GEMM_TUNE=exhaustive DLT_GEMM_VERBOSE=1 DLT_GEMM_PLAN_OUT=gpurun_out/plan_f32.json \
  timeout -k 10 700 python -u bench.py --precision fp32 --steps 2 --warmup 1 > gpurun_out/tune_f32.log 2>&1 \
  || { tail -30 gpurun_out/tune_f32.log; exit 1; }
grep '"metric"' gpurun_out/tune_f32.log | cut -c1-160
ls -la gpurun_out/plan_f32.json
for r in 1 2; do
  for plan in shipped merged; do
    if [ $plan = merged ]; then export DLT_GEMM_PLAN=gpurun_out/plan_f32.json; else unset DLT_GEMM_PLAN; fi
    timeout -k 10 300 python bench.py --precision fp32 --steps 6 --warmup 2 > gpurun_out/tf32_$plan.log 2>&1 \
      || { tail -20 gpurun_out/tf32_$plan.log; exit 1; }
    echo "$r $plan: $(grep '"metric"' gpurun_out/tf32_$plan.log | cut -c1-150)"
  done
done
