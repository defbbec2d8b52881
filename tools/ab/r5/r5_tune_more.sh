# round 5: exhaustive tuning of the keys the shipped plan lacks for fsdp_xl and --precision
# fp16 (merged into it), then A/B of those rows: shipped plan vs merged plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 800 python -u tools/tune_gemm_plan.py --merge --configs fsdp_xl,ddp_small_fp16 \
  --out gpurun_out/plan_more.json > gpurun_out/tune_more.log 2>&1 || { tail -30 gpurun_out/tune_more.log; exit 1; }
grep -E "step|wrote" gpurun_out/tune_more.log
for r in 1 2; do
  for plan in shipped merged; do
    if [ $plan = merged ]; then export DLT_GEMM_PLAN=gpurun_out/plan_more.json; else unset DLT_GEMM_PLAN; fi
    timeout -k 10 300 python bench.py --mode fsdp --model_size xl --batch_size 4 --grad_accum 8 --steps 4 --warmup 2 \
      > gpurun_out/tm_xl_$plan.log 2>&1 || { tail -20 gpurun_out/tm_xl_$plan.log; exit 1; }
    echo "$r xl $plan: $(grep '"metric"' gpurun_out/tm_xl_$plan.log | cut -c1-120)"
    timeout -k 10 300 python bench.py --precision fp16 --steps 10 --warmup 3 > gpurun_out/tm_f16_$plan.log 2>&1 \
      || { tail -20 gpurun_out/tm_f16_$plan.log; exit 1; }
    echo "$r fp16 $plan: $(grep '"metric"' gpurun_out/tm_f16_$plan.log | cut -c1-120)"
  done
done
