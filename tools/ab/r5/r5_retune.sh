# round 5: fresh exhaustive tuning of the headline step's GEMM keys vs the shipped plan
# (3 interleaved reps of the default bench)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/tune_gemm_plan.py --configs ddp_small --out gpurun_out/plan_fresh.json > gpurun_out/retune.log 2>&1 \
  || { tail -30 gpurun_out/retune.log; exit 1; }
grep -E "step|wrote" gpurun_out/retune.log
for r in 1 2 3; do
  for plan in shipped fresh; do
    if [ $plan = fresh ]; then export DLT_GEMM_PLAN=gpurun_out/plan_fresh.json; else unset DLT_GEMM_PLAN; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/rt.log 2>&1 || { tail -20 gpurun_out/rt.log; exit 1; }
    echo "$r $plan: $(grep '"metric"' gpurun_out/rt.log | cut -c1-100)"
  done
done
