# round 5: the shipped plan with the fp32 + fp16 pins added -- default, fp16 and fp32 benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for p in bf16 fp16 fp32; do
  steps=10; [ $p = fp32 ] && steps=6
  timeout -k 10 300 python bench.py --precision $p --steps $steps --warmup 3 > gpurun_out/pc_$p.log 2>&1 || { tail -20 gpurun_out/pc_$p.log; exit 1; }
  echo "$p: $(grep '"metric"' gpurun_out/pc_$p.log | cut -c1-130)"
done
