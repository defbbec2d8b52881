# round 5: FSDP reduce-scatter every micro-step (reference) vs once per step with deferred
# weight gradients (--fsdp_defer_sync), small and medium, 2 interleaved reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for r in 1 2; do
  for m in small medium; do
    if [ $m = small ]; then a="--batch_size 8 --grad_accum 4"; else a="--batch_size 4 --grad_accum 8"; fi
    for d in "" "--fsdp_defer_sync"; do
      timeout -k 10 300 python bench.py --mode fsdp --model_size $m $a --steps 8 --warmup 3 $d > gpurun_out/fd.log 2>&1 \
        || { tail -20 gpurun_out/fd.log; exit 1; }
      echo "$r $m ${d:-every}: $(grep '"metric"' gpurun_out/fd.log | cut -c1-110) $(grep -o '"peak_gb_per_gpu": [0-9.]*' gpurun_out/fd.log)"
    done
  done
done
