# round 4, end: SwiGLU output kept per layer from the forward (DLT_S_RING=0) vs rewritten into the ring by the
# fused down-dgrad epilogue (default); with the fused epilogue off for comparison
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/sr_$n.log 2> gpurun_out/sr_$n.err || { tail -20 gpurun_out/sr_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/sr_$n.log) $(grep -o '"peak_gb_per_gpu": [0-9.]*' gpurun_out/sr_$n.log)"; }
for rep in 1 2 3; do
  run ring.$rep DLT_S_RING=1 && run noring.$rep DLT_S_RING=0 &&
  run noring_nodsw.$rep DLT_S_RING=0 DLT_GEMM_PLAN=tools/ab/plan_nodsw.json || exit 1
done
