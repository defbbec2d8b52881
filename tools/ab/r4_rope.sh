# round 4, end: QKV + RoPE fused hand GEMM vs QKV GEMM (hipBLASLt or hand) + k_rope_qk_inplace, in the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/rp_$n.log 2> gpurun_out/rp_$n.err || { tail -20 gpurun_out/rp_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/rp_$n.log)"; }
for rep in 1 2 3; do
  run fused.$rep DLT_X=0 && run lib.$rep DLT_GEMM_PLAN=tools/ab/plan_norope.json && run hand.$rep DLT_GEMM_PLAN=tools/ab/plan_norope_hand.json || exit 1
done
