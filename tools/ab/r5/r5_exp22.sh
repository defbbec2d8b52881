# round 5 batch 22: hand QKV forward (separate RoPE), hand QKV + o, fused QKV + RoPE epilogue
# vs the shipped plan, 4 interleaved repetitions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
VARIANTS="lib:DLT_X=0 qkv:DLT_GEMM_PLAN=tools/ab/r5/plan_r5_one_qkv.json qkvo:DLT_GEMM_PLAN=tools/ab/r5/plan_r5_qkvo.json roped:DLT_GEMM_PLAN=tools/ab/r5/plan_r5_roped.json" \
  REPS=4 bash tools/ab/env_ab.sh
