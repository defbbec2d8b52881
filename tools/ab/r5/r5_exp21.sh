# round 5 batch 21: one forward role at a time on the persistent hand GEMM vs the shipped
# plan (library forwards), 3 interleaved repetitions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
V="lib:DLT_X=0"
for r in qkv o gu down head; do V="$V $r:DLT_GEMM_PLAN=tools/ab/r5/plan_r5_one_$r.json"; done
VARIANTS="$V" REPS=3 bash tools/ab/env_ab.sh
