# round 4, end: each hand dgrad pin flipped to hipBLASLt against the final plan (QKV forward on the library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/dg_$n.log 2> gpurun_out/dg_$n.err || { tail -20 gpurun_out/dg_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/dg_$n.log)"; }
for rep in 1 2 3; do
  run base.$rep DLT_X=0 || exit 1
  for v in dgqkv dgo dggu dglm; do run $v.$rep DLT_GEMM_PLAN=tools/ab/plan_e_$v.json || exit 1; done
done
