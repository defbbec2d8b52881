# round 4, end: AdamW with 4 float4 groups per thread (DLT_ADAMW_U=4, a knob of the reverted variant; the shipped kernel ignores it) vs 2 -- standalone, then the step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for u in 2 4 2 4; do DLT_ADAMW_U=$u timeout -k 10 120 python tools/adamw_bench.py 2>/dev/null || exit 1; done
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/aw_$n.log 2> gpurun_out/aw_$n.err || { tail -20 gpurun_out/aw_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/aw_$n.log)"; }
for rep in 1 2 3; do
  run u2.$rep DLT_ADAMW_U=2 && run u4.$rep DLT_ADAMW_U=4 || exit 1
done
