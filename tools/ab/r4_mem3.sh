# round 4: headline memory -- early chunked lm_head with / without the shared chunk buffer, mask regeneration
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/mm_$n.log 2> gpurun_out/mm_$n.err || { tail -20 gpurun_out/mm_$n.err; exit 1; }; }
for rep in 1 2; do
  run def.$rep DLT_X=0 && run hc2.$rep DLT_HEAD_CHUNKS=2 && run hc2ns.$rep DLT_HEAD_CHUNKS=2 DLT_HEAD_SHARE=0 &&
  run hc4ns.$rep DLT_HEAD_CHUNKS=4 DLT_HEAD_SHARE=0 || exit 1
done
for f in gpurun_out/mm_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
