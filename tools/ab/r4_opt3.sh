# round 4: overlapped optimizer, engine streams bound to queues first (A/B + profile)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/o3_$n.log 2> gpurun_out/o3_$n.err || { tail -20 gpurun_out/o3_$n.err; exit 1; }; }
for rep in 1 2; do
  run ov.$rep && run noov.$rep --no_overlap_optimizer || exit 1
done
for f in gpurun_out/o3_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
bash tools/ab/r4_prof2.sh ov3 > /dev/null
python tools/queue_map.py gpurun_out/prof_ov3/run_kernel_trace.csv 2>/dev/null || true
