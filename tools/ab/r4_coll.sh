# round 4: one-rank RCCL with forced collectives: fb vs ffbb window + HSA queue map of the ffbb step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
run() { n=$1; shift; timeout -k 10 300 env $R "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/c_$n.log 2> gpurun_out/c_$n.err || { tail -20 gpurun_out/c_$n.err; exit 1; }; }
run fb.1 MASTER_PORT=29611 && run ffbb.1 MASTER_PORT=29612 DLT_WINDOW_SCHED=ffbb && run plain.1 MASTER_PORT=29613 DLT_FORCE_COLLECTIVES=0 || exit 1
for f in gpurun_out/c_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
R0=$PWD
cd /tmp && export TMPDIR=/tmp
env $R MASTER_PORT=29614 DLT_WINDOW_SCHED=ffbb timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_cffbb" -o run --output-format csv \
  -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_cffbb.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_cffbb.log"; exit 1; }
cd "$R0"
f=$(find gpurun_out/prof_cffbb -name '*kernel_trace.csv' | head -1)
python tools/queue_map.py "$f"
python tools/step_profile.py "$f" > gpurun_out/step_cffbb.md; head -8 gpurun_out/step_cffbb.md
