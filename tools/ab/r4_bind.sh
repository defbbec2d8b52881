# round 4: engine streams bound to hardware queues at engine creation (DLT_BIND_STREAMS=1) vs lazily;
# no communicator / one-rank RCCL with forced collectives (fb and ffbb windows); queue map
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/b_$n.log 2> gpurun_out/b_$n.err || { tail -20 gpurun_out/b_$n.err; exit 1; }; }
run plain0 DLT_BIND_STREAMS=0 && run plain1 DLT_BIND_STREAMS=1 &&
run ffbb0 $R MASTER_PORT=29621 DLT_WINDOW_SCHED=ffbb DLT_BIND_STREAMS=0 &&
run ffbb1 $R MASTER_PORT=29622 DLT_WINDOW_SCHED=ffbb DLT_BIND_STREAMS=1 &&
run fb1 $R MASTER_PORT=29623 DLT_BIND_STREAMS=1 && run fb0 $R MASTER_PORT=29624 DLT_BIND_STREAMS=0 || exit 1
for f in gpurun_out/b_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
R0=$PWD
cd /tmp && export TMPDIR=/tmp
env $R MASTER_PORT=29625 DLT_WINDOW_SCHED=ffbb DLT_BIND_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_bffbb" -o run --output-format csv \
  -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_bffbb.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_bffbb.log"; exit 1; }
cd "$R0"
python tools/queue_map.py $(find gpurun_out/prof_bffbb -name '*kernel_trace.csv' | head -1)
