# round 5 batch 7: stream queue padding x window schedule, with and without a communicator
# (interleaved, 2 reps), plus the queue map of the no-communicator step with one pad queue
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" "$1" "$2"; }
C="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
port=29700
run() {
  n=$1; shift; port=$((port + 1))
  timeout -k 10 300 env MASTER_PORT=$port "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e7_$n.log 2> gpurun_out/e7_$n.err \
    || { tail -20 gpurun_out/e7_$n.err; exit 1; }
  show gpurun_out/e7_$n.log $n
}
for rep in 1 2; do
  run plain.$rep DLT_X=0 && run pad1.$rep DLT_QUEUE_PAD=1 && run pad2.$rep DLT_QUEUE_PAD=2 && \
    run cfb0.$rep $C DLT_WINDOW_SCHED=fb && run cfb3.$rep $C DLT_WINDOW_SCHED=fb DLT_QUEUE_PAD=3 && \
    run cffbb3.$rep $C DLT_WINDOW_SCHED=ffbb DLT_QUEUE_PAD=3 || exit 1
done
R0=$PWD
cd /tmp && export TMPDIR=/tmp
env DLT_QUEUE_PAD=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_e7_pad1" -o run --output-format csv \
  -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_e7_pad1.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_e7_pad1.log"; exit 1; }
cd "$R0"
python tools/queue_map.py gpurun_out/prof_e7_pad1/run_kernel_trace.csv
