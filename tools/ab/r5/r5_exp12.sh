# round 5 batch 12: default schedule with and without a communicator after the placement
# probe became opt-in (must match the round-start defaults: fb under collectives, unbound)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d.get('window'), d.get('stream_placement'))" "$1" "$2"; }
C="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
port=29900
run() {
  n=$1; shift; port=$((port + 1))
  timeout -k 10 300 env MASTER_PORT=$port "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e12_$n.log 2> gpurun_out/e12_$n.err \
    || { tail -20 gpurun_out/e12_$n.err; exit 1; }
  show gpurun_out/e12_$n.log $n
}
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "dispatch_independently or hand_kernels or window" > gpurun_out/e12_tests.log 2>&1 || { tail -30 gpurun_out/e12_tests.log; exit 1; }
tail -1 gpurun_out/e12_tests.log
for rep in 1 2; do
  run plain.$rep DLT_X=0 && run coll.$rep $C && run collpad3.$rep $C DLT_QUEUE_PAD=3 DLT_WINDOW_SCHED=ffbb || exit 1
done
