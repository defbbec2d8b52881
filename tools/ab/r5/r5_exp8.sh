# round 5 batch 8: full GPU suite (fp32 kernels, head_dim 128, stream placement probe), then
# the default schedule with and without a communicator (the probe now decides) vs fb
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/e8_tests.log 2>&1 \
  || { tail -40 gpurun_out/e8_tests.log; exit 1; }
tail -2 gpurun_out/e8_tests.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d.get('window'), d.get('stream_placement'))" "$1" "$2"; }
C="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
port=29800
run() {
  n=$1; shift; port=$((port + 1))
  timeout -k 10 300 env MASTER_PORT=$port "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e8_$n.log 2> gpurun_out/e8_$n.err \
    || { tail -20 gpurun_out/e8_$n.err; exit 1; }
  show gpurun_out/e8_$n.log $n
}
for rep in 1 2; do
  run plain.$rep DLT_X=0 && run coll.$rep $C && run collfb.$rep $C DLT_WINDOW_SCHED=fb || exit 1
done
# fp16 data gradients: hand-written (routed since round 5) vs hipBLASLt
runp() {
  n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 --precision fp16 > gpurun_out/e8_$n.log 2> gpurun_out/e8_$n.err \
    || { tail -20 gpurun_out/e8_$n.err; exit 1; }
  show gpurun_out/e8_$n.log $n
}
for rep in 1 2 3; do
  runp f16hand.$rep DLT_X=0 && runp f16lib.$rep DLT_GEMM_DGRAD=0 || exit 1
done
