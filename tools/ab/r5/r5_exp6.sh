# round 5 batch 6: fp32 kernel tests; head_dim 128 attention tests; queue maps of the forced-collective ffbb step with and
# without the stream queue padding, plus the padding's effect without a communicator
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp32_kernels_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/e6_tests.log 2>&1 || { tail -40 gpurun_out/e6_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/e6_tests.log | tail -14
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "attention or head_dim" > gpurun_out/e6_attn.log 2>&1 || { tail -40 gpurun_out/e6_attn.log; exit 1; }
tail -3 gpurun_out/e6_attn.log
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 500 --timeout-method thread \
  -k "hand_kernels" > gpurun_out/e6_dist.log 2>&1 || { tail -40 gpurun_out/e6_dist.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/e6_dist.log | tail -4
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" "$1" "$2"; }
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e6_$n.log 2> gpurun_out/e6_$n.err || { tail -20 gpurun_out/e6_$n.err; exit 1; }; show gpurun_out/e6_$n.log $n; }
run nocomm.pad0 DLT_X=0 && run nocomm.pad3 DLT_QUEUE_PAD=3 || exit 1
R0=$PWD
cd /tmp && export TMPDIR=/tmp
for pad in 0 3; do
  env RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=2965$pad DLT_FORCE_COLLECTIVES=1 \
    DLT_WINDOW_SCHED=ffbb DLT_QUEUE_PAD=$pad timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_e6_pad$pad" -o run \
    --output-format csv -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_e6_pad$pad.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_e6_pad$pad.log"; exit 1; }
done
env DLT_X=0 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_e6_nocomm" -o run --output-format csv \
  -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_e6_nocomm.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_e6_nocomm.log"; exit 1; }
cd "$R0"
for v in pad0 pad3 nocomm; do
  f=$(find gpurun_out/prof_e6_$v -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python tools/queue_map.py "$f"
done
