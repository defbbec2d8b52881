# round 5 batch 5: (a) forced-collective ffbb vs stream queue padding, (b) partial hand forward
# plans (o + down, + qkv) persistent vs one tile per workgroup, (c) start-delay desync in-step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" "$1" "$2"; }
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1 DLT_WINDOW_SCHED=ffbb"
runc() { n=$1; shift; timeout -k 10 300 env $R "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e5_$n.log 2> gpurun_out/e5_$n.err || { tail -20 gpurun_out/e5_$n.err; exit 1; }; show gpurun_out/e5_$n.log $n; }
runc pad0 MASTER_PORT=29641 && runc pad1 MASTER_PORT=29642 DLT_QUEUE_PAD=1 && runc pad2 MASTER_PORT=29643 DLT_QUEUE_PAD=2 && \
  runc pad3 MASTER_PORT=29644 DLT_QUEUE_PAD=3 || exit 1
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e5_$n.log 2> gpurun_out/e5_$n.err || { tail -20 gpurun_out/e5_$n.err; exit 1; }; show gpurun_out/e5_$n.log $n; }
for rep in 1 2; do
  run lib.$rep DLT_X=0 && run od.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_od.json && \
    run od1t.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_od.json DLT_GEMM_FWD_FLAGS=3340 && \
    run odq1t.$rep DLT_GEMM_PLAN=tools/ab/r5/plan_r5_odq.json DLT_GEMM_FWD_FLAGS=3340 && \
    run desync.$rep DLT_GEMM_FLAGS=201330188 || exit 1
done
