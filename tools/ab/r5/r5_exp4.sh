# round 5 batch 4: (a) dswiglu start-delay desync (isolated), (b) forced-collective ffbb with a
# high-priority RCCL stream, (c) hand forward GEMM plan with other forward launch flags
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
DSW_FLAGS=3084,201330188,419433996,671092236,1006636556 timeout -k 10 120 tools/cpp/gemm_bench dgrad 16384 3072 768 > gpurun_out/e4_dsw.log 2>&1 || { cat gpurun_out/e4_dsw.log; exit 1; }
cat gpurun_out/e4_dsw.log
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" "$1" "$2"; }
R="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DLT_FORCE_COLLECTIVES=1"
runc() { n=$1; shift; timeout -k 10 300 env $R "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e4_$n.log 2> gpurun_out/e4_$n.err || { tail -20 gpurun_out/e4_$n.err; exit 1; }; show gpurun_out/e4_$n.log $n; }
runc cfb MASTER_PORT=29631 && runc cffbb MASTER_PORT=29632 DLT_WINDOW_SCHED=ffbb && \
  runc cffbbhp MASTER_PORT=29633 DLT_WINDOW_SCHED=ffbb TORCH_NCCL_HIGH_PRIORITY=1 && \
  runc cfbhp MASTER_PORT=29634 TORCH_NCCL_HIGH_PRIORITY=1 && runc plain MASTER_PORT=29635 DLT_FORCE_COLLECTIVES=0 || exit 1
H=tools/ab/r5/plan_r5_fwdhand.json
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/e4_$n.log 2> gpurun_out/e4_$n.err || { tail -20 gpurun_out/e4_$n.err; exit 1; }; show gpurun_out/e4_$n.log $n; }
for rep in 1 2; do
  run lib.$rep DLT_X=0 && run hand.$rep DLT_GEMM_PLAN=$H && run handgrp.$rep DLT_GEMM_PLAN=$H DLT_GEMM_FWD_FLAGS=3072 && \
    run handnosc1.$rep DLT_GEMM_PLAN=$H DLT_GEMM_FWD_FLAGS=1036 || exit 1
done
