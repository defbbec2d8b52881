# round 4, end: knob sweep on the final tree (2 interleaved reps; DLT_X=0 = the default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 $BARGS > gpurun_out/sw_$n.log 2> gpurun_out/sw_$n.err || { tail -20 gpurun_out/sw_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/sw_$n.log) $(grep -o '"peak_gb_per_gpu": [0-9.]*' gpurun_out/sw_$n.log)"; }
for rep in 1 2; do
  run def.$rep DLT_X=0 &&
  run ring4.$rep DLT_SLOT_RING=4 &&
  run sring0.$rep DLT_S_RING=0 &&
  run mw0.$rep DLT_MAIN_WGRAD_LAYERS=0 &&
  run mw2.$rep DLT_MAIN_WGRAD_LAYERS=2 &&
  run pair.$rep DLT_ATTN_SCHED=pair &&
  run fl1036.$rep DLT_GEMM_FLAGS=1036 &&
  run hwq32.$rep DLT_HW_QUEUES=32 &&
  BARGS="--fusion 1" run fus1.$rep DLT_X=0 || exit 1
done
