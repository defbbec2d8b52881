# round 4, end: knob sweep on the final default (SwiGLU output per layer), 2 interleaved reps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 $BARGS > gpurun_out/sx_$n.log 2> gpurun_out/sx_$n.err || { tail -20 gpurun_out/sx_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/sx_$n.log) $(grep -o '"peak_gb_per_gpu": [0-9.]*' gpurun_out/sx_$n.log)"; }
for rep in 1 2; do
  run def.$rep DLT_X=0 &&
  run ring0.$rep DLT_SLOT_RING=0 &&
  run ring4.$rep DLT_SLOT_RING=4 &&
  run grid0.$rep DLT_FFBB_GEMM_GRID=0 &&
  run mw0.$rep DLT_MAIN_WGRAD_LAYERS=0 &&
  run xcd0.$rep DLT_ATTN_XCD=0 &&
  run fl1036.$rep DLT_GEMM_FLAGS=1036 &&
  run cent0.$rep DLT_CE_NT=0 &&
  run fwdnt0.$rep DLT_FWD_NT=0 || exit 1
done
