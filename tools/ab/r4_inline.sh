# round 4: the window's last layers' weight gradients per chain (DLT_INLINE_WGRAD_LAYERS) -- tests + in-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "ffbb_hand or forced_fused" > gpurun_out/i_t.log 2>&1 || { tail -40 gpurun_out/i_t.log; exit 1; }
tail -1 gpurun_out/i_t.log
DLT_INLINE_WGRAD_LAYERS=1 timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "ffbb_hand or forced_fused or window_ffbb_matches" > gpurun_out/i_t1.log 2>&1 || { tail -40 gpurun_out/i_t1.log; exit 1; }
tail -1 gpurun_out/i_t1.log
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/i_$n.log 2> gpurun_out/i_$n.err || { tail -20 gpurun_out/i_$n.err; exit 1; }; }
for rep in 1 2; do
  run l0.$rep DLT_INLINE_WGRAD_LAYERS=0 && run l1.$rep DLT_INLINE_WGRAD_LAYERS=1 && run l2.$rep DLT_INLINE_WGRAD_LAYERS=2 || exit 1
done
for f in gpurun_out/i_l*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
