# round 5: lazy (per-unit, next-forward) optimizer step -- GPU bitwise tests, then bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "lazy or bitwise_reproducible" > gpurun_out/lz_tests.log 2>&1 || { tail -40 gpurun_out/lz_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/lz_tests.log | tail -8
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/lz_$n.log 2> gpurun_out/lz_$n.err || { tail -20 gpurun_out/lz_$n.err; exit 1; }; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d['final_loss'])" gpurun_out/lz_$n.log $n; }
for rep in 1 2 3; do
  run off.$rep DLT_LAZY_OPT=off && run inline.$rep DLT_LAZY_OPT=inline && run stream.$rep DLT_LAZY_OPT=stream || exit 1
done
