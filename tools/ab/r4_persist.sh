# round 4: persistent dK/dV attention kernel -- bitwise tests, isolated bwd time, in-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 200 --timeout-method thread \
  > gpurun_out/p_t.log 2>&1 || { tail -40 gpurun_out/p_t.log; exit 1; }
tail -1 gpurun_out/p_t.log
for v in 0 1 0 1; do
  DLT_ATTN_PERSIST=$v timeout -k 10 120 python tools/bench_attn.py --B 16 --packed --iters 50 > gpurun_out/p_ab$v.log 2>&1 || { cat gpurun_out/p_ab$v.log; exit 1; }
  echo "persist=$v $(tail -1 gpurun_out/p_ab$v.log)"
done
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/p_$n.log 2> gpurun_out/p_$n.err || { tail -20 gpurun_out/p_$n.err; exit 1; }; }
for rep in 1 2; do
  run off.$rep DLT_ATTN_PERSIST=0 && run on.$rep DLT_ATTN_PERSIST=1 || exit 1
done
for f in gpurun_out/p_o*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
