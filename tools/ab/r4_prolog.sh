# round 4: attention kernels with the first tile's DMA overlapped with the row loads (current tree)
# vs HEAD's library (ops/_dlt_kernels_base.so): tests, isolated times, in-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 200 --timeout-method thread \
  > gpurun_out/pl_t.log 2>&1 || { tail -40 gpurun_out/pl_t.log; exit 1; }
tail -1 gpurun_out/pl_t.log
for lib in _dlt_kernels_base.so _dlt_kernels.so _dlt_kernels_base.so _dlt_kernels.so; do
  DLT_KERNEL_LIB=$lib timeout -k 10 120 python tools/bench_attn.py --B 16 --packed --iters 50 > gpurun_out/pl_ab.log 2>&1 || { cat gpurun_out/pl_ab.log; exit 1; }
  echo "$lib $(tail -2 gpurun_out/pl_ab.log | tr '\n' ' ')"
done
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/pl_$n.log 2> gpurun_out/pl_$n.err || { tail -20 gpurun_out/pl_$n.err; exit 1; }; }
for rep in 1 2; do
  run base.$rep DLT_KERNEL_LIB=_dlt_kernels_base.so && run new.$rep DLT_KERNEL_LIB=_dlt_kernels.so || exit 1
done
for f in gpurun_out/pl_base*.log gpurun_out/pl_new*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
