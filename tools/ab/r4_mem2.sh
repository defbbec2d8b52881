# round 4: default (s ring) vs memory-lean with / without the chunked early head; FSDP
# CPU offload with the staged D2H copies
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4_mem2_t.log 2>&1 || { tail -60 gpurun_out/r4_mem2_t.log; exit 1; }
tail -1 gpurun_out/r4_mem2_t.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/m2_default.$rep.log 2>gpurun_out/m2_default.$rep.err &&
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --memory_lean > gpurun_out/m2_lean.$rep.log 2>gpurun_out/m2_lean.$rep.err &&
  DLT_HEAD_CHUNKS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --memory_lean > gpurun_out/m2_leanc0.$rep.log 2>gpurun_out/m2_leanc0.$rep.err || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mode fsdp > gpurun_out/m2_fsdp.log 2>gpurun_out/m2_fsdp.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --mode fsdp --cpu_offload > gpurun_out/m2_fsdp_off.log 2>gpurun_out/m2_fsdp_off.err || exit 1
for f in gpurun_out/m2_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
