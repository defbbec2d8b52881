set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or gemm_planner_acc or plan_pin or splitk" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1; rc=$?; tail -3 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_attn.py --packed
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pattn -o run --output-format csv -- python3 tools/bench_attn.py --packed --iters 10 > gpurun_out/pattn.log 2>&1 && python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/pattn/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:8.1f} us  {r['Calls']:>4}  {r['Name'][:70]}")
PY
timeout -k 10 240 python -u bench.py --steps 15 --warmup 3 | tail -1 | cut -c1-150
