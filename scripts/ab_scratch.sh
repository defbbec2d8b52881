set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1; rc=$?; tail -2 gpurun_out/t_attn.log; [ $rc -eq 0 ] || exit $rc
for B in 8 16; do
  echo "B=$B: $(timeout -k 10 120 python tools/bench_attn.py --packed --B $B)"
done
run() { tag=$1; shift; timeout -k 10 240 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "fail $tag"; tail -5 gpurun_out/ab_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/ab_$tag.log | cut -c1-120)"; }
run b1 python -u bench.py --steps 20 --warmup 3
run b2 python -u bench.py --steps 20 --warmup 3
