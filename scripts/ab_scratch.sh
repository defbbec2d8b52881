set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?; tail -1 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 240 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "fail $tag"; tail -5 gpurun_out/ab_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/ab_$tag.log | cut -c1-110)"; }
for r in 1 2; do
run pre$r python -u bench.py --steps 20 --warmup 3
run nopre$r env DLT_MASK_PREFETCH=0 python -u bench.py --steps 20 --warmup 3
done
