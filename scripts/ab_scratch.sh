set -u
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 240 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "fail $tag"; tail -5 gpurun_out/ab_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/ab_$tag.log | cut -c1-110)"; }
for r in 1 2 3; do
run def$r python -u bench.py --steps 20 --warmup 3
run hp$r env DLT_MAIN_PRIO=high python -u bench.py --steps 20 --warmup 3
done
