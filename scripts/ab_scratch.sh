set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/tune_gemm_plan.py --out gpurun_out/gemm_plan_mi355x.json > gpurun_out/tune.log 2>&1; rc=$?; grep -E "^step|wrote" gpurun_out/tune.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/tune.log; exit $rc; }
run() { tag=$1; shift; timeout -k 10 240 "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "fail $tag"; tail -5 gpurun_out/ab_$tag.log; exit 1; }; echo "$tag: $(tail -1 gpurun_out/ab_$tag.log | cut -c1-110)"; }
for r in 1 2; do
run plan$r env DLT_GEMM_PLAN=gpurun_out/gemm_plan_mi355x.json python -u bench.py --steps 20 --warmup 3
run noplan$r env DLT_GEMM_PLAN=none python -u bench.py --steps 20 --warmup 3
done
