# round 4, end: upper bound of moving the RMSNorm weight-gradient column sums off the
# chain streams -- the same build with the column sums skipped (wrong norm grads; timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/cs_$n.log 2> gpurun_out/cs_$n.err || { tail -20 gpurun_out/cs_$n.err; exit 1; }; echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/cs_$n.log)"; }
for rep in 1 2 3; do
  run base.$rep DLT_KERNEL_LIB=_dlt_kernels_nocs.so && run skip.$rep DLT_KERNEL_LIB=_dlt_kernels_nocs.so DLT_SKIP_COLSUM=1 && run wide.$rep DLT_COLSUM_WIDE=1 || exit 1
done
