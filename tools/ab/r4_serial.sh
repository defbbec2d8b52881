# round 4: single-stream step (every kernel alone) -- bench + kernel-trace breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
export DLT_PIPELINE=0 DLT_WGRAD_STREAM=0 DLT_BWD_OVERLAP=0
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ser_bench.log 2> gpurun_out/ser_bench.err || { tail -20 gpurun_out/ser_bench.err; exit 1; }
tail -1 gpurun_out/ser_bench.log
bash tools/ab/r4_prof2.sh ser > /dev/null || exit 1
head -75 gpurun_out/step_ser.md
