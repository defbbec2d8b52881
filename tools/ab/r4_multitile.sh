set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "multi_tile" > gpurun_out/r4_mt.log 2>&1; tail -30 gpurun_out/r4_mt.log
