# round 5 batch 17: private norm-weight gradients for the second ffbb backward (no per-block
# wait on the first one): window / trainer GPU tests (bitwise vs sequential), then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "window or pipelined or ffbb or trainer or rccl or ddp" > gpurun_out/e17_tests.log 2>&1 || { tail -30 gpurun_out/e17_tests.log; exit 1; }
tail -1 gpurun_out/e17_tests.log
VARIANTS="priv:DLT_X=0 nopriv:DLT_PRIV_NORM=0 noshare:DLT_HEAD_SHARE=0" REPS=3 bash tools/ab/env_ab.sh
bash tools/ab/prof_step.sh r5priv > gpurun_out/e17_prof.txt 2>&1 || { tail -5 gpurun_out/e17_prof.txt; exit 1; }
python tools/concurrency.py gpurun_out/prof_r5priv/run_kernel_trace.csv | head -3
