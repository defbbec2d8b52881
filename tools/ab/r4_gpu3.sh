# round 4, third GPU pass: LDS-transposed stores, fp16 kernels + precision tests, ffbb ring, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/ab/r4_gemm_lt.sh > gpurun_out/r4_lt_all.log 2>&1 || { tail -30 gpurun_out/r4_lt_all.log; exit 1; }
cat gpurun_out/r4_lt_all.log
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "fp16 or precision or ffbb or pipelined_window or grads_vs_fp32 or dgrad or gemm_bf16 or attention_packed" > gpurun_out/r4_t3.log 2>&1 || { tail -60 gpurun_out/r4_t3.log; exit 1; }
grep -E 'PASS|FAIL|ERROR' gpurun_out/r4_t3.log | tail -40
REPS=2 STEPS=20 VARIANTS="ring3:DLT_SLOT_RING=3 ring0:DLT_SLOT_RING=0" bash tools/ab/r3b_env_ab.sh
