# round 4, second GPU pass: LDS-transposed stores, ffbb dY ring (tests + bench A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
bash tools/ab/r4_gemm_lt.sh > gpurun_out/r4_lt_all.log 2>&1 || { tail -30 gpurun_out/r4_lt_all.log; exit 1; }
cat gpurun_out/r4_lt_all.log
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "ffbb or pipelined_window" > gpurun_out/r4_t2.log 2>&1 || { tail -40 gpurun_out/r4_t2.log; exit 1; }
tail -3 gpurun_out/r4_t2.log
REPS=2 STEPS=20 VARIANTS="ring3:DLT_SLOT_RING=3 ring0:DLT_SLOT_RING=0" bash tools/ab/r3b_env_ab.sh
