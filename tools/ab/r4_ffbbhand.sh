set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -v --timeout 200 --timeout-method thread -k "ffbb_hand" > gpurun_out/r4_fh.log 2>&1; grep -E 'PASS|FAIL|Error|assert' gpurun_out/r4_fh.log | head -30
