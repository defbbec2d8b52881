#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attn or attention or dropout" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/attn_tests.log)"; [ $rc -eq 0 ] || exit $rc
bash tools/ab/attn_split.sh || exit 1
bash tools/ab/ab_kernels.sh 2
