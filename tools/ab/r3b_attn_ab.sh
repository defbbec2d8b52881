#!/bin/bash
# A/B of two kernel libraries (DLT_KERNEL_LIB) on the attention micro-bench and bench.py.
# LIBS="name:lib.so name2:lib2.so"; attention GPU tests run first with the default library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/attn_ab_tests.log 2>&1 || { tail -30 gpurun_out/attn_ab_tests.log; exit 1; }
tail -1 gpurun_out/attn_ab_tests.log
for rep in 1 2; do
  for spec in $LIBS; do
    name=${spec%%:*}; so=${spec#*:}
    DLT_KERNEL_LIB=$so timeout -k 10 120 python tools/bench_attn.py --packed --B 16 --iters 50 > gpurun_out/attn_$name.$rep.log 2>&1 \
      || { tail -20 gpurun_out/attn_$name.$rep.log; exit 1; }
    echo "$name $(tail -2 gpurun_out/attn_$name.$rep.log | tr '\n' ' ')"
  done
done
for rep in 1 2; do
  for spec in $LIBS; do
    name=${spec%%:*}; so=${spec#*:}
    DLT_KERNEL_LIB=$so timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/attnb_$name.$rep.log 2> gpurun_out/attnb_$name.$rep.err \
      || { tail -20 gpurun_out/attnb_$name.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/attnb_$name.$rep.log $name
  done
done
