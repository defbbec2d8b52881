#!/bin/bash
# Round-3 (session 2) baseline: headline bench, per-role GEMM timings at the chain shape, attention.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b_base.log 2> gpurun_out/b_base.err || { tail -20 gpurun_out/b_base.err; exit 1; }
cat gpurun_out/b_base.log
timeout -k 10 300 python -u tools/gemm_roles.py 16384 2 > gpurun_out/roles_base.log 2>&1 || { tail -20 gpurun_out/roles_base.log; exit 1; }
head -12 gpurun_out/roles_base.log
timeout -k 10 120 python -u tools/bench_attn.py --packed --B 16 > gpurun_out/attn_base.log 2>&1 || { tail -20 gpurun_out/attn_base.log; exit 1; }
cat gpurun_out/attn_base.log
