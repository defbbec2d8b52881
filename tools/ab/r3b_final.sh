#!/bin/bash
# End-of-session evidence: full GPU suite + headline/lean bench (r3_round.sh), then the bench table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/ab/r3_round.sh || exit 1
echo "bench table..."
timeout -k 10 900 python -u tools/bench_table.py --configs ddp_small,ddp_small_lean,fsdp_small,ddp_medium,fsdp_medium,fsdp_medium_noac,fsdp_xl \
  --out gpurun_out/r3b_bench_table.md > gpurun_out/r3b_bench_table.log 2>&1 || { tail -20 gpurun_out/r3b_bench_table.log; exit 1; }
cat gpurun_out/r3b_bench_table.md
