#!/bin/bash
# End-of-round: round_check.sh (GPU suite, smoke, bench, step trace), then the main
# bench-table rows on the same box.
set -u
bash tools/ab/round_check.sh || exit $?
timeout -k 10 900 python -u tools/bench_table.py --configs ddp_small,ddp_small_memfirst,ddp_small_lean,fsdp_small,ddp_small_fp16 \
  --steps 20 --out gpurun_out/bench_table_final.md > gpurun_out/bench_table_final.log 2>&1
rc=$?; echo "bench_table rc=$rc"; cat gpurun_out/bench_table_final.md; exit $rc
