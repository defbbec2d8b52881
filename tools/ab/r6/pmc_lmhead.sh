#!/bin/bash
# Counters of the lm_head forward: hipBLASLt vs fw4 variants, one impl per rocprofv3 run.
set -u
for impl in lib fw4x2 fw4s5x2e; do
  bash tools/ab/pmc_gemm.sh lm_$impl --shapes lm_head --impls $impl --iters 10 || exit 1
  python tools/pmc_raw.py gpurun_out/pmcg_lm_$impl > gpurun_out/pmcg_lm_$impl.txt
done
