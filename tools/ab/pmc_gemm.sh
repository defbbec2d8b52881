#!/bin/bash
# rocprofv3 counter passes over tools/bench_gemm_fwd.py runs (one rocprofv3 run per pass,
# within the per-block slot limits; never combined with trace domains).
# usage: bash tools/ab/pmc_gemm.sh <tag> <bench_gemm_fwd.py args...>; summary: tools/pmc_raw.py
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
out=gpurun_out/pmcg_$1; shift
mkdir -p $out
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES" \
            "FETCH_SIZE TCC_HIT_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $out/p$i -o run --output-format csv -- python3 tools/bench_gemm_fwd.py "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $out/p$i.log; exit 1; }
done
echo ok
