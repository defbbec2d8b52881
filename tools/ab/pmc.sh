#!/bin/bash
# rocprofv3 hardware-counter passes (one rocprofv3 run per pass, counters within the
# per-block limits; never combined with trace domains).  Usage: bash tools/ab/pmc.sh <tag> <python args...>
set -u
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc_$tag
A="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES"
B="FETCH_SIZE GRBM_GUI_ACTIVE"
C="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for pass in "$A" "$B" "$C"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/pmc_$tag/p$i -o run --output-format csv -- python3 "$@" \
    > gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -3 gpurun_out/pmc_$tag/p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
