#!/bin/bash
# Stream-K vs split-K hand-written weight gradient (T = 32768 deferred window), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
o=gpurun_out/wgrad_sk.log; : > $o
run() { echo "== $*" >> $o; env "$@" >> $o 2>&1 || { tail -5 $o; exit 1; }; }
for shp in "2304 768:4 7" "768 768:16 21" "6144 768:8" "768 3072:5" "50304 768:2"; do
  dims=${shp%%:*}; sp=${shp##*:}
  for s in $sp; do run GW_SPLITS=$s timeout -k 10 120 tools/cpp/gemm_bench wgrad 32768 $dims; done
  run GW_SPLITS=-1 timeout -k 10 120 tools/cpp/gemm_bench wgrad 32768 $dims
done
run GW_SPLITS=-1 GW_GC=32 timeout -k 10 120 tools/cpp/gemm_bench wgrad 32768 6144 768
run GW_SPLITS=-1 GW_GC=128 timeout -k 10 120 tools/cpp/gemm_bench wgrad 32768 6144 768
grep -E "wgrad T|stream-K" $o
