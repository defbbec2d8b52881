#!/bin/bash
# Per-kernel attention times (rocprofv3 --stats) at equal tokens, S = 1024 .. 16384.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for s in "1024 16" "2048 8" "4096 4" "16384 1"; do
  set -- $s
  rm -rf gpurun_out/ak_$1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ak_$1 -o run --output-format csv -- python3 tools/bench_attn.py --packed --S $1 --B $2 --p 0.1 > gpurun_out/ak_$1.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "fail $1"; tail -5 gpurun_out/ak_$1.log; exit $rc; }
  f=$(find gpurun_out/ak_$1 -name "*kernel_stats.csv" | head -1)
  echo "== S$1 B$2"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'attn' in n or 'dropout' in n: print('  %-40s calls %5s avg %8.1f us' % (n[:40], r['Calls'], float(r['AverageNs'])/1e3))
"
done
