#!/bin/bash
# Kernel stats of the fused decode step (graph replays) for GPT-2 small, B = 1.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_dec
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec -o run --output-format csv -- python3 tools/bench_decode.py small 1 100 > gpurun_out/prof_dec.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_dec.log; exit $rc; }
f=$(find gpurun_out/prof_dec -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
rows=sorted(csv.DictReader(open('$f')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:24]: print('%-60s calls %6s avg %7.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
f=$(find gpurun_out/prof_dec -name "*kernel_trace.csv" | head -1)
python3 -c "
import csv
rows=sorted(csv.DictReader(open('$f')), key=lambda r: int(r['Start_Timestamp']))
# last 61 k_dec kernels = one replayed step
dec=[r for r in rows if 'k_dec' in r['Kernel_Name']]
step=dec[-61:]
t0=int(step[0]['Start_Timestamp']); t1=int(step[-1]['End_Timestamp'])
busy=sum(int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in step)
print('one step: span %.1f us, kernel busy %.1f us, %d kernels' % ((t1-t0)/1e3, busy/1e3, len(step)))
"
