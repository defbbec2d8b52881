#!/bin/bash
# gc.freeze() after trainer setup (default) vs off, same box; GC collection counts/times.
mkdir -p gpurun_out
for r in 1 2; do for f in 0 1; do
  DLT_GC_FREEZE=$f timeout -k 10 300 python tools/gc_probe.py > gpurun_out/gc_$f.log 2>&1 || exit 1
  echo "freeze=$f: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gc_$f.log) $(grep '^gc:' gpurun_out/gc_$f.log)"
done; done
