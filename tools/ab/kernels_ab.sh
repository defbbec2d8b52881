#!/bin/bash
# Same-box A/B of a kernel change: bench.py with ops/_dlt_kernels_base.so (built from
# another revision by tools/ab/build_base_lib.sh) against the current ops/_dlt_kernels.so,
# alternating.  usage: bash tools/ab/kernels_ab.sh [rounds] [bench args...]
set -u
mkdir -p gpurun_out
R=${1:-2}; shift || true
for r in $(seq 1 $R); do
  for v in base new; do
    lib=_dlt_kernels.so; [ $v = base ] && lib=_dlt_kernels_base.so
    DLT_KERNEL_LIB=$lib timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 "$@" > gpurun_out/abk_$v$r.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/abk_$v$r.log; exit 1; }
    echo "$v#$r: $(tail -1 gpurun_out/abk_$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
