#!/bin/bash
# Kernel-trace of bench.py with and without an (idle) RCCL communicator at world size 1.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_plain gpurun_out/prof_nccl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plain -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_plain.log 2>&1 || exit 1
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29551
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nccl -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_nccl.log 2>&1 || exit 1
for t in plain nccl; do
  f=$(find gpurun_out/prof_$t -name "*kernel_trace.csv" | head -1)
  python tools/step_profile.py "$f" > gpurun_out/step_$t.md 2>&1
  echo "== $t"; head -20 gpurun_out/step_$t.md
done
