#!/bin/bash
# Long-context rows: the same 32768 tokens per optimizer step at seq 1024 / 4096 / 16384,
# plus standalone attention timings at those lengths.
set -u
mkdir -p gpurun_out
for cfg in "1024 8 4" "4096 2 4" "16384 1 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --seq_len $1 --batch_size $2 --grad_accum $3 --steps 8 --warmup 3 \
    --model_override max_seq_len=$1 > gpurun_out/long_$1.log 2>&1
  rc=$?; echo "seq $1 B$2 GA$3 rc=$rc: $(tail -1 gpurun_out/long_$1.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done
for s in "1024 8" "4096 2" "16384 1"; do
  set -- $s
  timeout -k 10 120 python -u tools/bench_attn.py --packed --S $1 --B $2 > gpurun_out/long_attn_$1.log 2>&1
  rc=$?; echo "attn S$1 B$2 rc=$rc: $(tail -2 gpurun_out/long_attn_$1.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
