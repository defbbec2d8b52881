#!/bin/bash
# One forced-collective RCCL rank: which round-6 comm change costs the step?  Variants:
# shipped; RCCL channel floor off (NCCL_MIN_NCHANNELS=4); head-bucket split off
# (DLT_DDP_SPLIT_HEAD=0); high-priority collective stream off.  Plain (no collectives) first.
mkdir -p gpurun_out
set -o pipefail
run() {  # $1 = tag, $2 = port, rest = env
  local tag=$1 port=$2; shift 2
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus 1 --steps 20 --warmup 3 > "gpurun_out/rk_$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(grep '"metric"' "gpurun_out/rk_$tag.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("window"), d.get("window_choice"))')"
  return $rc
}
for r in 1 2; do
  run plain$r 2953$r DLT_FORCE_COLLECTIVES=0 && \
  run forced$r 2954$r DLT_FORCE_COLLECTIVES=1 && \
  run ch4_$r 2955$r DLT_FORCE_COLLECTIVES=1 NCCL_MIN_NCHANNELS=4 && \
  run nosplit$r 2956$r DLT_FORCE_COLLECTIVES=1 DLT_DDP_SPLIT_HEAD=0 && \
  run noprio$r 2957$r DLT_FORCE_COLLECTIVES=1 TORCH_NCCL_HIGH_PRIORITY=0 || exit 1
done
