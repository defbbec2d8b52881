#!/bin/bash
# One forced-collective RCCL rank: dense embedding part (new default) vs the row-sparse
# union (DLT_DDP_SPARSE_ROWS=0.5, host sync per step), plain runs as reference.
mkdir -p gpurun_out
set -o pipefail
run() {
  local tag=$1 port=$2; shift 2
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus 1 --steps 20 --warmup 3 > "gpurun_out/rs_$tag.log" 2>&1
  local rc=$?
  echo "$tag rc=$rc: $(grep '"metric"' "gpurun_out/rs_$tag.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("window"), d.get("window_choice"))')"
  return $rc
}
for r in 1 2 3; do
  run plain$r 2961$r DLT_FORCE_COLLECTIVES=0 && \
  run dense$r 2962$r DLT_FORCE_COLLECTIVES=1 && \
  run sparse$r 2963$r DLT_FORCE_COLLECTIVES=1 DLT_DDP_SPARSE_ROWS=0.5 || exit 1
done
