#!/bin/bash
# Usage: scripts/train_fsdp.sh [NUM_GPUS] [MODEL_SIZE] [EXTRA ARGS...]
# (reference: scripts/train_fsdp.sh -- same arguments; ROCm device discovery)
set -e
cd "$(dirname "$0")/.."
source scripts/common.sh
NUM_GPUS=${1:-$(detect_gpus)}
MODEL_SIZE=${2:-medium}
shift 2 2>/dev/null || shift $# 2>/dev/null || true
if [ -z "${HIP_VISIBLE_DEVICES:-}" ]; then
  export HIP_VISIBLE_DEVICES=$(seq -s, 0 $((NUM_GPUS - 1)))
fi
echo "Training GPT-2 ${MODEL_SIZE} with FSDP on ${NUM_GPUS} MI355X GPU(s)"
maybe_build
python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc_per_node="${NUM_GPUS}" \
  src/training/fsdp_trainer.py --model_size "${MODEL_SIZE}" --batch_size 4 --max_steps 1000 \
  --sharding FULL_SHARD "$@"
echo "Training complete!"
