#!/bin/bash
# GPU discovery for MI355X nodes (the reference uses nvidia-smi / CUDA_VISIBLE_DEVICES).
detect_gpus() {
  if command -v amd-smi >/dev/null 2>&1; then
    n=$(amd-smi list 2>/dev/null | grep -c '^GPU')
  elif command -v rocm-smi >/dev/null 2>&1; then
    n=$(rocm-smi --showid 2>/dev/null | grep -cE '^GPU\[')
  else
    n=$(python3 -c 'import torch; print(torch.cuda.device_count())' 2>/dev/null)
  fi
  [ -z "$n" ] || [ "$n" = "0" ] && n=1
  echo "$n"
}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}   # dmabuf IPC for RCCL
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}
export NCCL_DEBUG=${NCCL_DEBUG:-WARN}
