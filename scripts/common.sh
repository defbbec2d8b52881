#!/bin/bash
# Shared setup for scripts/train_{ddp,fsdp}.sh: MI355X GPU discovery and the RCCL / HIP
# environment for one node of 8 GPUs on point-to-point xGMI (the reference uses
# nvidia-smi / CUDA_VISIBLE_DEVICES and NCCL_DEBUG / NCCL_IB_DISABLE, scripts/train_fsdp.sh:28-29).
detect_gpus() {
  local n=""
  if [ "${DLT_FORCE_CPU:-0}" = "1" ]; then
    n=1
  elif command -v amd-smi >/dev/null 2>&1; then
    n=$(amd-smi list 2>/dev/null | grep -c '^GPU' || true)
  elif command -v rocm-smi >/dev/null 2>&1; then
    n=$(rocm-smi --showid 2>/dev/null | grep -cE '^GPU\[' || true)
  fi
  if [ -z "$n" ] || [ "$n" = "0" ]; then
    n=$(python3 -c 'import torch; print(torch.cuda.device_count())' 2>/dev/null || echo 1)
  fi
  [ -z "$n" ] || [ "$n" = "0" ] && n=1
  echo "$n"
}
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}   # dmabuf IPC for RCCL
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}
export NCCL_DEBUG=${NCCL_DEBUG:-WARN}
export NCCL_IB_DISABLE=${NCCL_IB_DISABLE:-1}     # one node: every peer is an xGMI link
# The remaining RCCL defaults (channel count, stream priority) are set per process by
# distributed_llm_trainer_amd.parallel.comm_env before the communicator is created.

# Build the gfx950 kernel libraries in-tree unless told not to (incremental: a no-op when
# every object is newer than its source).
maybe_build() {
  if [ "${DLT_SKIP_BUILD:-0}" != "1" ] && [ "${DLT_FORCE_CPU:-0}" != "1" ]; then
    python3 -m distributed_llm_trainer_amd.ops.build
  fi
}
