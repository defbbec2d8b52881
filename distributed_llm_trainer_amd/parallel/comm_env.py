"""RCCL / HIP environment for one node of MI355X GPUs on a point-to-point xGMI mesh.

RCCL reads its tuning variables once, when a communicator is created, so these are set
per process *before* ``torch.distributed.init_process_group`` (``training/common.py``
``setup_distributed`` calls :func:`apply`).  A variable the user already exported is never
overridden; ``DLT_COMM_ENV=0`` skips the module entirely.  The reference sets only
``NCCL_DEBUG`` / ``NCCL_IB_DISABLE`` in its launcher (``scripts/train_fsdp.sh:28-29``) and
leaves NCCL's NVSwitch-oriented defaults alone (``ddp_trainer.py:167-172``).

Why these values, for 8 MI355X with 7 xGMI links per GPU (~153 GB/s per link) and no switch:

* ``NCCL_IB_DISABLE=1`` (single node only: every peer is one xGMI hop away) -- RCCL would
  otherwise probe the NICs and may route a ring through them.
* ``NCCL_MIN_NCHANNELS=32`` -- a channel is one ring and one workgroup of the collective
  kernel.  On a switchless mesh a ring only loads the two links it uses, so the bandwidth
  of a large all-reduce grows with the number of rings RCCL lays over the 7 links; one
  workgroup moves ~20-30 GB/s, so 7 links x ~64 GB/s per direction need >= 16-24 of them.
  The DDP runtime's buckets are 64 MB (small: 607 MB of fp32 gradients, ~10 buckets per
  step) and the FSDP units 28-118 MB: bandwidth-bound messages, never latency-bound.  32
  channels cost 32 of 256 CUs only while a bucket is on the wire (DDP small at W = 8:
  ~3.5 ms of a 40 ms step overlapped with the backward, ~1 % of the step's CU-time), while
  the exposed tail -- the head bucket after the embedding backward -- is pure bandwidth.
  Only a floor is set: RCCL may still pick more for its own topology model.
* ``TORCH_NCCL_HIGH_PRIORITY=1`` -- the collectives' stream is created at high priority.
  The engine keeps two compute streams saturated with large kernels; a bucket's RCCL
  kernel then takes the next free CUs instead of queueing behind the compute streams'
  backlog (neutral on one forced-collective rank, ``tools/ab/README.md``; the multi-rank
  benefit is unmeasured here -- no 8-GPU node is available to this build).
* ``TORCH_NCCL_AVOID_RECORD_STREAMS=1`` -- the DDP buckets are enqueued from the engine's
  weight-gradient stream and waited for explicitly (``DDPRuntime.finish``), so the
  caching allocator needs no cross-stream ``record_stream`` bookkeeping per collective.
* ``TORCH_NCCL_ASYNC_ERROR_HANDLING=3`` -- a failed or timed-out collective
  (``DLT_PG_TIMEOUT``) tears the process group down and raises instead of hanging the
  step (SURVEY §5.3 failure detection).
* ``HSA_ENABLE_IPC_MODE_LEGACY=0`` -- this host driver supports dmabuf IPC only; RCCL's
  peer mappings fail with ``hipIpcGetMemHandle: invalid argument`` without it.
* ``NCCL_DEBUG=WARN`` -- the reference launcher's level.

Protocols (LL / LL128 / Simple) are left to RCCL's size-based choice: the 4-byte loss
and found-inf all-reduces want LL, the buckets Simple.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

# variable -> value; set only when absent from the environment
COMMON: Dict[str, str] = {
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
    "NCCL_DEBUG": "WARN",
    "NCCL_MIN_NCHANNELS": "32",
    "TORCH_NCCL_HIGH_PRIORITY": "1",
    "TORCH_NCCL_AVOID_RECORD_STREAMS": "1",
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "3",
}
SINGLE_NODE: Dict[str, str] = {
    "NCCL_IB_DISABLE": "1",
}

applied: Dict[str, str] = {}  # what the last apply() set (for logs and tests)


def single_node(world_size: Optional[int] = None, local_world_size: Optional[int] = None) -> bool:
    """All ranks on this node (torchrun exports LOCAL_WORLD_SIZE and WORLD_SIZE)."""
    w = world_size if world_size is not None else int(os.environ.get("WORLD_SIZE", "1"))
    lw = local_world_size if local_world_size is not None else int(os.environ.get("LOCAL_WORLD_SIZE", str(w)))
    return lw >= w


def apply(world_size: Optional[int] = None, local_world_size: Optional[int] = None) -> Dict[str, str]:
    """Export the defaults above that the environment does not set yet; returns what was
    set.  Must run before the first communicator is created."""
    applied.clear()
    if os.environ.get("DLT_COMM_ENV", "1") == "0":
        return dict(applied)
    want = dict(COMMON)
    if single_node(world_size, local_world_size):
        want.update(SINGLE_NODE)
    for k, v in want.items():
        if k not in os.environ:
            os.environ[k] = v
            applied[k] = v
    return dict(applied)
