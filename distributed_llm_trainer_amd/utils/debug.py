"""Debug / failure-injection hooks (SURVEY §5.2, §5.3 -- absent in the reference).

* ``replica_checksum`` / ``check_replicas``: bit-exact checksum of a rank's flat
  parameter buffer, all-gathered and compared.  DDP replicas must stay identical; a
  mismatch (a missed all-reduce, a non-deterministic kernel feeding the optimizer, a
  rank that skipped a step) is reported with the diverging ranks instead of silently
  training N different models.  Enabled in the trainers by ``DLT_CHECK_REPLICAS=N``
  (check after init and every N optimizer steps).
* ``maybe_inject_fault``: ``DLT_FAULT_INJECT="<step>[:<rank>]"`` kills the process
  (exit code 17) when that optimizer step is reached -- the hook the resume tests use
  to prove that ``--resume_from`` reproduces an uninterrupted run exactly.
"""
from __future__ import annotations

import os
import sys
from typing import Optional

import torch
import torch.distributed as dist

FAULT_EXIT_CODE = 17


def replica_checksum(flat: torch.Tensor) -> torch.Tensor:
    """Order-independent exact checksum: int64 sums of the raw 32-bit words (two
    different weightings so swapped values are caught too)."""
    w = flat.detach().contiguous().view(torch.int32).to(torch.int64)
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([w.sum(), (w * idx).sum()])


def check_replicas(flat: torch.Tensor, group=None, what: str = "parameters") -> None:
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    cs = replica_checksum(flat)
    if dist.get_backend(group) == "nccl" and not cs.is_cuda:
        cs = cs.cuda()
    out = [torch.empty_like(cs) for _ in range(world)]
    dist.all_gather(out, cs, group=group)
    ref = out[0]
    bad = [r for r, c in enumerate(out) if not torch.equal(c, ref)]
    if bad:
        raise RuntimeError(f"replica divergence: {what} of ranks {bad} differ from rank 0 "
                           f"(checksums {[tuple(c.tolist()) for c in out]})")


def replica_check_interval() -> int:
    return int(os.environ.get("DLT_CHECK_REPLICAS", "0") or 0)


def maybe_inject_fault(step: int, rank: int) -> None:
    spec: Optional[str] = os.environ.get("DLT_FAULT_INJECT")
    if not spec:
        return
    parts = spec.split(":")
    at = int(parts[0])
    who = int(parts[1]) if len(parts) > 1 else None
    if step == at and (who is None or who == rank):
        print(f"[dlt] injected fault at step {step} on rank {rank}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(FAULT_EXIT_CODE)
