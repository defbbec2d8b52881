"""Pieces shared by the DDP and FSDP trainers: process-group bootstrap, device
selection, seeding, LR schedule, memory stats and the YAML/CLI config merge."""
from __future__ import annotations

import datetime
import math
import os
import random
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist


def setup_distributed(require: bool = False, timeout_s: Optional[float] = None):
    """Returns (distributed, rank, world_size, local_rank).

    Backend: "nccl" (= RCCL on ROCm) when a GPU is present, else "gloo" (CPU tests /
    the plumbing config).  ``DLT_PG_TIMEOUT`` (seconds) bounds every collective so a
    dead rank surfaces as an error instead of a hang.
    """
    distributed = dist.is_initialized() or "RANK" in os.environ or require
    if distributed and not dist.is_initialized():
        # RCCL's xGMI defaults, read when the communicator is created (parallel/comm_env.py)
        from ..parallel import comm_env
        comm_env.apply()
        backend = os.environ.get("DLT_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        t = timeout_s or float(os.environ.get("DLT_PG_TIMEOUT", "1800"))
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=t))
        if backend == "nccl" and torch.cuda.is_available():
            lr = _device_index(int(os.environ.get("LOCAL_RANK", 0)))
            torch.cuda.set_device(lr)
            kw["device_id"] = torch.device(f"cuda:{lr}")
        dist.init_process_group(**kw)
    if distributed:
        return True, dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", 0))
    return False, 0, 1, 0


def _device_index(local_rank: int) -> int:
    """GPU of a local rank.  One rank per GPU; ``DLT_SHARE_GPU=1`` folds ranks onto the
    visible GPUs (local_rank mod count) -- only for rehearsing multi-rank code paths
    with the gloo backend on a 1-GPU box (RCCL itself rejects two ranks per GPU)."""
    if os.environ.get("DLT_SHARE_GPU") == "1":
        return local_rank % max(1, torch.cuda.device_count())
    return local_rank


def select_device(local_rank: int) -> torch.device:
    if torch.cuda.is_available() and os.environ.get("DLT_FORCE_CPU") != "1":
        d = torch.device(f"cuda:{_device_index(local_rank)}")
        torch.cuda.set_device(d)
        return d
    return torch.device("cpu")


def seed_all(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


def cosine_lr(step: int, lr: float, warmup: int, max_steps: int, clamp: bool = True) -> float:
    """Linear warmup then cosine to 0.1*lr (``ddp_trainer.py:262-271``).  The DDP
    reference does not clamp the decay ratio (LR rises again after max_steps, Q6);
    ``clamp=True`` applies the FSDP trainer's clamp (``fsdp_trainer.py:354``)."""
    if step < warmup:
        return lr * (step / warmup)
    denom = max(1, max_steps - warmup)
    ratio = (step - warmup) / denom
    if clamp:
        ratio = min(ratio, 1.0)
    coeff = 0.5 * (1.0 + math.cos(math.pi * ratio))
    min_lr = 0.1 * lr
    return min_lr + coeff * (lr - min_lr)


def memory_stats(device) -> dict:
    """GB (1e9), like ``fsdp_trainer.py:496-505``."""
    if torch.device(device).type != "cuda":
        return {"allocated_gb": 0.0, "reserved_gb": 0.0, "max_allocated_gb": 0.0}
    return {"allocated_gb": torch.cuda.memory_allocated(device) / 1e9,
            "reserved_gb": torch.cuda.memory_reserved(device) / 1e9,
            "max_allocated_gb": torch.cuda.max_memory_allocated(device) / 1e9}


FUSE_TOKENS = 16384  # rows of a fused micro-step chain (GEMM M) the auto rule aims for


def micro_step_fusion(requested: int, GA: int, micro_bs: int, seq_len: int, gpu_engine: bool) -> int:
    """Number of micro-steps executed as one chain (a divisor of GA).

    Measured on one MI355X (small, micro-batch 8 x GA 4, seq 1024): chains of 16
    sequences (F = 2, GEMM M = 16384) run 43.2 ms per optimizer step vs 46.1 ms for
    four 8-sequence chains -- the projection GEMMs reach ~1 PF/s at M >= 16384 (vs
    0.4-0.9 at 8192) and two chains still pipeline (profiles/r2_microbatch_ab.md).
    ``requested`` > 0 forces F (must divide GA); 0 = auto (GPU engine only)."""
    if requested > 0:
        if GA % requested:
            raise ValueError(f"micro_step_fusion={requested} must divide gradient_accumulation_steps={GA}")
        return requested
    if not gpu_engine or GA < 2:
        return 1
    best = 1
    for f in range(1, GA + 1):
        if GA % f == 0 and f * micro_bs * seq_len <= FUSE_TOKENS and GA // f >= 2:
            best = f
    return best


def gemm_plan_hook() -> None:
    """After a step: write the GEMM plan file once if ``DLT_GEMM_PLAN`` asks for one
    (``ops/gemm.py`` ``maybe_save_plan``; a no-op without the planner)."""
    if not (os.environ.get("DLT_GEMM_PLAN") or os.environ.get("DLT_GEMM_PLAN_OUT")):
        return
    from ..ops import gemm
    gemm.maybe_save_plan()


def global_mean_loss(total: torch.Tensor, world: int) -> float:
    """Mean of the ranks' step losses (the reference logs rank 0's local
    loss; that line is kept, the metrics JSONL also gets this).  A collective: every
    rank must call it on the same steps."""
    t = total.detach().reshape(1).float().clone()
    dist.all_reduce(t)
    return float(t.item()) / world


def unwrap_batch(batch):
    if isinstance(batch, dict):
        return batch["input_ids"]
    if isinstance(batch, (list, tuple)):
        return batch[0]
    return batch
