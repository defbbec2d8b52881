"""Tracing hooks: roctx ranges (visible in rocprofv3 --marker-trace / rocprof
timelines) and an optional torch.profiler trace (``--profile DIR``).

The reference has no instrumentation beyond wall-clock prints."""
from __future__ import annotations

import os

import torch

_ENABLED = os.environ.get("DLT_ROCTX", "0") == "1"


def range_push(name: str) -> None:
    if _ENABLED and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds


def range_pop() -> None:
    if _ENABLED and torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


class Profiler:
    """torch.profiler with CPU + GPU (roctracer) activity, 2 warmup + 3 active steps."""

    def __init__(self, out_dir, enabled: bool = True, wait: int = 1, warmup: int = 2, active: int = 3):
        self.prof = None
        if enabled and out_dir:
            os.makedirs(out_dir, exist_ok=True)
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(
                activities=acts, schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=active),
                on_trace_ready=torch.profiler.tensorboard_trace_handler(out_dir), record_shapes=True)
            self.prof.__enter__()

    def step(self) -> None:
        if self.prof is not None:
            self.prof.step()

    def close(self) -> None:
        if self.prof is not None:
            self.prof.__exit__(None, None, None)
            self.prof = None
