"""MI355X-native distributed GPT pre-training engine.

Same capabilities and user-facing surface as zhc180/distributed-llm-trainer
(DDP / FSDP trainers, LLaMA-style "GPT-2" presets, checkpoint format, data loaders,
inference), rebuilt around hand-written HIP/CDNA4 kernels (``ops``), a fused
forward/backward executor (``models.engine``) and RCCL-based DDP/FSDP runtimes
(``parallel``).
"""
import os as _os

__version__ = "0.1.0"


def _ensure_hw_queues() -> None:
    """Give the HIP runtime enough hardware queues for the engine's streams.

    HIP maps streams round-robin onto ``GPU_MAX_HW_QUEUES`` hardware queues (4 by
    default).  An RCCL communicator creates streams of its own, after which the engine's
    two compute streams (pipelined micro-step chains, weight-gradient GEMMs) can share
    one hardware queue and run serialised: measured on one MI355X with an idle 1-rank
    RCCL communicator, 43.3 -> 45.0-47.1 ms per optimizer step (kernel-busy 161 % -> 98 %
    of the span), back to 43.1-43.4 ms with 8 or 16 queues (profiles/r2_hw_queues.md).
    The runtime reads the variable once, when it initialises (first GPU call), so this
    runs at import.  ``DLT_HW_QUEUES`` sets the minimum (0 = leave the variable alone).
    """
    try:
        want = int(_os.environ.get("DLT_HW_QUEUES", "16"))
    except ValueError:
        want = 16
    try:
        have = int(_os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        have = 4
    if want > 0 and have < want:
        new = str(min(want, 32))
        _os.environ["GPU_MAX_HW_QUEUES"] = new
        # tell the host application once (rank 0 only) that its HIP runtime config changed
        if _os.environ.get("RANK", "0") == "0" and _os.environ.get("DLT_QUIET", "0") != "1":
            import sys
            late = False
            torch = sys.modules.get("torch")
            if torch is not None:
                try:
                    late = bool(torch.cuda.is_initialized())
                except Exception:  # pragma: no cover
                    late = False
            msg = (f"[distributed_llm_trainer_amd] GPU_MAX_HW_QUEUES {have} -> {new} "
                   "(engine streams; DLT_HW_QUEUES=0 keeps the runtime default)")
            if late:
                msg += ("; WARNING: the HIP runtime is already initialised in this process, "
                        "so the new value has no effect (import this package before the first GPU call)")
            print(msg, file=sys.stderr, flush=True)


_ensure_hw_queues()
