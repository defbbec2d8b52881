"""Training-side configuration dataclasses (field names/defaults = the reference).

* ``TrainingConfig``      -- ``ddp_trainer.py:34-63``
* ``FSDPTrainingConfig``  -- ``fsdp_trainer.py:78-93`` (exported as ``TrainingConfig``
  from ``training.fsdp_trainer`` for API parity)
* ``FSDPConfig``          -- ``fsdp_trainer.py:53-75``

Additions are appended after the reference fields with defaults that reproduce the
reference behaviour (e.g. ``seed``), or enable MI355X-specific knobs
(``bucket_cap_mb``, ``reduce_dtype``, ``hip_graphs``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass
class TrainingConfig:
    # Data
    batch_size: int = 8
    max_seq_len: int = 1024
    # Optimization
    learning_rate: float = 6e-4
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    grad_clip: float = 1.0
    # Schedule
    max_steps: int = 10000
    warmup_steps: int = 1000
    log_interval: int = 1
    eval_interval: int = 500
    save_interval: int = 1000
    # Mixed precision
    mixed_precision: str = "bf16"
    # Gradient accumulation
    gradient_accumulation_steps: int = 4
    # Checkpointing
    checkpoint_dir: str = "checkpoints"
    resume_from: Optional[str] = None
    # ---- additions (MI355X build)
    seed: int = 1234
    bucket_cap_mb: float = 64.0
    reduce_dtype: str = "fp32"         # gradient all-reduce wire dtype: fp32 | bf16
    lr_schedule_fix: bool = True       # set LR before the step + clamp cosine (Q5/Q6)
    adam_eps: float = 1e-8
    defer_wgrad: bool = True           # one weight-grad GEMM per layer per optimizer step
    # which weight gradients defer_wgrad defers: "all", or a comma list of qkv / o / gu / down
    # / head, or "none" (the others run in each micro-step chain's backward); --memory_lean: "none"
    defer_roles: str = "all"
    pipeline_micro_steps: bool = True  # overlap fwd(k+1) with bwd(k) on two HIP streams (engine path)
    # execute F consecutive micro-steps as one forward/backward chain of F*batch_size rows
    # (loss normalised per micro-step, so the gradient is the reference's GA average);
    # 0 = auto (GPU engine: largest F with F*batch_size*seq <= 16384 tokens and >= 2
    # chains left to pipeline), 1 = off
    micro_step_fusion: int = 0
    # --memory_first: the reference's per-GPU memory (8.2 GB at micro-batch 8) over speed --
    # no weight gradient deferred (defer_roles "none", chunked lm_head), micro-steps run
    # unfused (micro_step_fusion 0 -> 1), the SwiGLU output rewritten by the backward
    # instead of kept (engine s_refill); profiles/r6_memory.md
    memory_first: bool = False
    # engine path: record the optimizer step and apply it unit by unit where the next
    # forward first needs each unit ("inline": on that chain's stream; "stream": on a
    # stream of its own; "off": the reference's end-of-step update, weights final when
    # train_step returns).  Readers outside a forward flush it (save, state_dict, eval):
    # DistributedTrainer.flush_optimizer.  See training/optim.py LazyStep.
    lazy_optimizer: str = "inline"


@dataclass
class FSDPTrainingConfig:
    batch_size: int = 4
    max_seq_len: int = 1024
    learning_rate: float = 3e-4
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    grad_clip: float = 1.0
    max_steps: int = 10000
    warmup_steps: int = 1000
    log_interval: int = 10
    save_interval: int = 1000
    gradient_accumulation_steps: int = 8
    checkpoint_dir: str = "checkpoints_fsdp"
    # ---- additions
    resume_from: Optional[str] = None
    seed: int = 1234
    lr_schedule_fix: bool = True
    adam_eps: float = 1e-8
    eval_interval: int = 500
    pipeline_micro_steps: bool = True  # overlap fwd(k+1) with bwd(k) on two HIP streams
    # F micro-steps per executed chain, as in TrainingConfig (0 = auto, 1 = off); the
    # per-micro-step reduce-scatter (Q15 parity) then runs once per chain -- the same sum
    micro_step_fusion: int = 0


@dataclass
class FSDPConfig:
    sharding_strategy: str = "FULL_SHARD"     # FULL_SHARD | SHARD_GRAD_OP | NO_SHARD | HYBRID_SHARD
    cpu_offload: bool = False
    mixed_precision: str = "bf16"             # bf16 | fp16 | fp32
    backward_prefetch: str = "BACKWARD_PRE"   # BACKWARD_PRE | BACKWARD_POST | NONE
    activation_checkpointing: bool = True
    limit_all_gathers: bool = True
    # ---- additions
    reduce_dtype: str = "bf16"                # reduce-scatter wire dtype (reference: bf16)
    sync_every_micro_step: bool = True        # reference reduce-scatters every micro-step (Q15)
