"""MI355X-native distributed GPT pre-training engine.

Same capabilities and user-facing surface as zhc180/distributed-llm-trainer
(DDP / FSDP trainers, LLaMA-style "GPT-2" presets, checkpoint format, data loaders,
inference), rebuilt around hand-written HIP/CDNA4 kernels (``ops``), a fused
forward/backward executor (``models.engine``) and RCCL-based DDP/FSDP runtimes
(``parallel``).
"""
__version__ = "0.1.0"
