"""Fused ops: HIP/CDNA4 kernels on GPU, plain-PyTorch references on CPU.

``for_device(device)`` returns a namespace with the same functions for either
backend.  On a CUDA(HIP) device the HIP library is mandatory: there is no silent
fallback to eager PyTorch (set ``DLT_ALLOW_REFERENCE_ON_GPU=1`` only for debugging).
"""
from __future__ import annotations

import os
import types

import torch

from . import reference, rng

_FUNCS = ("rope_tables", "embedding_fwd", "embedding_bwd", "add_dropout_rmsnorm_fwd", "rmsnorm_bwd",
          "rope_qkv_fwd", "rope_qkv_bwd", "attention_fwd", "attention_bwd", "swiglu_fwd", "swiglu_bwd",
          "cross_entropy_fwd_bwd", "scale_bf16", "rope_qk_inplace", "attention_fwd_packed",
          "attention_bwd_packed")


def _namespace(mod, name):
    ns = types.SimpleNamespace(backend=name)
    for f in _FUNCS:
        setattr(ns, f, getattr(mod, f))
    return ns


CPU_OPS = _namespace(reference, "reference")


# HIP-only: the fused one-token decode step (eval/decode.py DecodeGraph)
_HIP_ONLY = ("dec_norm_qkv", "dec_attn", "dec_gemv_res", "dec_norm_gu", "dec_norm_head", "dec_sample", "dec_advance", "dec_sample_workspace",
             "DECODE_BATCHES")


def hip_ops():
    from . import hip
    hip.lib()  # loud failure if the library is missing
    ns = _namespace(hip, "hip")
    for f in _HIP_ONLY:
        setattr(ns, f, getattr(hip, f))
    return ns


# the attention-side ops whose HIP kernels are specialised for head_dims 64 / 128
_ATTN_FUNCS = ("rope_qkv_fwd", "rope_qkv_bwd", "attention_fwd", "attention_bwd", "rope_qk_inplace",
               "attention_fwd_packed", "attention_bwd_packed")


def for_device(device, head_dim: int = 64, act_dtype=torch.bfloat16) -> types.SimpleNamespace:
    """Op namespace for ``device``.  On the GPU every op is a HIP kernel: bf16 / fp16
    activations on the 16-bit kernels, fp32 (``--mixed_precision fp32``) on the fp32
    kernels (``csrc/fp32.hip``; the ``hip`` wrappers dispatch on the tensor dtype).  The
    flash attention kernels take head_dim 64 and 128 in every precision; a model with
    another head_dim (the reference allows any ``hidden % heads == 0``, ``config.py:38-39``,
    with an even head_dim for its rotate_half) runs attention on native kernels
    (``ops/attn_gemm.py``, ``attn_backend == "gemm"``, with a one-time warning): heads under
    128 zero-padded onto the flash kernels, wider ones as GEMMs over the dense scores around
    HIP row kernels.  Its RoPE runs on the 16-bit HIP kernel when that takes the head_dim
    (% 16), else on the fp32 HIP kernel over the widened values.  No op falls back to
    PyTorch reference ops on the GPU."""
    dev = torch.device(device)
    if dev.type == "cuda":
        if os.environ.get("DLT_ALLOW_REFERENCE_ON_GPU") == "1":
            return _namespace(reference, "reference")
        ns = hip_ops()
        ns.attn_backend = "hip"
        from .hip import ATTN_HEAD_DIMS
        from .hip_f32 import ATTN_HEAD_DIMS as F32_HEAD_DIMS
        native_hd = F32_HEAD_DIMS if act_dtype == torch.float32 else ATTN_HEAD_DIMS
        if head_dim not in native_hd:
            import warnings

            from . import attn_gemm
            if head_dim % 2:
                raise NotImplementedError(f"head_dim {head_dim}: RoPE (rotate_half) needs an even head_dim")
            rope16 = act_dtype == torch.float32 or head_dim % 16 == 0
            route = ("zero-padded onto the flash kernels" if attn_gemm.pad_dim(act_dtype, head_dim)
                     else "batched GEMMs + HIP row kernels")
            warnings.warn(f"head_dim {head_dim}: the HIP flash attention kernels take head_dim {native_hd}; attention "
                          f"runs {route} for this model (RoPE: "
                          f"{'HIP kernel' if rope16 else 'fp32 HIP kernel on widened values'})")
            for f in _ATTN_FUNCS:
                if not f.startswith("rope") or not rope16:
                    setattr(ns, f, getattr(attn_gemm, f))
            ns.attn_backend = "gemm"
        return ns
    return CPU_OPS
