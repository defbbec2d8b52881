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


def for_device(device) -> types.SimpleNamespace:
    dev = torch.device(device)
    if dev.type == "cuda":
        if os.environ.get("DLT_ALLOW_REFERENCE_ON_GPU") == "1":
            return _namespace(reference, "reference")
        return hip_ops()
    return CPU_OPS
