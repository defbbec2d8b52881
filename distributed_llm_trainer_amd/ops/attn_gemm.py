"""Attention for head_dims without a flash kernel (not 64 / 128), on native kernels.

The reference accepts any ``hidden % heads == 0`` (``config.py:38-39``); the MFMA flash
kernels exist for head_dim 64 and 128.  Any other head_dim runs the GEMM formulation of
``hip_f32``: q / k / v widened to fp32, the six S x S x hd products as batched hipBLASLt
fp32 GEMMs around the ``k_f32_attn_softmax`` / ``_dsoftmax`` row kernels (same dropout
keep bits as every other path), the result narrowed back to the activation dtype.  That
is the arithmetic of the PyTorch reference attention (``reference.py:180-227``: fp32
scores, fp32 softmax), with HIP kernels in place of the ATen masking / softmax / dropout
over the [S, S] matrix.  Rows longer than 4096 keys, or score buffers over
``hip_f32.GEMM_ATTN_BYTES``, use the reference ops (the same choice is made for a
forward and its backward, from the shapes alone).
"""
from __future__ import annotations

import torch

from . import hip_f32, reference


def fits(B: int, nh: int, S: int, hd: int) -> bool:
    return hd % 2 == 0 and hd <= 256 and S <= 4096 and 2 * B * nh * S * S * 4 <= hip_f32.GEMM_ATTN_BYTES


def _f32(t: torch.Tensor) -> torch.Tensor:
    return (t if t.dtype == torch.float32 else t.float()).contiguous()


def _narrow(o32: torch.Tensor, dtype, out):
    if out is None:
        return o32 if dtype == torch.float32 else o32.to(dtype)
    if out.data_ptr() != o32.data_ptr():
        out.copy_(o32)
    return out


def _heads32(qkv, B, S, nh, hd):
    q32 = _f32(qkv)
    H = nh * hd
    return hip_f32._relayout(hip_f32._packed_ptrs(q32, 3, H), (S * 3 * H, 3 * H, hd), B, S, nh, hd, qkv.device)


def attention_fwd_packed(qkv, B, S, nh, p, key, out=None, mask=None, store_mask=True):
    hd = qkv.shape[1] // (3 * nh)
    if not fits(B, nh, S, hd):
        return reference.attention_fwd_packed(qkv, B, S, nh, p, key, out=out, mask=mask)
    q4, k4, v4 = _heads32(qkv, B, S, nh, hd)
    o32 = out if out is not None and out.dtype == torch.float32 else None
    o32, aux = hip_f32._gemm_fwd(q4, k4, v4, B, nh, S, hd, p, key, qkv.device, o32, mask, store_mask)
    return _narrow(o32, qkv.dtype, out), aux


def attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=None):
    hd = qkv.shape[1] // (3 * nh)
    if not fits(B, nh, S, hd):
        return reference.attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=out)
    q4, k4, v4 = _heads32(qkv, B, S, nh, hd)
    dq, dk, dv = hip_f32._gemm_bwd(q4, k4, v4, _f32(o), _f32(do), aux, B, nh, S, hd, p, key, qkv.device)
    del q4, k4, v4
    o32 = out if out is not None and out.dtype == torch.float32 else None
    return _narrow(hip_f32.rope_qkv_bwd(dq, dk, dv, cos, sin, out=o32), qkv.dtype, out)


def attention_fwd(q, k, v, p, key, causal=True, store_mask=True, out=None, mask=None):
    if not causal:
        raise NotImplementedError("only causal attention is implemented (the model is a causal LM)")
    B, nh, S, hd = q.shape
    if not fits(B, nh, S, hd):
        return reference.attention_fwd(q, k, v, p, key, causal, out=out)
    o32 = out if out is not None and out.dtype == torch.float32 else None
    o32, aux = hip_f32._gemm_fwd(_f32(q), _f32(k), _f32(v), B, nh, S, hd, p, key, q.device, o32, mask, store_mask)
    return _narrow(o32, q.dtype, out), aux


def attention_bwd(q, k, v, o, do, aux, p, key, causal=True):
    B, nh, S, hd = q.shape
    if not fits(B, nh, S, hd):
        return reference.attention_bwd(q, k, v, o, do, aux, p, key, causal)
    g = hip_f32._gemm_bwd(_f32(q), _f32(k), _f32(v), _f32(o), _f32(do), aux, B, nh, S, hd, p, key, q.device)
    return tuple(t if t.dtype == q.dtype else t.to(q.dtype) for t in g)
