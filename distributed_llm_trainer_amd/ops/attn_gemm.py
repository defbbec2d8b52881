"""Attention for head_dims without a flash kernel (not 64 / 128), on native kernels only.

The reference accepts any ``hidden % heads == 0`` (``config.py:38-39``; its rotate_half
needs an even head_dim); the MFMA flash kernels exist for head_dim 64 and 128.  Routes,
first that applies -- none calls the PyTorch reference ops:

* head_dim < 128 (``PAD_FLASH``), any precision: the heads zero-padded to 64 / 128 and the
  flash kernels (16-bit MFMA, or fp32 VALU) run with the unpadded head_dim's score scale --
  the zero columns add nothing to q·k, P·V or the gradients, so this is exact; any length.
  The padding costs 128 / head_dim in FLOPs (head_dim 96: 1.33x) plus the layout copies
  (``k_relayout16`` / the fp32 relayout).
* else (head_dim > 128) attention as batched hipBLASLt GEMMs over the dense [S, S] scores
  around the row kernels of ``csrc/attn_gemm.hip`` (causal softmax / its backward, the same
  dropout keep bits as every other path; rows of any length):

  * 16-bit activations, head_dim % 16 == 0: 16-bit MFMA GEMMs (through the autotuned
    planner, ``ops/gemm.py``) with fp32 scores and dO·Vᵀ, P / Pd / dS rounded to 16 bits
    as operands -- the flash kernels' arithmetic; q / k / v / dO reach the head-major
    layout through ``k_relayout16`` and the gradient leaves through the 16-bit inverse-RoPE
    kernel.
  * otherwise: q / k / v widened to fp32 and ``hip_f32``'s fp32 formulation, the result
    narrowed back -- the arithmetic of the PyTorch reference attention
    (``reference.py:180-227``: fp32 scores, fp32 softmax).

  The score buffers are sized by B * nh * S^2; past ``GEMM_ROUTE_BYTES`` the route raises
  (loudly) instead of falling back.
* RoPE for a 16-bit head_dim the 16-bit kernel does not take (head_dim % 16): widened to
  fp32, rotated by the fp32 HIP kernel, rounded back once (``rope_*`` below).

A forward and its backward make the same choice (from the shapes and the dtype alone).
"""
from __future__ import annotations

import math
import os

import torch

from . import hip_f32

_HK = {torch.bfloat16: 0, torch.float16: 1}
PAD_FLASH = os.environ.get("DLT_ATTN_PAD", "1") != "0"


def pad_dim(dtype, hd: int):
    """The flash head_dim a head of ``hd`` is zero-padded to (16-bit: any hd; fp32: even
    hd -- its layout copy moves element pairs), or None."""
    if not PAD_FLASH or hd >= 128 or (dtype not in _HK and (dtype != torch.float32 or hd % 2)):
        return None
    return 64 if hd < 64 else 128


# the GEMM route's live score buffers (8-12 B per score) may take this much of the HBM
# (MI355X: 288 GB per GPU); beyond it the route raises instead of degrading silently
GEMM_ROUTE_BYTES = int(float(os.environ.get("DLT_ATTN_GEMM_GB", "96")) * (1 << 30))


def fits(B: int, nh: int, S: int, hd: int) -> bool:
    """Shapes the GEMM formulation takes (its live score buffers: 8-12 B per score)."""
    return hd % 2 == 0 and 3 * B * nh * S * S * 4 <= GEMM_ROUTE_BYTES


def _need_fit(B: int, nh: int, S: int, hd: int) -> None:
    if not fits(B, nh, S, hd):
        raise NotImplementedError(
            f"attention at head_dim {hd}, S {S}, B*nh {B * nh}: no flash kernel takes this head_dim and the GEMM "
            f"formulation's [S, S] score buffers ({3 * B * nh * S * S * 4 / 2**30:.1f} GiB) exceed "
            f"DLT_ATTN_GEMM_GB={GEMM_ROUTE_BYTES / 2**30:.0f}; use a smaller micro-batch or head_dim <= 128")


def use16(dtype, B: int, nh: int, S: int, hd: int) -> bool:
    """16-bit GEMMs (vs fp32 widening) for these operands."""
    from . import gemm
    return dtype in _HK and hd % 16 == 0 and gemm.available()


def _relayout16(src, sstr, dst, dstr, B, S, nh, hd, n, sts=0, dts=0):
    hip_f32._chk(hip_f32._lib().dlt_relayout16(hip_f32._p(src), hip_f32._p(dst), *sstr, *dstr, sts, dts, B, S, nh, hd, n,
                                               hip_f32._st()), "relayout16")


def _heads16(t, B, S, nh, hd, n):
    """The n [B*S, nh*hd] column blocks of t (row stride t.stride(0)) -> [n, B, nh, S, hd]."""
    H, ld = nh * hd, t.stride(0)
    out = torch.empty(n, B, nh, S, hd, dtype=t.dtype, device=t.device)
    _relayout16(t, (S * ld, ld, hd), out, (nh * S * hd, hd, S * hd), B, S, nh, hd, n, H, B * nh * S * hd)
    return out


def _pad16(src, sstr, B, S, nh, hd, Dp, n, sts):
    """n [b, s, h, d < hd] blocks of src -> zero-padded head-major [n, B, nh, S, Dp]."""
    out = torch.zeros(n, B, nh, S, Dp, dtype=src.dtype, device=src.device)
    _relayout16(src, sstr, out, (nh * S * Dp, Dp, S * Dp), B, S, nh, hd, n, sts, B * nh * S * Dp)
    return out


def _rows_padded(t, B, S, nh, hd, Dp):
    """[B*S, nh*hd] -> zero-padded [B*S, nh*Dp]."""
    out = torch.zeros(B * S, nh * Dp, dtype=t.dtype, device=t.device)
    _relayout16(t.contiguous(), (S * nh * hd, nh * hd, hd), out, (S * nh * Dp, nh * Dp, Dp), B, S, nh, hd, 1)
    return out


def _fwd_pad(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask, dt):
    from . import hip
    o_p, aux = hip.attention_fwd(q4p[0], q4p[1], q4p[2], p, key, True, store_mask=store_mask, mask=mask,
                                 scale=1.0 / math.sqrt(hd))
    H = nh * hd
    o = torch.empty(B * S, H, dtype=dt, device=q4p.device) if out is None else out
    if o.dtype != dt or not o.is_contiguous() or o.numel() != B * S * H:
        raise ValueError("attn_gemm: out must be a contiguous [B*S, H] tensor of the activation dtype")
    _relayout16(o_p, (S * nh * Dp, nh * Dp, Dp), o, (S * H, H, hd), B, S, nh, hd, 1)
    return o, aux


def _bwd_pad(q4p, o, do, aux, B, S, nh, hd, Dp, p, key):
    """(dq, dk, dv) [3, B, nh, S, hd] from the padded flash backward."""
    from . import hip
    dq, dk, dv = hip.attention_bwd(q4p[0], q4p[1], q4p[2], _rows_padded(o, B, S, nh, hd, Dp),
                                   _rows_padded(do, B, S, nh, hd, Dp), aux, p, key, scale=1.0 / math.sqrt(hd))
    g = torch.empty(3, B, nh, S, hd, dtype=dq.dtype, device=dq.device)
    for j, t in enumerate((dq, dk, dv)):
        _relayout16(t, (nh * S * Dp, Dp, S * Dp), g[j], (nh * S * hd, hd, S * hd), B, S, nh, hd, 1)
    return g


def _fwd16(q4, k4, v4, B, nh, S, hd, p, key, out, mask, store_mask):
    dt, dev = q4.dtype, q4.device
    H = nh * hd
    lse = torch.empty(B, nh, S, dtype=torch.float32, device=dev)
    mask, dscale = hip_f32._mask(B, nh, S, p, key, dev, mask)
    T, BH = hip_f32.attn_blocks(S), B * nh
    if T > 1:
        sc = torch.empty(B, nh, S, S, dtype=torch.float32, device=dev)
        hip_f32.blocked_scores(q4.reshape(BH, S, hd), k4.reshape(BH, S, hd), sc.view(BH, S, S), T, S, hd)
    else:
        sc = hip_f32._bmm("nt", q4, k4, torch.float32)
    pm = torch.empty(B, nh, S, S, dtype=dt, device=dev)
    hip_f32._chk(hip_f32._lib().dlt_attn16_softmax(hip_f32._p(sc), hip_f32._p(pm), hip_f32._p(lse), hip_f32._p(mask),
                                                   BH, S, 1.0 / math.sqrt(hd), dscale, S // T if T > 1 else 0,
                                                   _HK[dt], hip_f32._st()), "attn16_softmax")
    del sc
    if T > 1:
        o4 = torch.empty(B, nh, S, hd, dtype=dt, device=dev)
        hip_f32.blocked_rows(pm.view(BH, S, S), v4.reshape(BH, S, hd), o4.view(BH, S, hd), T, S, hd)
    else:
        o4 = hip_f32._bmm("nn", pm, v4)
    del pm
    o = torch.empty(B * S, H, dtype=dt, device=dev) if out is None else out
    if o.dtype != dt or not o.is_contiguous() or o.numel() != B * S * H:
        raise ValueError("attn_gemm: out must be a contiguous [B*S, H] tensor of the activation dtype")
    _relayout16(o4, (nh * S * hd, hd, S * hd), o, (S * H, H, hd), B, S, nh, hd, 1)
    return o, hip_f32._h().AttnAux((lse, mask if store_mask else None))


def _bwd16(q4, k4, v4, o, do, aux, B, nh, S, hd, p, key):
    """(dq, dk, dv) as contiguous [B, nh, S, hd] in the activation dtype."""
    dt, dev = q4.dtype, q4.device
    lse, mask = aux if isinstance(aux, tuple) else (aux, None)
    o, do = o.contiguous(), do.contiguous()
    mask, dscale = hip_f32._mask(B, nh, S, p, key, dev, mask)
    do4 = _heads16(do, B, S, nh, hd, 1)[0]
    T, BH = hip_f32.attn_blocks(S), B * nh
    q3, k3, v3, do3 = (t.reshape(BH, S, hd) for t in (q4, k4, v4, do4))
    if T > 1:
        sc = torch.empty(B, nh, S, S, dtype=torch.float32, device=dev)
        dp = torch.empty_like(sc)
        hip_f32.blocked_scores(q3, k3, sc.view(BH, S, S), T, S, hd)
        hip_f32.blocked_scores(do3, v3, dp.view(BH, S, S), T, S, hd)
    else:
        sc = hip_f32._bmm("nt", q4, k4, torch.float32)
        dp = hip_f32._bmm("nt", do4, v4, torch.float32)
    pd = torch.empty(B, nh, S, S, dtype=dt, device=dev)
    ds = torch.empty_like(pd)
    hip_f32._chk(hip_f32._lib().dlt_attn16_dsoftmax(
        hip_f32._p(sc), hip_f32._p(dp), hip_f32._p(pd), hip_f32._p(ds), hip_f32._p(lse), hip_f32._p(o), hip_f32._p(do),
        hip_f32._p(mask), B, nh, S, hd, 1.0 / math.sqrt(hd), dscale, S // T if T > 1 else 0, _HK[dt],
        hip_f32._st()), "attn16_dsoftmax")
    del sc, dp
    if T > 1:
        dq, dk, dv = (torch.empty(B, nh, S, hd, dtype=dt, device=dev) for _ in range(3))
        hip_f32.blocked_cols(pd.view(BH, S, S), do3, dv.view(BH, S, hd), T, S, hd)
        del pd
        hip_f32.blocked_rows(ds.view(BH, S, S), k3, dq.view(BH, S, hd), T, S, hd)
        hip_f32.blocked_cols(ds.view(BH, S, S), q3, dk.view(BH, S, hd), T, S, hd)
        return dq, dk, dv
    dv = hip_f32._bmm("tn", pd, do4)
    del pd
    return hip_f32._bmm("nn", ds, k4), hip_f32._bmm("tn", ds, q4), dv


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


# ------------------------------------------------------------- fp32 padded flash
def _pad32(ptrs, sstr, B, S, nh, hd, Dp, device):
    """len(ptrs) fp32 [b, s, h, d < hd] blocks (element at ptr + b*sstr[0] + s*sstr[1] +
    h*sstr[2] + d) -> zero-padded head-major [n, B, nh, S, Dp]."""
    out = torch.zeros(len(ptrs), B, nh, S, Dp, dtype=torch.float32, device=device)
    hip_f32._relayout(ptrs, sstr, B, S, nh, hd, device, [hip_f32._p(out[j]) for j in range(len(ptrs))],
                      (nh * S * Dp, Dp, S * Dp))
    return out


def _rows32(t, B, S, nh, hd, Dp):
    """fp32 [B*S, nh*hd] -> zero-padded [B*S, nh*Dp]."""
    t = t.contiguous()
    hip_f32._req32(t, "attn_pad32.rows")
    out = torch.zeros(B * S, nh * Dp, dtype=torch.float32, device=t.device)
    hip_f32._relayout([hip_f32._p(t)], (S * nh * hd, nh * hd, hd), B, S, nh, hd, t.device, [hip_f32._p(out)],
                      (S * nh * Dp, nh * Dp, Dp))
    return out


def _fwd_pad32(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask):
    dev = q4p.device
    hm = (nh * S * Dp, S * Dp, Dp)
    o_p, aux = hip_f32._fwd(hip_f32._p(q4p[0]), hip_f32._p(q4p[1]), hip_f32._p(q4p[2]), hm, B, nh, S, Dp, p, key, dev,
                            None, mask, store_mask, scale=1.0 / math.sqrt(hd))
    o = torch.empty(B * S, nh * hd, dtype=torch.float32, device=dev) if out is None else out
    hip_f32._req32(o, "attn_pad32.o", B * S * nh * hd)
    hip_f32._relayout([hip_f32._p(o_p)], (S * nh * Dp, nh * Dp, Dp), B, S, nh, hd, dev, [hip_f32._p(o)],
                      (S * nh * hd, nh * hd, hd))
    return o, aux


def _bwd_pad32(q4p, o, do, aux, B, S, nh, hd, Dp, p, key):
    """(dq, dk, dv) fp32 [3, B, nh, S, hd] from the padded fp32 flash backward."""
    dev = q4p.device
    hm = (nh * S * Dp, S * Dp, Dp)
    g_p = torch.empty(3, B, nh, S, Dp, dtype=torch.float32, device=dev)
    hip_f32._bwd(hip_f32._p(q4p[0]), hip_f32._p(q4p[1]), hip_f32._p(q4p[2]), hm, _rows32(o, B, S, nh, hd, Dp),
                 _rows32(do, B, S, nh, hd, Dp), aux, B, nh, S, Dp, p, key, dev,
                 tuple(hip_f32._p(g_p[j]) for j in range(3)), hm, scale=1.0 / math.sqrt(hd))
    g = torch.empty(3, B, nh, S, hd, dtype=torch.float32, device=dev)
    hip_f32._relayout([hip_f32._p(g_p[j]) for j in range(3)], (nh * S * Dp, Dp, S * Dp), B, S, nh, hd, dev,
                      [hip_f32._p(g[j]) for j in range(3)], (nh * S * hd, hd, S * hd))
    return g


# ------------------------------------------------------------------ RoPE (16-bit, hd % 16)
def rope_qk_inplace(qkv, B, S, nh, cos, sin):
    """RoPE on the q / k blocks of a 16-bit packed QKV whose head_dim the 16-bit kernel does
    not take: widened to fp32 (exact), rotated by the fp32 HIP kernel, rounded back once --
    the 16-bit kernel's arithmetic (fp32 rotation of the 16-bit values)."""
    w = qkv.float()
    hip_f32.rope_qk_inplace(w, B, S, nh, cos, sin)
    qkv.copy_(w)
    return qkv


def rope_qkv_fwd(qkv, B, S, nh, cos, sin):
    q, k, v = hip_f32.rope_qkv_fwd(qkv.float(), B, S, nh, cos, sin)
    return q.to(qkv.dtype), k.to(qkv.dtype), v.to(qkv.dtype)


def rope_qkv_bwd(dq, dk, dv, cos, sin, out=None):
    r = hip_f32.rope_qkv_bwd(dq.float(), dk.float(), dv.float(), cos, sin)
    return r.to(dk.dtype) if out is None else out.copy_(r)


def _rope_bwd(dq, dk, dv, cos, sin, out=None):
    """Inverse RoPE into the packed gradient on whichever HIP kernel takes the head_dim."""
    from . import hip
    hd = dk.shape[-1]
    if dk.dtype == torch.float32:
        return hip_f32.rope_qkv_bwd(dq, dk, dv, cos, sin, out=out)
    if hd % 16 == 0:
        return hip.rope_qkv_bwd(dq, dk, dv, cos, sin, out=out)
    return rope_qkv_bwd(dq, dk, dv, cos, sin, out=out)


# ----------------------------------------------------------------------- entry points
def attention_fwd_packed(qkv, B, S, nh, p, key, out=None, mask=None, store_mask=True):
    hd = qkv.shape[1] // (3 * nh)
    Dp = pad_dim(qkv.dtype, hd)
    H, ld = nh * hd, qkv.stride(0)
    if Dp and qkv.dtype == torch.float32:
        q4p = _pad32(hip_f32._packed_ptrs(qkv, 3, H), (S * ld, ld, hd), B, S, nh, hd, Dp, qkv.device)
        return _fwd_pad32(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask)
    if Dp:
        q4p = _pad16(qkv, (S * ld, ld, hd), B, S, nh, hd, Dp, 3, nh * hd)
        return _fwd_pad(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask, qkv.dtype)
    _need_fit(B, nh, S, hd)
    if use16(qkv.dtype, B, nh, S, hd):
        q4, k4, v4 = _heads16(qkv, B, S, nh, hd, 3)
        return _fwd16(q4, k4, v4, B, nh, S, hd, p, key, out, mask, store_mask)
    q4, k4, v4 = _heads32(qkv, B, S, nh, hd)
    o32 = out if out is not None and out.dtype == torch.float32 else None
    o32, aux = hip_f32._gemm_fwd(q4, k4, v4, B, nh, S, hd, p, key, qkv.device, o32, mask, store_mask)
    return _narrow(o32, qkv.dtype, out), aux


def attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=None):
    hd = qkv.shape[1] // (3 * nh)
    Dp = pad_dim(qkv.dtype, hd)
    H, ld = nh * hd, qkv.stride(0)
    if Dp and qkv.dtype == torch.float32:
        q4p = _pad32(hip_f32._packed_ptrs(qkv, 3, H), (S * ld, ld, hd), B, S, nh, hd, Dp, qkv.device)
        g = _bwd_pad32(q4p, o, do, aux, B, S, nh, hd, Dp, p, key)
        del q4p
        return _rope_bwd(g[0], g[1], g[2], cos, sin, out=out)
    if Dp:
        q4p = _pad16(qkv, (S * ld, ld, hd), B, S, nh, hd, Dp, 3, nh * hd)
        g = _bwd_pad(q4p, o, do, aux, B, S, nh, hd, Dp, p, key)
        del q4p
        return _rope_bwd(g[0], g[1], g[2], cos, sin, out=out)
    _need_fit(B, nh, S, hd)
    if use16(qkv.dtype, B, nh, S, hd):
        from . import hip
        q4, k4, v4 = _heads16(qkv, B, S, nh, hd, 3)
        dq, dk, dv = _bwd16(q4, k4, v4, o, do, aux, B, nh, S, hd, p, key)
        del q4, k4, v4
        return hip.rope_qkv_bwd(dq, dk, dv, cos, sin, out=out)
    q4, k4, v4 = _heads32(qkv, B, S, nh, hd)
    dq, dk, dv = hip_f32._gemm_bwd(q4, k4, v4, _f32(o), _f32(do), aux, B, nh, S, hd, p, key, qkv.device)
    del q4, k4, v4
    o32 = out if out is not None and out.dtype == torch.float32 else None
    return _narrow(hip_f32.rope_qkv_bwd(dq, dk, dv, cos, sin, out=o32), qkv.dtype, out)


def attention_fwd(q, k, v, p, key, causal=True, store_mask=True, out=None, mask=None):
    if not causal:
        raise NotImplementedError("only causal attention is implemented (the model is a causal LM)")
    B, nh, S, hd = q.shape
    Dp = pad_dim(q.dtype, hd)
    hm = (nh * S * hd, hd, S * hd)
    if Dp and q.dtype == torch.float32:
        ts = [t.contiguous() for t in (q, k, v)]
        q4p = _pad32([hip_f32._p(t) for t in ts], hm, B, S, nh, hd, Dp, q.device)
        return _fwd_pad32(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask)
    if Dp:
        q4p = torch.stack([_pad16(t.contiguous(), hm, B, S, nh, hd, Dp, 1, 0)[0] for t in (q, k, v)])
        return _fwd_pad(q4p, B, S, nh, hd, Dp, p, key, out, mask, store_mask, q.dtype)
    _need_fit(B, nh, S, hd)
    if use16(q.dtype, B, nh, S, hd):
        return _fwd16(q.contiguous(), k.contiguous(), v.contiguous(), B, nh, S, hd, p, key, out, mask, store_mask)
    o32 = out if out is not None and out.dtype == torch.float32 else None
    o32, aux = hip_f32._gemm_fwd(_f32(q), _f32(k), _f32(v), B, nh, S, hd, p, key, q.device, o32, mask, store_mask)
    return _narrow(o32, q.dtype, out), aux


def attention_bwd(q, k, v, o, do, aux, p, key, causal=True):
    B, nh, S, hd = q.shape
    Dp = pad_dim(q.dtype, hd)
    hm = (nh * S * hd, hd, S * hd)
    if Dp and q.dtype == torch.float32:
        ts = [t.contiguous() for t in (q, k, v)]
        q4p = _pad32([hip_f32._p(t) for t in ts], hm, B, S, nh, hd, Dp, q.device)
        return tuple(_bwd_pad32(q4p, o, do, aux, B, S, nh, hd, Dp, p, key).unbind(0))
    if Dp:
        q4p = torch.stack([_pad16(t.contiguous(), hm, B, S, nh, hd, Dp, 1, 0)[0] for t in (q, k, v)])
        return tuple(_bwd_pad(q4p, o, do, aux, B, S, nh, hd, Dp, p, key).unbind(0))
    _need_fit(B, nh, S, hd)
    if use16(q.dtype, B, nh, S, hd):
        return _bwd16(q.contiguous(), k.contiguous(), v.contiguous(), o, do, aux, B, nh, S, hd, p, key)
    g = hip_f32._gemm_bwd(_f32(q), _f32(k), _f32(v), _f32(o), _f32(do), aux, B, nh, S, hd, p, key, q.device)
    return tuple(t if t.dtype == q.dtype else t.to(q.dtype) for t in g)
