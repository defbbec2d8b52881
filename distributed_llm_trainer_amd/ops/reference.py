"""Plain-PyTorch (fp32-accumulating) reference implementations of every fused op.

These define the numerical contract of the HIP kernels in ``ops/csrc`` and are the
CPU execution path of the engine (``models/engine.py``), which lets the hand-written
forward/backward of the whole model be validated against autograd on CPU.

Reference semantics being reproduced (``/root/reference/src/models/gpt.py``):
RMSNorm ``:66-67`` (eps 1e-6, fp32 math), RoPE ``:82-98,116-118,144-147`` (NeoX
half-split), attention ``:199-240`` (causal, scale 1/sqrt(hd), fp32 softmax, dropout on
probabilities), SwiGLU ``:278-282``, shifted cross-entropy ``:449-453``
(ignore_index -100, mean over valid targets).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import rng

IGNORE_INDEX = -100


# ----------------------------------------------------------------- embedding
def embedding_fwd(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    return weight.index_select(0, ids.reshape(-1)).float()


def embedding_bwd(ids: torch.Tensor, dout: torch.Tensor, dweight: torch.Tensor) -> None:
    dweight.index_add_(0, ids.reshape(-1), dout.reshape(-1, dout.shape[-1]).to(dweight.dtype))


# --------------------------------------------------- residual add + dropout + RMSNorm
def dropout_apply(x: torch.Tensor, key: int, p: float) -> torch.Tensor:
    if p <= 0.0:
        return x
    keep = rng.keep_mask(x.shape, key, p, device=x.device)
    return torch.where(keep, x / (1.0 - p), torch.zeros((), dtype=x.dtype, device=x.device))


def add_dropout_rmsnorm_fwd(resid: Optional[torch.Tensor], delta: Optional[torch.Tensor],
                            weight: torch.Tensor, eps: float, p: float, key: int,
                            out_dtype=torch.bfloat16, y_out=None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """x = resid + dropout(delta);  y = x * rsqrt(mean(x^2)+eps) * w.

    Returns (x fp32, y out_dtype, rstd fp32[M]).  ``resid``/``delta`` may be None.
    """
    if resid is None:
        x = dropout_apply(delta.float(), key, p)
    elif delta is None:
        x = resid.float()
    else:
        x = resid.float() + dropout_apply(delta.float(), key, p)
    rstd = torch.rsqrt(x.pow(2).mean(dim=-1, keepdim=True) + eps)
    y = (x * rstd * weight.float()).to(out_dtype)
    if y_out is not None:
        y_out.copy_(y)
        y = y_out
    return x, y, rstd.squeeze(-1)


def rmsnorm_bwd(dy: torch.Tensor, x: torch.Tensor, rstd: torch.Tensor, weight: torch.Tensor,
                dres: Optional[torch.Tensor], dweight: torch.Tensor, p_prev: float, key_prev: int,
                dy_scale: Optional[torch.Tensor] = None,
                want_ddelta: bool = True, ddelta_out=None, dy_mul: float = 1.0) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Backward of add_dropout_rmsnorm.

    dx = dres + J_rmsnorm^T dy ; ddelta = dropout_bwd(dx) (grad for the delta that was
    added with dropout key ``key_prev``).  ``dweight`` (fp32) is accumulated in place.
    ``dy_scale`` (0-dim tensor) multiplies ``dy`` first (used for the loss scale).
    """
    out_dt = dy.dtype
    dy = dy.float()
    if dy_scale is not None:
        dy = dy * dy_scale.float()
    if dy_mul != 1.0:
        dy = dy * dy_mul
    r = rstd.float().unsqueeze(-1)
    xh = x.float() * r
    w = weight.float()
    dweight += (dy * xh).sum(dim=0).to(dweight.dtype)
    g = dy * w
    h = x.shape[-1]
    dx = r * (g - xh * (g * xh).sum(dim=-1, keepdim=True) / h)
    if dres is not None:
        dx = dx + dres.float()
    ddelta = None
    if want_ddelta:
        ddelta = dropout_apply(dx, key_prev, p_prev).to(out_dt)
        if ddelta_out is not None:
            ddelta_out.copy_(ddelta)
            ddelta = ddelta_out
    return dx, ddelta


# ------------------------------------------------------------------- RoPE
def rope_tables(head_dim: int, seq_len: int, base: float = 10000.0, device=None):
    """cos/sin [S, hd/2] fp32 (the reference caches the duplicated [S, hd] form)."""
    inv_freq = 1.0 / (base ** (torch.arange(0, head_dim, 2, device=device).float() / head_dim))
    t = torch.arange(seq_len, device=device).float()
    freqs = torch.outer(t, inv_freq)
    return freqs.cos(), freqs.sin()


def _rot(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    half = x.shape[-1] // 2
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def rope_qkv_fwd(qkv: torch.Tensor, B: int, S: int, nh: int, cos: torch.Tensor, sin: torch.Tensor):
    """qkv [B*S, 3H] -> q, k, v [B, nh, S, hd] bf16 (q,k rotated in fp32)."""
    hd = qkv.shape[-1] // (3 * nh)
    t = qkv.view(B, S, 3, nh, hd).float()
    c = cos[:S].view(1, S, 1, hd // 2)
    s = sin[:S].view(1, S, 1, hd // 2)
    q = _rot(t[:, :, 0], c, s).transpose(1, 2)
    k = _rot(t[:, :, 1], c, s).transpose(1, 2)
    v = t[:, :, 2].transpose(1, 2)
    dt = qkv.dtype
    return q.to(dt).contiguous(), k.to(dt).contiguous(), v.to(dt).contiguous()


def rope_qkv_bwd(dq: torch.Tensor, dk: torch.Tensor, dv: torch.Tensor,
                 cos: torch.Tensor, sin: torch.Tensor, out=None) -> torch.Tensor:
    """Inverse rotation; returns dqkv [B*S, 3H] in dq's dtype."""
    B, nh, S, hd = dq.shape
    c = cos[:S].view(1, 1, S, hd // 2)
    s = sin[:S].view(1, 1, S, hd // 2)
    gq = _rot(dq.float(), c, -s)
    gk = _rot(dk.float(), c, -s)
    res = torch.stack([gq, gk, dv.float()], dim=0).permute(1, 3, 0, 2, 4).reshape(B * S, 3 * nh * hd).to(dq.dtype)
    if out is not None:
        out.copy_(res)
        return out
    return res


def _qkv_views(qkv: torch.Tensor, B: int, S: int, nh: int):
    hd = qkv.shape[-1] // (3 * nh)
    t = qkv.view(B, S, 3, nh, hd)
    return t, hd


def rope_qk_inplace(qkv: torch.Tensor, B: int, S: int, nh: int, cos: torch.Tensor, sin: torch.Tensor):
    """Rotate the q and k column blocks of the packed [B*S, 3H] QKV in place."""
    t, hd = _qkv_views(qkv, B, S, nh)
    c = cos[:S].view(1, S, 1, hd // 2)
    s = sin[:S].view(1, S, 1, hd // 2)
    for j in (0, 1):
        t[:, :, j] = _rot(t[:, :, j].float(), c, s).to(qkv.dtype)
    return qkv


def _split_packed(qkv, B, S, nh):
    t, _ = _qkv_views(qkv, B, S, nh)
    return tuple(t[:, :, j].transpose(1, 2).contiguous() for j in range(3))


def attention_fwd_packed(qkv: torch.Tensor, B: int, S: int, nh: int, p: float, key: int, out=None, mask=None):
    """Causal attention straight on the (already roped) packed [B*S, 3H] QKV."""
    q, k, v = _split_packed(qkv, B, S, nh)
    return attention_fwd(q, k, v, p, key, True, out=out)


def attention_bwd_packed(qkv, o, do, lse, p: float, key: int, B: int, S: int, nh: int,
                         cos: torch.Tensor, sin: torch.Tensor, out=None) -> torch.Tensor:
    """Backward of attention_fwd_packed + the in-place RoPE: dqkv [B*S, 3H] (pre-RoPE)."""
    q, k, v = _split_packed(qkv, B, S, nh)
    dq, dk, dv = attention_bwd(q, k, v, o, do, lse, p, key, True)
    res = rope_qkv_bwd(dq.float(), dk.float(), dv.float(), cos, sin).to(qkv.dtype)
    if out is not None:
        out.copy_(res)
        return out
    return res


# -------------------------------------------------------------- attention
def attention_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, p: float, key: int,
                  causal: bool = True, out=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """q,k,v [B, nh, S, hd] -> o [B*S, nh*hd] (q dtype), lse [B, nh, S] fp32."""
    B, nh, S, hd = q.shape
    scale = 1.0 / math.sqrt(hd)
    s = torch.matmul(q.float(), k.float().transpose(-2, -1)) * scale
    if causal:
        mask = torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), diagonal=1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    prob = torch.exp(s - lse.unsqueeze(-1))
    if p > 0.0:
        keep = rng.attn_keep_mask(B * nh, S, S, key, p, device=q.device).view(B, nh, S, S)
        prob = torch.where(keep, prob / (1.0 - p), torch.zeros((), device=q.device))
    o = torch.matmul(prob, v.float())
    o = o.transpose(1, 2).reshape(B * S, nh * hd).to(q.dtype)
    if out is not None:
        out.copy_(o)
        o = out
    return o, lse


def attention_bwd(q, k, v, o, do, lse, p: float, key: int, causal: bool = True):
    """Flash-style backward from (o, lse).  do/o are [B*S, H]; returns dq, dk, dv [B,nh,S,hd]."""
    B, nh, S, hd = q.shape
    scale = 1.0 / math.sqrt(hd)
    qf, kf, vf = q.float(), k.float(), v.float()
    of = o.float().view(B, S, nh, hd).transpose(1, 2)
    dof = do.float().view(B, S, nh, hd).transpose(1, 2)
    s = torch.matmul(qf, kf.transpose(-2, -1)) * scale
    if causal:
        mask = torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), diagonal=1)
        s = s.masked_fill(mask, float("-inf"))
    prob = torch.exp(s - lse.unsqueeze(-1))
    if p > 0.0:
        keep = rng.attn_keep_mask(B * nh, S, S, key, p, device=q.device).view(B, nh, S, S)
        pd = torch.where(keep, prob / (1.0 - p), torch.zeros((), device=q.device))
    else:
        keep, pd = None, prob
    dv = torch.matmul(pd.transpose(-2, -1), dof)
    dpd = torch.matmul(dof, vf.transpose(-2, -1))
    dp = torch.where(keep, dpd / (1.0 - p), torch.zeros((), device=q.device)) if keep is not None else dpd
    delta = (dof * of).sum(dim=-1, keepdim=True)
    ds = prob * (dp - delta)
    dq = torch.matmul(ds, kf) * scale
    dk = torch.matmul(ds.transpose(-2, -1), qf) * scale
    dt = q.dtype
    return dq.to(dt), dk.to(dt), dv.to(dt)


# ----------------------------------------------------------------- SwiGLU
def swiglu_fwd(gu: torch.Tensor, out=None) -> torch.Tensor:
    """gu [M, 2I] (gate | up) -> silu(gate) * up [M, I]."""
    i = gu.shape[-1] // 2
    g, u = gu[:, :i].float(), gu[:, i:].float()
    r = (g * torch.sigmoid(g) * u).to(gu.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def swiglu_bwd(gu: torch.Tensor, da: torch.Tensor, out=None, s_out=None) -> torch.Tensor:
    """``s_out``: also writes s = silu(g) * u (as swiglu_fwd)."""
    i = gu.shape[-1] // 2
    if s_out is not None:
        swiglu_fwd(gu, out=s_out)
    g, u = gu[:, :i].float(), gu[:, i:].float()
    d = da.float()
    sg = torch.sigmoid(g)
    silu = g * sg
    dg = d * u * sg * (1.0 + g * (1.0 - sg))
    du = d * silu
    r = torch.cat([dg, du], dim=-1).to(gu.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


# ------------------------------------------------------ cross-entropy (fused with grad)
def cross_entropy_fwd_bwd(logits: torch.Tensor, targets: torch.Tensor, vocab: int,
                          n_valid: torch.Tensor, grad_scale: float = 1.0) -> torch.Tensor:
    """Per-row loss [M] fp32; ``logits`` [M, Vp] is overwritten with
    grad_scale * dloss_mean/dlogits.

    Columns >= vocab are padding and get zero gradient.  Rows whose target is
    IGNORE_INDEX get zero loss and zero gradient.  ``n_valid`` is a 0-dim tensor.
    """
    lf = logits[:, :vocab].float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = targets != IGNORE_INDEX
    tgt = torch.where(valid, targets, torch.zeros_like(targets))
    picked = lf.gather(1, tgt.unsqueeze(1)).squeeze(1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    grad = torch.exp(lf - lse.unsqueeze(1))
    grad.scatter_add_(1, tgt.unsqueeze(1), -torch.ones_like(picked).unsqueeze(1))
    grad = grad * (valid.float() * grad_scale / n_valid.float().clamp(min=1)).unsqueeze(1)
    logits.zero_()
    logits[:, :vocab] = grad.to(logits.dtype)
    return loss


# -------------------------------------------------------------- optimizer
def adamw_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
               shadow: Optional[torch.Tensor], lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, grad_scale: torch.Tensor) -> None:
    """torch.optim.AdamW semantics (decoupled wd, bias correction), grad pre-scaled."""
    g = grad.float() * grad_scale.float()
    param.mul_(1.0 - lr * weight_decay)
    exp_avg.lerp_(g, 1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if shadow is not None:
        shadow.copy_(param.to(shadow.dtype))


def sumsq(x: torch.Tensor, out: torch.Tensor) -> None:
    out += x.float().pow(2).sum()


def scale_bf16(x: torch.Tensor, scale: torch.Tensor, out: torch.Tensor = None, mul: float = 1.0) -> torch.Tensor:
    """y = x * scale * mul (scale: 0-d/1-element device tensor), result in x's dtype."""
    y = (x.float() * scale.reshape(()).float() * mul).to(x.dtype)
    return y if out is None else out.copy_(y)
