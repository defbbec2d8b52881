"""fp32-activation wrappers (``csrc/fp32.hip``) behind the op functions of ``ops/hip.py``.

``hip.<op>`` hands over here when its activation tensor is fp32: the engine's
``--mixed_precision fp32`` mode (the reference's fp32 path, ``ddp_trainer.py:137-139``)
then runs HIP kernels for every non-GEMM op, as bf16 / fp16 do; the GEMMs are hipBLASLt
fp32.  Same semantics and dropout bits as ``ops/reference.py``; attention supports
head_dim 64 and 128 (the flash kernels; the GEMM formulation takes any head_dim <= 256).
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import rng

c_void_p, c_int, c_float, c_uint32, c_long = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint32, ctypes.c_long

SIGS = {
    "dlt_f32_norm_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_uint32,
                         c_uint32, c_float, c_void_p],
    "dlt_f32_norm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_float, c_int, c_int, c_uint32, c_uint32, c_float, c_void_p],
    "dlt_f32_rope": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_long, c_long,
                     c_long, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p],
    "dlt_f32_swiglu_fwd": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "dlt_f32_swiglu_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "dlt_f32_cross_entropy": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p],
    "dlt_f32_scale": [c_void_p, c_void_p, c_long, c_void_p, c_float, c_void_p],
    "dlt_f32_attn_fwd": [c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_void_p, c_void_p, c_void_p, c_int,
                         c_int, c_int, c_int, c_float, c_float, c_void_p],
    "dlt_f32_attn_bwd": [c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_long, c_long, c_int, c_int, c_int, c_int,
                         c_float, c_float, c_void_p],
    "dlt_f32_attn_softmax": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_int, c_void_p],
    "dlt_f32_attn_dsoftmax": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                              c_float, c_float, c_int, c_void_p],
    # 16-bit GEMM-formulated attention (csrc/attn_gemm.hip, used by ops/attn_gemm.py)
    "dlt_attn16_softmax": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_int, c_int,
                           c_void_p],
    "dlt_attn16_dsoftmax": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                            c_int, c_int, c_float, c_float, c_int, c_int, c_void_p],
    "dlt_relayout16": [c_void_p, c_void_p, c_long, c_long, c_long, c_long, c_long, c_long, c_long, c_long, c_int, c_int,
                       c_int, c_int, c_int, c_void_p],
}

ATTN_HEAD_DIMS = (64, 128)

# fp32 attention: "gemm" -- the dense [S, S] score matrix of every (b, h) through batched
# hipBLASLt fp32 GEMMs (MFMA) around two row kernels; "flash" -- the lane-per-query VALU
# kernels (no [S, S] buffer); "auto" -- gemm while S <= 4096 and its two score buffers fit
# in GEMM_ATTN_BYTES.  The causal half the GEMMs compute for nothing is cheaper than the
# flash kernels' LDS-broadcast-bound FMAs (profiles/r5_fp32_attention.md).
ATTN_IMPL = os.environ.get("DLT_F32_ATTN", "auto")
GEMM_ATTN_BYTES = 16 << 30
BMM_PLANNER = os.environ.get("DLT_F32_BMM", "torch") == "planner"
ATTN_BLOCKS = int(os.environ.get("DLT_ATTN_BLOCKS", "4"))


def _h():
    from . import hip
    return hip


def _req32(t: torch.Tensor, name: str, numel=None):
    _h()._req(t, torch.float32, name, numel)


def _chk(rc, name):
    _h()._chk(rc, name)


def _p(t):
    return _h()._p(t)


def _st():
    return _h()._stream()


def _lib():
    return _h().lib()


# ---------------------------------------------------------------- RMSNorm
def add_dropout_rmsnorm_fwd(resid, delta, weight, eps, p, key, y_out=None):
    src = resid if resid is not None else delta
    M, H = src.shape
    for t, n in ((resid, "resid"), (delta, "delta")):
        if t is not None:
            _req32(t, "rmsnorm_f32." + n, M * H)
    w = weight.float().contiguous()
    if w.numel() != H:
        raise ValueError("rmsnorm_f32.weight: expected H elements")
    y = torch.empty(M, H, dtype=torch.float32, device=src.device) if y_out is None else y_out
    _req32(y, "rmsnorm_f32.y", M * H)
    rstd = torch.empty(M, dtype=torch.float32, device=src.device)
    if delta is None:
        x, xo = resid, None
    else:
        x = torch.empty(M, H, dtype=torch.float32, device=src.device)
        xo = x
    thr = rng.keep_threshold(p)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    _chk(_lib().dlt_f32_norm_fwd(_p(resid), _p(delta), _p(w), _p(xo), _p(y), _p(rstd), M, H, float(eps),
                                 key & 0xFFFFFFFF, thr, dscale, _st()), "f32_norm_fwd")
    return x, y, rstd


def rmsnorm_bwd(dy, x, rstd, weight, dres, dweight, p_prev, key_prev, dy_scale=None, want_ddelta=True,
                ddelta_out=None, dy_mul: float = 1.0):
    M, H = x.shape
    _req32(dy, "rmsnorm_bwd_f32.dy", M * H)
    _req32(x, "rmsnorm_bwd_f32.x", M * H)
    _req32(rstd, "rmsnorm_bwd_f32.rstd", M)
    if dres is not None:
        _req32(dres, "rmsnorm_bwd_f32.dres", M * H)
    _req32(dweight, "rmsnorm_bwd_f32.dweight", H)
    w = weight.float().contiguous()
    scale_t = dy_scale.reshape(1).float().contiguous() if dy_scale is not None else None
    dx = torch.empty(M, H, dtype=torch.float32, device=x.device)
    dd = None
    if want_ddelta:
        dd = torch.empty(M, H, dtype=torch.float32, device=x.device) if ddelta_out is None else ddelta_out
        _req32(dd, "rmsnorm_bwd_f32.ddelta", M * H)
    thr = rng.keep_threshold(p_prev)
    dscale = 1.0 / (1.0 - p_prev) if thr else 1.0
    nb = min(1024, (M + 3) // 4)
    ws = torch.empty(max(nb, 1) * H, dtype=torch.float32, device=x.device)
    _chk(_lib().dlt_f32_norm_bwd(_p(dy), _p(x), _p(rstd), _p(w), _p(dres), _p(dx), _p(dd), _p(dweight), _p(ws),
                                 _p(scale_t), float(dy_mul), M, H, key_prev & 0xFFFFFFFF, thr, dscale, _st()),
         "f32_norm_bwd")
    return dx, dd


# ------------------------------------------------------------------- RoPE
def rope_qk_inplace(qkv, B, S, nh, cos, sin, sign: float = 1.0):
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    _req32(qkv, "rope_qk_f32.qkv")
    H = nh * hd
    base = qkv.data_ptr()
    ptr = [ctypes.c_void_p(base + j * H * 4) for j in range(3)]
    st = (S * threeH, threeH, hd)
    if cos.shape[0] < S or cos.shape[1] != hd // 2 or sin.shape != cos.shape:
        raise ValueError("rope tables too short")
    c, s = cos.contiguous(), sin.contiguous()
    _chk(_lib().dlt_f32_rope(*ptr, *ptr, *st, *st, _p(c), _p(s), B, S, nh, hd, float(sign), 2, _st()), "f32_rope_qk")
    return qkv


def rope_qkv_fwd(qkv, B, S, nh, cos, sin):
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    _req32(qkv, "rope_qkv_f32.qkv")
    q = torch.empty(B, nh, S, hd, dtype=torch.float32, device=qkv.device)
    k, v = torch.empty_like(q), torch.empty_like(q)
    H = nh * hd
    src = [ctypes.c_void_p(qkv.data_ptr() + j * H * 4) for j in range(3)]
    c, s = cos.contiguous(), sin.contiguous()
    if c.shape[0] < S or c.shape[1] != hd // 2:
        raise ValueError("rope tables too short")
    _chk(_lib().dlt_f32_rope(*src, _p(q), _p(k), _p(v), S * threeH, threeH, hd, nh * S * hd, hd, S * hd, _p(c), _p(s),
                             B, S, nh, hd, 1.0, 3, _st()), "f32_rope_qkv")
    return q, k, v


def rope_qkv_bwd(dq, dk, dv, cos, sin, out=None):
    B, nh, S, hd = dk.shape
    for t, n in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        _req32(t.contiguous(), "rope_bwd_f32." + n)
    dq, dk, dv = dq.contiguous(), dk.contiguous(), dv.contiguous()
    H = nh * hd
    if out is None:
        out = torch.empty(B * S, 3 * H, dtype=torch.float32, device=dk.device)
    _req32(out, "rope_bwd_f32.out", B * S * 3 * H)
    dst = [ctypes.c_void_p(out.data_ptr() + j * H * 4) for j in range(3)]
    c, s = cos.contiguous(), sin.contiguous()
    _chk(_lib().dlt_f32_rope(_p(dq), _p(dk), _p(dv), *dst, nh * S * hd, hd, S * hd, S * 3 * H, 3 * H, hd, _p(c), _p(s),
                             B, S, nh, hd, -1.0, 3, _st()), "f32_rope_qkv_bwd")
    return out


# -------------------------------------------------------------- attention
def _check_hd(hd):
    if hd not in ATTN_HEAD_DIMS:
        raise NotImplementedError(f"fp32 attention kernels take head_dim 64 or 128 (got {hd})")


def _mask(B, nh, S, p, key, device, mask=None):
    thr = rng.keep_threshold(p)
    if not thr:
        return None, 1.0
    if mask is None:
        mask = _h().attention_dropout_mask(B, nh, S, p, key, device=device)
    return mask, 1.0 / (1.0 - p)


def _use_gemm(B, nh, S, hd):
    if ATTN_IMPL not in ("auto", "gemm", "flash"):
        raise ValueError(f"DLT_F32_ATTN={ATTN_IMPL!r}: expected auto, gemm or flash")
    if ATTN_IMPL == "flash":
        return False
    fits = S <= 4096 and hd <= 256 and 2 * B * nh * S * S * 4 <= GEMM_ATTN_BYTES
    if ATTN_IMPL == "gemm" and not fits:
        raise ValueError(f"fp32 GEMM attention: S={S}, hd={hd}, B*nh={B * nh} exceeds its limits")
    return fits


def _relayout(src, sstr, B, S, nh, hd, device, dst=None, dstr=None):
    """Strided copy of len(src) tensors (element (b, s, h, d) at ptr + b*st[0] + s*st[1] +
    h*st[2] + d) into head-major [n, B, nh, S, hd] (k_f32_rope without rotation), or into
    ``dst`` pointers with strides ``dstr``."""
    n = len(src)
    out = None
    if dst is None:
        out = torch.empty(n, B, nh, S, hd, dtype=torch.float32, device=device)
        dst, dstr = [_p(out[j]) for j in range(n)], (nh * S * hd, hd, S * hd)
    pad = [None] * (3 - n)
    _chk(_lib().dlt_f32_rope(*src, *pad, *dst, *pad, *sstr, *dstr, None, None, B, S, nh, hd, 1.0, n, _st()),
         "f32_relayout")
    return out


def _bmm(kind, a, b, out_dtype=None):
    """Batched row-major products over contiguous [..., r, c] operands: "nt" a @ b^T,
    "nn" a @ b, "tn" a^T @ b, output in ``out_dtype`` (default: the operands').  fp32:
    torch.matmul (hipBLASLt's heuristic pick) by default; BMM_PLANNER routes them through
    the autotuned planner of ops/gemm.py instead (within 1 % of torch.matmul in the fp32
    step, tools/ab/README.md).  16-bit operands always take the planner (fp32
    scores from 16-bit operands are not a torch.matmul form)."""
    from . import gemm
    out_dtype = out_dtype or a.dtype
    if a.dtype == torch.float32 and not (BMM_PLANNER and gemm.available()):
        a2 = a.transpose(-1, -2) if kind == "tn" else a
        return torch.matmul(a2, b.transpose(-1, -2) if kind == "nt" else b)
    *lead, ra, ca = a.shape
    rb, cb = b.shape[-2:]
    bt = a.numel() // (ra * ca)
    M, K = (ca, ra) if kind == "tn" else (ra, ca)
    N = rb if kind == "nt" else cb
    c = torch.empty(*lead, M, N, dtype=out_dtype, device=a.device)
    sa, sb, sc = ra * ca, rb * cb, M * N
    if kind == "nt":    # C^T = op_T(B_c) . A_c
        gemm._gemm_batched(1, 0, N, M, K, b, cb, sb, a, ca, sa, c, N, sc, bt)
    elif kind == "nn":  # C^T = B_c . A_c
        gemm._gemm_batched(0, 0, N, M, K, b, cb, sb, a, ca, sa, c, N, sc, bt)
    else:               # C^T = B_c . op_T(A_c)
        gemm._gemm_batched(0, 1, N, M, K, b, cb, sb, a, ca, sa, c, N, sc, bt)
    return c


def attn_blocks(S: int) -> int:
    """Row blocks T of the causal GEMMs (``DLT_ATTN_BLOCKS``, default 4; needs the planner):
    query block i (S/T rows) multiplies only the keys below its end, so the products do
    (T+1)/(2T) of the dense work (T = 4: 62.5 %) and the row kernels write only the columns
    the next products read.  1 = dense."""
    from . import gemm
    T = ATTN_BLOCKS
    while T > 1 and (S % (4 * T) or S // T < 64):
        T //= 2
    return T if T > 1 and gemm.available() else 1


def _gb(kind, a, b, c, M, N, K, lda, ldb, ldc, sa, sb, scc, bt):
    """One batched row-major product through the planner on (possibly offset) views:
    "nt" C = A B^T, "nn" C = A B, "tn" C = A^T B; leading dims / batch strides explicit."""
    from . import gemm
    ta, tb = {"nt": (1, 0), "nn": (0, 0), "tn": (0, 1)}[kind]
    gemm._gemm_batched(ta, tb, N, M, K, b, ldb, sb, a, lda, sa, c, ldc, scc, bt)


def blocked_scores(x3, y3, out3, T, S, hd):
    """out3[:, block i, :L_i] = x3[:, block i] @ y3[:, :L_i]^T (x3 / y3 [BH, S, hd], out3 [BH, S, S])."""
    Sb, BH = S // T, x3.shape[0]
    for i in range(T):
        _gb("nt", x3[:, i * Sb:], y3, out3[:, i * Sb:], Sb, (i + 1) * Sb, hd, hd, hd, S, S * hd, S * hd, S * S, BH)


def blocked_rows(p3, y3, out3, T, S, hd):
    """out3[:, block i] = p3[:, block i, :L_i] @ y3[:, :L_i] (P.V, dS.K)."""
    Sb, BH = S // T, p3.shape[0]
    for i in range(T):
        _gb("nn", p3[:, i * Sb:], y3, out3[:, i * Sb:], Sb, hd, (i + 1) * Sb, S, hd, hd, S * S, S * hd, S * hd, BH)


def blocked_cols(p3, y3, out3, T, S, hd):
    """out3[:, block j] = p3[:, j*Sb:, block j]^T @ y3[:, j*Sb:] (Pd^T.dO, dS^T.Q)."""
    Sb, BH = S // T, p3.shape[0]
    for j in range(T):
        _gb("tn", p3[:, j * Sb:, j * Sb:], y3[:, j * Sb:], out3[:, j * Sb:], Sb, hd, S - j * Sb, S, hd, hd, S * S,
            S * hd, S * hd, BH)


def _packed_ptrs(t, n, H):
    return [ctypes.c_void_p(t.data_ptr() + j * H * 4) for j in range(n)]


def _gemm_fwd(q4, k4, v4, B, nh, S, hd, p, key, device, out, mask, store_mask):
    o = torch.empty(B * S, nh * hd, dtype=torch.float32, device=device) if out is None else out
    _req32(o, "attn_f32.o", B * S * nh * hd)
    lse = torch.empty(B, nh, S, dtype=torch.float32, device=device)
    mask, dscale = _mask(B, nh, S, p, key, device, mask)
    T, BH = attn_blocks(S), B * nh
    if T > 1:
        sc = torch.empty(B, nh, S, S, dtype=torch.float32, device=device)
        blocked_scores(q4.view(BH, S, hd), k4.view(BH, S, hd), sc.view(BH, S, S), T, S, hd)
    else:
        sc = _bmm("nt", q4, k4)
    _chk(_lib().dlt_f32_attn_softmax(_p(sc), _p(lse), _p(mask), BH, S, 1.0 / math.sqrt(hd), dscale,
                                     S // T if T > 1 else 0, _st()), "f32_attn_softmax")
    if T > 1:
        o4 = torch.empty(B, nh, S, hd, dtype=torch.float32, device=device)
        blocked_rows(sc.view(BH, S, S), v4.view(BH, S, hd), o4.view(BH, S, hd), T, S, hd)
    else:
        o4 = _bmm("nn", sc, v4)
    del sc
    _relayout([_p(o4)], (nh * S * hd, hd, S * hd), B, S, nh, hd, device, [_p(o)], (S * nh * hd, nh * hd, hd))
    return o, _h().AttnAux((lse, mask if store_mask else None))


def _gemm_bwd(q4, k4, v4, o, do, aux, B, nh, S, hd, p, key, device):
    """(dq, dk, dv) as contiguous [B, nh, S, hd]."""
    lse, mask = aux if isinstance(aux, tuple) else (aux, None)
    _req32(lse, "attn_bwd_f32.lse", B * nh * S)
    _req32(o, "attn_bwd_f32.o", B * S * nh * hd)
    _req32(do, "attn_bwd_f32.do", B * S * nh * hd)
    mask, dscale = _mask(B, nh, S, p, key, device, mask)
    do4 = _relayout([_p(do)], (S * nh * hd, nh * hd, hd), B, S, nh, hd, device)[0]
    T, BH = attn_blocks(S), B * nh
    if T > 1:
        q3, k3, v3, do3 = (t.view(BH, S, hd) for t in (q4, k4, v4, do4))
        sc = torch.empty(B, nh, S, S, dtype=torch.float32, device=device)
        dp = torch.empty_like(sc)
        blocked_scores(q3, k3, sc.view(BH, S, S), T, S, hd)
        blocked_scores(do3, v3, dp.view(BH, S, S), T, S, hd)
    else:
        sc = _bmm("nt", q4, k4)
        dp = _bmm("nt", do4, v4)
    _chk(_lib().dlt_f32_attn_dsoftmax(_p(sc), _p(dp), _p(lse), _p(o), _p(do), _p(mask), B, nh, S, hd,
                                      1.0 / math.sqrt(hd), dscale, S // T if T > 1 else 0, _st()), "f32_attn_dsoftmax")
    if T > 1:
        dq, dk, dv = (torch.empty(B, nh, S, hd, dtype=torch.float32, device=device) for _ in range(3))
        blocked_cols(sc.view(BH, S, S), do3, dv.view(BH, S, hd), T, S, hd)
        del sc
        blocked_rows(dp.view(BH, S, S), k3, dq.view(BH, S, hd), T, S, hd)
        blocked_cols(dp.view(BH, S, S), q3, dk.view(BH, S, hd), T, S, hd)
        return dq, dk, dv
    dv = _bmm("tn", sc, do4)
    del sc
    dq = _bmm("nn", dp, k4)
    dk = _bmm("tn", dp, q4)
    return dq, dk, dv


def _fwd(qp, kp, vp, strides, B, nh, S, hd, p, key, device, out, mask, store_mask=True, scale=None):
    """The VALU flash forward; ``scale`` overrides 1/sqrt(hd) (heads zero-padded to hd)."""
    _check_hd(hd)
    o = torch.empty(B * S, nh * hd, dtype=torch.float32, device=device) if out is None else out
    _req32(o, "attn_f32.o", B * S * nh * hd)
    lse = torch.empty(B, nh, S, dtype=torch.float32, device=device)
    mask, dscale = _mask(B, nh, S, p, key, device, mask)
    sc = 1.0 / math.sqrt(hd) if scale is None else float(scale)
    _chk(_lib().dlt_f32_attn_fwd(qp, kp, vp, *strides, _p(o), _p(lse), _p(mask), B, nh, S, hd, sc, dscale, _st()),
         "f32_attn_fwd")
    # store_mask=False: the keep bits only live for this call (the backward regenerates them)
    return o, _h().AttnAux((lse, mask if store_mask else None))


def attention_fwd(q, k, v, p, key, causal=True, store_mask=True, out=None, mask=None):
    if not causal:
        raise NotImplementedError("only causal attention is implemented (the model is a causal LM)")
    B, nh, S, hd = q.shape
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _req32(t, "attn_f32." + n, B * nh * S * hd)
    if _use_gemm(B, nh, S, hd):
        return _gemm_fwd(q, k, v, B, nh, S, hd, p, key, q.device, out, mask, store_mask)
    return _fwd(_p(q), _p(k), _p(v), (nh * S * hd, S * hd, hd), B, nh, S, hd, p, key, q.device, out, mask,
                store_mask)


def attention_fwd_packed(qkv, B, S, nh, p, key, out=None, mask=None, store_mask=True):
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    if M != B * S or hd * 3 * nh != threeH:
        raise ValueError("packed attention: qkv must be [B*S, 3*nh*hd]")
    _req32(qkv, "attn_f32.qkv")
    H = nh * hd
    if _use_gemm(B, nh, S, hd):
        q4, k4, v4 = _relayout(_packed_ptrs(qkv, 3, H), (S * threeH, threeH, hd), B, S, nh, hd, qkv.device)
        return _gemm_fwd(q4, k4, v4, B, nh, S, hd, p, key, qkv.device, out, mask, store_mask)
    ptr = [ctypes.c_void_p(qkv.data_ptr() + j * H * 4) for j in range(3)]
    return _fwd(*ptr, (S * threeH, hd, threeH), B, nh, S, hd, p, key, qkv.device, out, mask, store_mask)


def _bwd(qp, kp, vp, strides, o, do, aux, B, nh, S, hd, p, key, device, gp, gstrides, scale=None):
    _check_hd(hd)
    lse, mask = aux if isinstance(aux, tuple) else (aux, None)
    _req32(lse, "attn_bwd_f32.lse", B * nh * S)
    _req32(o, "attn_bwd_f32.o", B * S * nh * hd)
    _req32(do, "attn_bwd_f32.do", B * S * nh * hd)
    mask, dscale = _mask(B, nh, S, p, key, device, mask)
    delta = torch.empty(B, nh, S, dtype=torch.float32, device=device)
    _chk(_lib().dlt_f32_attn_bwd(qp, kp, vp, *strides, _p(o), _p(do), _p(lse), _p(mask), _p(delta), *gp, *gstrides,
                                 B, nh, S, hd, 1.0 / math.sqrt(hd) if scale is None else float(scale), dscale, _st()),
         "f32_attn_bwd")


def attention_bwd(q, k, v, o, do, aux, p, key, causal=True):
    B, nh, S, hd = q.shape
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _req32(t, "attn_bwd_f32." + n, B * nh * S * hd)
    if _use_gemm(B, nh, S, hd):
        return _gemm_bwd(q, k, v, o, do, aux, B, nh, S, hd, p, key, q.device)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    st = (nh * S * hd, S * hd, hd)
    _bwd(_p(q), _p(k), _p(v), st, o, do, aux, B, nh, S, hd, p, key, q.device, (_p(dq), _p(dk), _p(dv)), st)
    return dq, dk, dv


def attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=None):
    """dqkv [B*S, 3H] (pre-RoPE): the attention backward writes raw dq / dk / dv into the
    packed layout, then the inverse rotation runs in place on the q and k blocks."""
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    _req32(qkv, "attn_bwd_f32.qkv")
    H = nh * hd
    dqkv = torch.empty(M, threeH, dtype=torch.float32, device=qkv.device) if out is None else out
    _req32(dqkv, "attn_bwd_f32.dqkv", M * threeH)
    if _use_gemm(B, nh, S, hd):
        q4, k4, v4 = _relayout(_packed_ptrs(qkv, 3, H), (S * threeH, threeH, hd), B, S, nh, hd, qkv.device)
        dq, dk, dv = _gemm_bwd(q4, k4, v4, o, do, aux, B, nh, S, hd, p, key, qkv.device)
        del q4, k4, v4
        return rope_qkv_bwd(dq, dk, dv, cos, sin, out=dqkv)
    src = [ctypes.c_void_p(qkv.data_ptr() + j * H * 4) for j in range(3)]
    dst = [ctypes.c_void_p(dqkv.data_ptr() + j * H * 4) for j in range(3)]
    st = (S * threeH, hd, threeH)
    _bwd(*src, st, o, do, aux, B, nh, S, hd, p, key, qkv.device, dst, st)
    rope_qk_inplace(dqkv, B, S, nh, cos, sin, sign=-1.0)
    return dqkv


# ----------------------------------------------------------------- SwiGLU
def swiglu_fwd(gu, out=None):
    M, twoI = gu.shape
    _req32(gu, "swiglu_f32.gu")
    out = torch.empty(M, twoI // 2, dtype=torch.float32, device=gu.device) if out is None else out
    _req32(out, "swiglu_f32.out", M * twoI // 2)
    _chk(_lib().dlt_f32_swiglu_fwd(_p(gu), _p(out), M, twoI // 2, _st()), "f32_swiglu_fwd")
    return out


def swiglu_bwd(gu, da, out=None, s_out=None):
    M, twoI = gu.shape
    _req32(gu, "swiglu_bwd_f32.gu")
    _req32(da, "swiglu_bwd_f32.da", M * twoI // 2)
    out = torch.empty_like(gu) if out is None else out
    _req32(out, "swiglu_bwd_f32.out", M * twoI)
    if s_out is not None:
        _req32(s_out, "swiglu_bwd_f32.s_out", M * twoI // 2)
    _chk(_lib().dlt_f32_swiglu_bwd(_p(gu), _p(da), _p(out), _p(s_out), M, twoI // 2, _st()), "f32_swiglu_bwd")
    return out


# ------------------------------------------------------------ cross-entropy
def cross_entropy_fwd_bwd(logits, targets, vocab, n_valid, grad_scale: float = 1.0):
    M, Vp = logits.shape
    _req32(logits, "ce_f32.logits")
    targets = targets.contiguous()
    if targets.dtype != torch.int64 or targets.numel() != M:
        raise ValueError("ce.targets must be int64 [M]")
    nv = n_valid.reshape(1).to(torch.int64).contiguous()
    loss = torch.empty(M, dtype=torch.float32, device=logits.device)
    _chk(_lib().dlt_f32_cross_entropy(_p(logits), _p(targets), _p(nv), _p(loss), M, Vp, vocab, float(grad_scale),
                                      _st()), "f32_cross_entropy")
    return loss


def scale(x, s, out=None, mul: float = 1.0):
    s = s.reshape(1).float().contiguous()
    _req32(x, "scale_f32.x")
    y = torch.empty_like(x) if out is None else out
    _req32(y, "scale_f32.out", x.numel())
    _chk(_lib().dlt_f32_scale(_p(x), _p(y), x.numel(), _p(s), float(mul), _st()), "f32_scale")
    return y
