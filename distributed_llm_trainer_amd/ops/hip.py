"""ctypes bindings for the gfx950 kernel library (``ops/_dlt_kernels.so``).

Every wrapper validates shapes/dtypes/contiguity on the host BEFORE launching (a
mis-shaped launch of a hand-written kernel must never reach the GPU), allocates
outputs with the torch caching allocator and launches on the current HIP stream, so
the calls are graph-capturable and ordered with hipBLASLt GEMMs and RCCL.

Import is loud: on a GPU box, a missing or stale library raises instead of silently
falling back to PyTorch ops.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional

import torch

from . import rng

_LIB = None
# DLT_KERNEL_DEBUG=1 loads the bounds-checked build (ops/build.py --debug);
# DLT_KERNEL_LIB=<file in ops/> loads another build of the same sources (same-box A/B
# of a kernel change: tools/ab/kernels_ab.sh)
_LIBPATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "_dlt_kernels_debug.so" if os.environ.get("DLT_KERNEL_DEBUG") == "1"
                        else os.path.basename(os.environ.get("DLT_KERNEL_LIB", "_dlt_kernels.so")))

c_void_p, c_int, c_float, c_uint32, c_int64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint32, ctypes.c_int64

_SIGS = {
    "dlt_add_dropout_rmsnorm_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                    c_int, c_float, c_uint32, c_uint32, c_float, c_int, c_void_p],
    "dlt_rmsnorm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_void_p, c_float, c_int, c_int, c_uint32, c_uint32, c_float, c_int, c_void_p],
    "dlt_embedding_fwd": [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_embedding_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_embedding_bwd_chunk": [],
    "dlt_splitk_acc": [c_void_p, c_void_p, ctypes.c_long, c_int, c_void_p],
    "dlt_splitk_sum_bf16": [c_void_p, c_void_p, ctypes.c_long, c_int, c_int, c_void_p],
    "dlt_rope_qkv_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                         c_int, c_void_p],
    "dlt_rope_qkv_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_int, c_int, c_void_p],
    "dlt_swiglu_fwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_swiglu_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_cross_entropy_fwd_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int,
                                  c_void_p],
    "dlt_sumsq": [c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    "dlt_clip_coef": [c_void_p, c_void_p, c_float, c_float, c_float, c_void_p],
    "dlt_adamw": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float,
                  c_float, c_float, c_float, c_void_p, c_void_p],
    "dlt_adamw_ex": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float,
                     c_float, c_float, c_float, c_void_p, c_int, c_void_p],
    "dlt_adamw_f16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float,
                      c_float, c_float, c_float, c_void_p, c_void_p],
    "dlt_cast_bf16": [c_void_p, c_void_p, c_int64, c_int, c_void_p],
    "dlt_add_bf16_f32": [c_void_p, c_void_p, c_int64, c_int, c_void_p],
    "dlt_gemm_wgrad": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                       c_void_p],
    "dlt_gemm_wgrad_sk": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_void_p],
    "dlt_scale_bf16": [c_void_p, c_void_p, ctypes.c_long, c_void_p, c_float, c_int, c_void_p],
    "dlt_gemm_bf16_tn": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_void_p],
    "dlt_gemm_fw4": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                     c_int, c_void_p],
    "dlt_gemm_bf16_qkv_rope": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                               c_void_p],
    "dlt_gemm_bf16_gu_swiglu": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "dlt_gemm_bf16_nn": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_void_p],
    "dlt_gemm_bf16_down_swiglu_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      c_int, c_void_p],
    "dlt_attn_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                     c_uint32, c_uint32, c_float, c_int, c_int, c_void_p],
    "dlt_attn_dropout_mask": [c_void_p, c_int, c_int, c_int, c_uint32, c_uint32, c_void_p],
    "dlt_attn_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, c_int, c_void_p],
    "dlt_attn_fwd_ex": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                        c_float, c_uint32, c_uint32, c_float, c_int, ctypes.c_long, c_int, c_int, c_int, c_void_p],
    "dlt_attn_bwd_ex": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, ctypes.c_long, c_int, c_int,
                        ctypes.c_long, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "dlt_rope_qk_inplace": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "dlt_dec_norm_qkv": [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "dlt_dec_attn": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p],
    "dlt_dec_gemv_res": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_dec_norm_gu": [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_dec_norm_head": [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "dlt_dec_sample": [c_void_p, c_int, c_int, c_float, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_int, c_int,
                       c_void_p, c_void_p],
    "dlt_dec_sample_ws_ints": [c_int],
    "dlt_dec_advance": [c_void_p, c_void_p],
}


def library_path() -> str:
    return _LIBPATH


def lib():
    """Load (once) the kernel library; raises with a clear message if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(_LIBPATH):
            raise RuntimeError(
                f"MI355X kernel library not built: {_LIBPATH} missing. Run "
                "`python -m distributed_llm_trainer_amd.ops.build` (or __graft_entry__.build()).")
        import torch  # noqa: F401  (load torch's HIP runtime first so the .so binds to it)
        L = ctypes.CDLL(_LIBPATH)
        from . import hip_f32
        for name, argt in {**_SIGS, **hip_f32.SIGS}.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = c_int
        L.dlt_gemm_wgrad_sk_scratch.argtypes = [c_int, c_int, c_int, c_int]
        L.dlt_gemm_wgrad_sk_scratch.restype = ctypes.c_long
        _LIB = L
    return _LIB


# ---------------------------------------------------------------- fused decode step
DECODE_BATCHES = (1, 2, 4, 8)


def _dec_w(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.data_ptr() % 16:
        raise ValueError(f"{name}: expected a contiguous, 16-byte aligned bf16 weight")


def dec_norm_qkv(h, ln, eps, wqkv, cos, sin, pos, q_out, kc, vc, nh):
    """h [B, H] fp32 -> RMSNorm -> QKV GEMV -> RoPE; k/v rows written into the caches
    [B, nh, maxS, 64] at device position ``pos`` (int64 [1]); q (roped, bf16) into q_out."""
    B, H = h.shape
    _req(h, torch.float32, "dec.h", B * H)
    w, wbf16 = _norm_weight(ln, H, "dec.ln1")
    _dec_w(wqkv, "dec.wqkv")
    _req(q_out, torch.bfloat16, "dec.q", B * H)
    _req(pos, torch.int64, "dec.pos", 1)
    maxS = kc.shape[2]
    if kc.shape != (B, nh, maxS, 64) or vc.shape != kc.shape or wqkv.shape != (3 * H, H) or cos.shape[0] < maxS:
        raise ValueError("dec_norm_qkv: shape mismatch")
    _chk(lib().dlt_dec_norm_qkv(_p(h), _p(w), wbf16, float(eps), _p(wqkv), _p(cos), _p(sin), _p(pos), _p(q_out),
                                _p(kc), _p(vc), B, H, nh, maxS, _stream()), "dec_norm_qkv")


def dec_attn(q, kc, vc, pos, o_out, scale):
    B, nh, maxS, hd = kc.shape
    H = nh * hd
    _req(q, torch.bfloat16, "dec.q", B * H)
    _req(o_out, torch.bfloat16, "dec.o", B * H)
    _chk(lib().dlt_dec_attn(_p(q), _p(kc), _p(vc), _p(pos), _p(o_out), B, H, nh, maxS, float(scale), _stream()),
         "dec_attn")


def dec_gemv_res(x, w, h):
    """h += bf16(x @ w^T) (fp32 residual); x [B, K] bf16, w [R, K] bf16, h [B, R] fp32."""
    B, K = x.shape
    R = w.shape[0]
    _req(x, torch.bfloat16, "dec.x", B * K)
    _dec_w(w, "dec.w")
    _req(h, torch.float32, "dec.h", B * R)
    if w.shape[1] != K:
        raise ValueError("dec_gemv_res: shape mismatch")
    _chk(lib().dlt_dec_gemv_res(_p(x), _p(w), _p(h), B, R, K, _stream()), "dec_gemv_res")


def dec_norm_gu(h, ln, eps, wgu, s_out):
    B, H = h.shape
    I = wgu.shape[0] // 2
    _req(h, torch.float32, "dec.h", B * H)
    w, wbf16 = _norm_weight(ln, H, "dec.ln2")
    _dec_w(wgu, "dec.wgu")
    _req(s_out, torch.bfloat16, "dec.s", B * I)
    _chk(lib().dlt_dec_norm_gu(_p(h), _p(w), wbf16, float(eps), _p(wgu), _p(s_out), B, H, I, _stream()),
         "dec_norm_gu")


def dec_norm_head(h, ln, eps, emb, logits, V):
    B, H = h.shape
    _req(h, torch.float32, "dec.h", B * H)
    w, wbf16 = _norm_weight(ln, H, "dec.norm")
    _dec_w(emb, "dec.lm_head")
    _req(logits, torch.float32, "dec.logits", B * V)
    if emb.shape[0] < V or emb.shape[1] != H:
        raise ValueError("dec_norm_head: shape mismatch")
    _chk(lib().dlt_dec_norm_head(_p(h), _p(w), wbf16, float(eps), _p(emb), _p(logits), B, H, V, _stream()),
         "dec_norm_head")


def dec_sample_workspace(B: int, device) -> torch.Tensor:
    """Scratch of the split (16 workgroups per row) top-k sampler."""
    return torch.empty(int(lib().dlt_dec_sample_ws_ints(B)), dtype=torch.int32, device=device)


def dec_sample(logits, temperature, top_k, seed, pos, ids, hist, hist_base, ws=None):
    """One top-k multinomial draw per row of ``logits`` [B, V] (fp32) on the device: the
    id goes to ``ids`` (B int64, the next decode step's input) and to
    ``hist[b, pos + 1 - hist_base]`` (int64 [B, L]) when inside the history.  With ``ws``
    (:func:`dec_sample_workspace`) and 1 <= top_k <= 64 the row is split over 16
    workgroups."""
    B, V = logits.shape
    if ws is not None:
        _req(ws, torch.int32, "dec.sample_ws", int(lib().dlt_dec_sample_ws_ints(B)))
    _req(logits, torch.float32, "dec.logits", B * V)
    _req(pos, torch.int64, "dec.pos", 1)
    _req(ids, torch.int64, "dec.ids", B)
    _req(hist, torch.int64, "dec.hist")
    if hist.dim() != 2 or hist.shape[0] != B:
        raise ValueError("dec_sample: hist must be [B, L]")
    _chk(lib().dlt_dec_sample(_p(logits), B, V, float(temperature), int(top_k), int(seed) & 0xFFFFFFFF, _p(pos),
                              _p(ids), _p(hist), hist.shape[1], int(hist_base), _p(ws), _stream()), "dec_sample")


def dec_advance(pos):
    _req(pos, torch.int64, "dec.pos", 1)
    _chk(lib().dlt_dec_advance(_p(pos), _stream()), "dec_advance")


def _p(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _chk(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed (code {rc})")


def _req(t: torch.Tensor, dtype, name: str, numel: Optional[int] = None):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a GPU tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: expected {numel} elements, got {t.numel()}")
    if t.data_ptr() % 16:
        raise ValueError(f"{name}: must be 16-byte aligned")


# 16-bit activation formats of the kernels (csrc/common.h HK): bf16 = 0, fp16 = 1
_HK = {torch.bfloat16: 0, torch.float16: 1}


def _hk(t: torch.Tensor, name: str) -> int:
    if t.dtype not in _HK:
        raise TypeError(f"{name}: expected bf16 or fp16 activations, got {t.dtype}")
    return _HK[t.dtype]


def _req_act(t: torch.Tensor, dtype, name: str, numel: Optional[int] = None) -> int:
    """_req for a 16-bit activation tensor of the given format; returns its HK code."""
    if dtype not in _HK:
        raise TypeError(f"{name}: the HIP kernels take bf16 or fp16 activations, not {dtype}")
    _req(t, dtype, name, numel)
    return _HK[dtype]


# ------------------------------------------------------------------ tables
def rope_tables(head_dim: int, seq_len: int, device=None):
    from .reference import rope_tables as rt
    c, s = rt(head_dim, seq_len, device=device)
    return c.contiguous(), s.contiguous()


# ---------------------------------------------------------------- split-K
def splitk_acc(part: torch.Tensor, dw: torch.Tensor) -> None:
    """dw += part.sum(0) in fixed order (deterministic); part [splits, *dw.shape] fp32."""
    _req(dw, torch.float32, "splitk_acc.dw")
    _req(part, torch.float32, "splitk_acc.part")
    n = dw.numel()
    if part.numel() % n or n % 4:
        raise ValueError("splitk_acc: part must hold whole copies of dw and dw.numel() % 4 == 0")
    _chk(lib().dlt_splitk_acc(_p(part), _p(dw), n, part.numel() // n, _stream()), "splitk_acc")


def splitk_sum_bf16(part: torch.Tensor, out: torch.Tensor) -> None:
    """out (bf16 or fp16) = part.sum(0) in fixed order; part [splits, *out.shape] fp32."""
    hk = _req_act(out, out.dtype, "splitk_sum_bf16.out")
    _req(part, torch.float32, "splitk_sum_bf16.part")
    n = out.numel()
    if part.numel() % n or n % 4 or out.data_ptr() % 8:
        raise ValueError("splitk_sum_bf16: part must hold whole copies of out, out.numel() % 4 == 0")
    _chk(lib().dlt_splitk_sum_bf16(_p(part), _p(out), n, part.numel() // n, hk, _stream()), "splitk_sum_bf16")


# ---------------------------------------------------------------- embedding
def embedding_fwd(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    ids = ids.reshape(-1).contiguous()
    if ids.dtype != torch.int64:
        ids = ids.long()
    M = ids.numel()
    V, H = weight.shape
    wdt = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}.get(weight.dtype)
    if wdt is None:
        raise TypeError("embedding weight must be fp32, bf16 or fp16")
    _req(weight, weight.dtype, "embedding.weight")
    out = torch.empty(M, H, dtype=torch.float32, device=weight.device)
    _chk(lib().dlt_embedding_fwd(_p(ids), _p(weight), wdt, _p(out), M, H, V, _stream()), "embedding_fwd")
    return out


def embedding_bwd(ids: torch.Tensor, dout: torch.Tensor, dweight: torch.Tensor) -> None:
    """dweight[ids[m]] += dout[m], deterministically: a stable sort groups equal ids
    (rocPRIM radix sort via torch.sort), the kernels sum each run in position order
    with one writer per row (no float atomics)."""
    ids = ids.reshape(-1)
    M = ids.numel()
    H = dweight.shape[-1]
    _req(dout, torch.float32, "embedding_bwd.dout", M * H)
    _req(dweight, torch.float32, "embedding_bwd.dweight")
    if M == 0:
        return
    if dweight.shape[0] >= 2 ** 31:
        raise ValueError("embedding_bwd: vocabulary too large for int32 ids")
    sids, perm = torch.sort(ids.to(torch.int32), stable=True)  # 32-bit keys: half the radix passes
    ch = lib().dlt_embedding_bwd_chunk()
    ws = torch.empty(2 * (-(-M // ch)) * H, dtype=torch.float32, device=dout.device)
    _chk(lib().dlt_embedding_bwd(_p(sids), _p(perm), _p(dout), _p(dweight), _p(ws), M, H, dweight.shape[0],
                                 _stream()), "embedding_bwd")


# ---------------------------------------------------------------- RMSNorm
def _norm_weight(weight: torch.Tensor, H: int, name: str, act=torch.bfloat16):
    """(tensor, is_16bit): fp32 norm weights, and 16-bit ones in the activation format
    (the gathered FSDP unit), are read in place by the kernels; others are upcast once."""
    if weight.dtype not in (torch.float32, act):
        weight = weight.float()
    align = 8 if weight.dtype != torch.float32 else 16  # u16x4 / float4 loads
    if not weight.is_contiguous() or weight.data_ptr() % align:
        weight = weight.contiguous().clone()
    if not weight.is_cuda or weight.numel() != H:
        raise ValueError(f"{name}: expected a GPU tensor of {H} elements")
    return weight, int(weight.dtype != torch.float32)


def add_dropout_rmsnorm_fwd(resid, delta, weight, eps, p, key, out_dtype=torch.bfloat16, y_out=None):
    if out_dtype == torch.float32:
        from . import hip_f32
        return hip_f32.add_dropout_rmsnorm_fwd(resid, delta, weight, eps, p, key, y_out=y_out)
    src = resid if resid is not None else delta
    M, H = src.shape
    if out_dtype not in _HK:
        raise TypeError("HIP rmsnorm emits bf16 or fp16")
    if resid is not None:
        _req(resid, torch.float32, "rmsnorm.resid", M * H)
    if delta is not None:
        _req_act(delta, out_dtype, "rmsnorm.delta", M * H)
    w, wbf16 = _norm_weight(weight, H, "rmsnorm.weight", out_dtype)
    y = torch.empty(M, H, dtype=out_dtype, device=src.device) if y_out is None else y_out
    hk = _req_act(y, out_dtype, "rmsnorm.y", M * H)
    rstd = torch.empty(M, dtype=torch.float32, device=src.device)
    if delta is None:
        x, xo = resid, None       # x is just the residual: no copy
    else:
        x = torch.empty(M, H, dtype=torch.float32, device=src.device)
        xo = x
    thr = rng.keep_threshold(p)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    _chk(lib().dlt_add_dropout_rmsnorm_fwd(_p(resid), _p(delta), _p(w), wbf16, _p(xo), _p(y), _p(rstd), M, H,
                                           float(eps),
                                           key & 0xFFFFFFFF, thr, dscale, hk, _stream()), "add_dropout_rmsnorm_fwd")
    return x, y, rstd


def rmsnorm_bwd(dy, x, rstd, weight, dres, dweight, p_prev, key_prev, dy_scale=None, want_ddelta=True,
                ddelta_out=None, dy_mul: float = 1.0):
    if dy.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.rmsnorm_bwd(dy, x, rstd, weight, dres, dweight, p_prev, key_prev, dy_scale, want_ddelta, ddelta_out,
                                   dy_mul)
    M, H = x.shape
    act = dy.dtype
    hk = _req_act(dy, act, "rmsnorm_bwd.dy", M * H)
    _req(x, torch.float32, "rmsnorm_bwd.x", M * H)
    _req(rstd, torch.float32, "rmsnorm_bwd.rstd", M)
    if dres is not None:
        _req(dres, torch.float32, "rmsnorm_bwd.dres", M * H)
    _req(dweight, torch.float32, "rmsnorm_bwd.dweight", H)
    w, wbf16 = _norm_weight(weight, H, "rmsnorm_bwd.weight", act)
    scale_t = None
    if dy_scale is not None:
        scale_t = dy_scale.reshape(1).float().contiguous()
    dx = torch.empty(M, H, dtype=torch.float32, device=x.device)
    dd = None
    if want_ddelta:
        dd = torch.empty(M, H, dtype=act, device=x.device) if ddelta_out is None else ddelta_out
        _req(dd, act, "rmsnorm_bwd.ddelta", M * H)
    thr = rng.keep_threshold(p_prev)
    dscale = 1.0 / (1.0 - p_prev) if thr else 1.0
    # per-block dw partials (two-stage column reduction instead of same-address atomics)
    ws = torch.empty(min((M + 3) // 4, 1024) * H, dtype=torch.float32, device=x.device)
    _chk(lib().dlt_rmsnorm_bwd(_p(dy), _p(x), _p(rstd), _p(w), wbf16, _p(dres), _p(dx), _p(dd), _p(dweight), _p(ws),
                               _p(scale_t), float(dy_mul), M, H, key_prev & 0xFFFFFFFF, thr, dscale, hk, _stream()),
         "rmsnorm_bwd")
    return dx, dd


# ------------------------------------------------------------------- RoPE
def rope_qkv_fwd(qkv, B, S, nh, cos, sin):
    if qkv.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    if M != B * S or hd * 3 * nh != threeH:
        raise ValueError("rope_qkv_fwd: bad shapes")
    hk = _req_act(qkv, qkv.dtype, "rope.qkv")
    if cos.shape[0] < S or cos.shape[1] != hd // 2:
        raise ValueError("rope tables too short")
    q = torch.empty(B, nh, S, hd, dtype=qkv.dtype, device=qkv.device)
    k = torch.empty_like(q)
    v = torch.empty_like(q)
    _chk(lib().dlt_rope_qkv_fwd(_p(qkv), _p(cos), _p(sin), _p(q), _p(k), _p(v), B, S, nh, hd, hk, _stream()),
         "rope_qkv_fwd")
    return q, k, v


def rope_qkv_bwd(dq, dk, dv, cos, sin, out=None):
    if dk.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.rope_qkv_bwd(dq, dk, dv, cos, sin, out=out)
    B, nh, S, hd = dk.shape
    act = dk.dtype
    for t, n in ((dk, "dk"), (dv, "dv")):
        hk = _req_act(t, act, "rope_bwd." + n, B * nh * S * hd)
    dqf = dq if dq.dtype == torch.float32 else None
    dqb = dq if dq.dtype == act else None
    _req(dq, dq.dtype, "rope_bwd.dq", B * nh * S * hd)
    if out is None:
        out = torch.empty(B * S, 3 * nh * hd, dtype=act, device=dk.device)
    _req(out, act, "rope_bwd.out", B * S * 3 * nh * hd)
    _chk(lib().dlt_rope_qkv_bwd(_p(dqb), _p(dqf), _p(dk), _p(dv), _p(cos), _p(sin), _p(out), B, S, nh, hd, hk,
                                _stream()),
         "rope_qkv_bwd")
    return out


def rope_qk_inplace(qkv, B, S, nh, cos, sin):
    """Rotate the q and k column blocks of the packed [B*S, 3H] QKV in place."""
    if qkv.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.rope_qk_inplace(qkv, B, S, nh, cos, sin)
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    if M != B * S or hd * 3 * nh != threeH or hd % 16:
        raise ValueError("rope_qk_inplace: bad shapes")
    hk = _req_act(qkv, qkv.dtype, "rope_qk.qkv")
    if cos.shape[0] < S or cos.shape[1] != hd // 2 or sin.shape != cos.shape:
        raise ValueError("rope tables too short")
    _req(cos, torch.float32, "rope_qk.cos")
    _req(sin, torch.float32, "rope_qk.sin")
    _chk(lib().dlt_rope_qk_inplace(_p(qkv), _p(cos), _p(sin), M, S, nh, hd, hk, _stream()), "rope_qk_inplace")
    return qkv


def _off(t: torch.Tensor, elems: int):
    return ctypes.c_void_p(t.data_ptr() + elems * t.element_size())


# -------------------------------------------------------------- attention
class AttnAux(tuple):
    """(lse [B,nh,S] fp32, keep-bit masks [2, B*nh, ceil(S/32), S] int32 or None:
    [0] = bits by (key word, query), [1] = bits by (query word, key); word-major)."""


# head dims of the 16-bit MFMA attention kernels (template parameter D of attention.hip)
ATTN_HEAD_DIMS = (64, 128)


def attention_dropout_mask(B, nh, S, p, key, device=None):
    """Keep-bit masks [2, B*nh, ceil(S/32), S] for attention dropout (None if p == 0).
    Data-independent, so the engine builds them on a side stream ahead of time."""
    thr = rng.keep_threshold(p)
    if not thr:
        return None
    mask = torch.empty(2, B * nh, (S + 31) // 32, S, dtype=torch.int32, device=device)
    _chk(lib().dlt_attn_dropout_mask(_p(mask), B, nh, S, key & 0xFFFFFFFF, thr, _stream()), "attn_dropout_mask")
    return mask


def attention_fwd(q, k, v, p, key, causal=True, store_mask=True, out=None, mask=None, scale=None):
    """Returns (o [B*S, nh*hd] bf16, aux).  With dropout on, the keep bits are written
    to a bitmask consumed by attention_bwd (no re-hashing in the backward); pass
    ``mask`` from ``attention_dropout_mask`` to skip generating it here.  ``scale``:
    the score scale (default 1/sqrt(hd); ops/attn_gemm.py runs zero-padded heads with
    the unpadded head_dim's)."""
    if q.dtype == torch.float32:
        from . import hip_f32
        if scale is not None:
            raise NotImplementedError("fp32 attention: the score scale is 1/sqrt(head_dim)")
        return hip_f32.attention_fwd(q, k, v, p, key, causal, store_mask=store_mask, out=out, mask=mask)
    if not causal:
        raise NotImplementedError("only causal attention is implemented (the model is a causal LM)")
    B, nh, S, hd = q.shape
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        hk = _req_act(t, q.dtype, "attn." + n, B * nh * S * hd)
    if hd not in ATTN_HEAD_DIMS:
        raise NotImplementedError(f"attention kernels take head_dim {ATTN_HEAD_DIMS} (got {hd})")
    o = torch.empty(B * S, nh * hd, dtype=q.dtype, device=q.device) if out is None else out
    _req(o, q.dtype, "attn.o", B * S * nh * hd)
    lse = torch.empty(B, nh, S, dtype=torch.float32, device=q.device)
    thr = rng.keep_threshold(p)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    gen = 1
    if not thr:
        mask = None
    elif mask is not None:
        _req(mask, torch.int32, "attn.mask", 2 * B * nh * S * ((S + 31) // 32))
        gen = 0
    else:
        # [0] row layout (lane = query), [1] transposed (lane = key) -- see attention.hip;
        # with store_mask=False it only lives for this call (the backward regenerates it)
        mask = torch.empty(2, B * nh, (S + 31) // 32, S, dtype=torch.int32, device=q.device)
    _chk(lib().dlt_attn_fwd(_p(q), _p(k), _p(v), _p(o), _p(lse), _p(mask), B, nh, S, hd,
                            1.0 / math.sqrt(hd) if scale is None else float(scale),
                            key & 0xFFFFFFFF, thr, dscale, gen, hk, _stream()), "attn_fwd")
    return o, AttnAux((lse, mask if (store_mask or gen == 0) else None))


def _packed_dims(qkv, B, S, nh):
    M, threeH = qkv.shape
    hd = threeH // (3 * nh)
    if M != B * S or hd * 3 * nh != threeH:
        raise ValueError("packed attention: qkv must be [B*S, 3*nh*hd]")
    if hd not in ATTN_HEAD_DIMS:
        raise NotImplementedError(f"attention kernels take head_dim {ATTN_HEAD_DIMS} (got {hd})")
    _req_act(qkv, qkv.dtype, "attn.qkv")
    return M, nh * hd, hd


def attention_fwd_packed(qkv, B, S, nh, p, key, out=None, mask=None, store_mask=True):
    """Causal attention reading q/k/v straight from the packed (roped) [B*S, 3H] QKV.
    Returns (o [B*S, H] bf16, aux) like :func:`attention_fwd`."""
    if qkv.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.attention_fwd_packed(qkv, B, S, nh, p, key, out=out, mask=mask, store_mask=store_mask)
    M, H, hd = _packed_dims(qkv, B, S, nh)
    hk = _HK[qkv.dtype]
    o = torch.empty(M, H, dtype=qkv.dtype, device=qkv.device) if out is None else out
    _req(o, qkv.dtype, "attn.o", M * H)
    lse = torch.empty(B, nh, S, dtype=torch.float32, device=qkv.device)
    thr = rng.keep_threshold(p)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    gen = 1
    if not thr:
        mask = None
    elif mask is not None:
        _req(mask, torch.int32, "attn.mask", 2 * B * nh * S * ((S + 31) // 32))
        gen = 0
    else:  # with store_mask=False it only lives for this call (the backward regenerates it)
        mask = torch.empty(2, B * nh, (S + 31) // 32, S, dtype=torch.int32, device=qkv.device)
    _chk(lib().dlt_attn_fwd_ex(_p(qkv), _off(qkv, H), _off(qkv, 2 * H), _p(o), _p(lse), _p(mask), B, nh, S, hd,
                               1.0 / math.sqrt(hd), key & 0xFFFFFFFF, thr, dscale, gen, S * 3 * H, hd, 3 * H, hk,
                               _stream()), "attn_fwd_packed")
    return o, AttnAux((lse, mask if (store_mask or gen == 0) else None))


def attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=None):
    """Backward of :func:`attention_fwd_packed` + the in-place RoPE: returns dqkv
    [B*S, 3H] (gradient w.r.t. the pre-rotation QKV GEMM output); dq/dk/dv are written
    into it by the attention kernels with the inverse rotation in their epilogue."""
    if qkv.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin, out=out)
    M, H, hd = _packed_dims(qkv, B, S, nh)
    hk = _HK[qkv.dtype]
    for t, nm in ((o, "o"), (do, "do")):
        _req(t, qkv.dtype, "attn_bwd." + nm, M * H)
    lse, mask = aux if isinstance(aux, tuple) else (aux, None)
    _req(lse, torch.float32, "attn_bwd.lse", B * nh * S)
    if cos.shape[0] < S or cos.shape[1] != hd // 2 or sin.shape != cos.shape:
        raise ValueError("rope tables too short")
    _req(cos, torch.float32, "attn_bwd.cos")
    _req(sin, torch.float32, "attn_bwd.sin")
    thr = rng.keep_threshold(p)
    if thr and mask is None:  # forward ran with store_mask=False: regenerate the keep bits only
        mask = attention_dropout_mask(B, nh, S, p, key, device=qkv.device)
    if not thr:
        mask = None
    dqkv = torch.empty(M, 3 * H, dtype=qkv.dtype, device=qkv.device) if out is None else out
    _req(dqkv, qkv.dtype, "attn_bwd.dqkv", M * 3 * H)
    delta = torch.empty(B, nh, S, dtype=torch.float32, device=qkv.device)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    st = S * 3 * H
    _chk(lib().dlt_attn_bwd_ex(_p(qkv), _off(qkv, H), _off(qkv, 2 * H), _p(o), _p(do), _p(lse), _p(mask), _p(delta),
                               _p(dqkv), _off(dqkv, H), _off(dqkv, 2 * H), B, nh, S, hd, 1.0 / math.sqrt(hd), dscale,
                               st, hd, 3 * H, st, hd, 3 * H, _p(cos), _p(sin), hk, _stream()), "attn_bwd_packed")
    return dqkv


def attention_bwd(q, k, v, o, do, aux, p, key, causal=True, scale=None):
    if q.dtype == torch.float32:
        from . import hip_f32
        if scale is not None:
            raise NotImplementedError("fp32 attention: the score scale is 1/sqrt(head_dim)")
        return hip_f32.attention_bwd(q, k, v, o, do, aux, p, key, causal)
    B, nh, S, hd = q.shape
    n = B * nh * S * hd
    for t, nm in ((q, "q"), (k, "k"), (v, "v"), (o, "o"), (do, "do")):
        hk = _req_act(t, q.dtype, "attn_bwd." + nm, n)
    if isinstance(aux, tuple):
        lse, mask = aux
    else:
        lse, mask = aux, None
    _req(lse, torch.float32, "attn_bwd.lse", B * nh * S)
    thr = rng.keep_threshold(p)
    if thr and mask is None:  # forward ran with store_mask=False: regenerate the keep bits only
        mask = attention_dropout_mask(q.shape[0], q.shape[1], q.shape[2], p, key, device=q.device)
    if not thr:
        mask = None
    delta = torch.empty(B, nh, S, dtype=torch.float32, device=q.device)
    dq = torch.empty_like(q)
    dk = torch.empty_like(k)
    dv = torch.empty_like(v)
    dscale = 1.0 / (1.0 - p) if thr else 1.0
    _chk(lib().dlt_attn_bwd(_p(q), _p(k), _p(v), _p(o), _p(do), _p(lse), _p(mask), _p(delta), _p(dq), _p(dk), _p(dv),
                            B, nh, S, hd, 1.0 / math.sqrt(hd) if scale is None else float(scale), dscale, hk,
                            _stream()), "attn_bwd")
    return dq, dk, dv


# ----------------------------------------------------------------- SwiGLU
def swiglu_fwd(gu, out=None):
    if gu.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.swiglu_fwd(gu, out=out)
    M, twoI = gu.shape
    hk = _req_act(gu, gu.dtype, "swiglu.gu")
    if out is None:
        out = torch.empty(M, twoI // 2, dtype=gu.dtype, device=gu.device)
    _req(out, gu.dtype, "swiglu.out", M * twoI // 2)
    _chk(lib().dlt_swiglu_fwd(_p(gu), _p(out), M, twoI // 2, hk, _stream()), "swiglu_fwd")
    return out


def swiglu_bwd(gu, da, out=None, s_out=None):
    """dgu = SwiGLU backward; ``s_out``: also writes s = silu(g) * u (the forward's bits)."""
    if gu.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.swiglu_bwd(gu, da, out=out, s_out=s_out)
    M, twoI = gu.shape
    hk = _req_act(gu, gu.dtype, "swiglu_bwd.gu")
    _req(da, gu.dtype, "swiglu_bwd.da", M * twoI // 2)
    if out is None:
        out = torch.empty_like(gu)
    _req(out, gu.dtype, "swiglu_bwd.out", M * twoI)
    if s_out is not None:
        _req(s_out, gu.dtype, "swiglu_bwd.s_out", M * twoI // 2)
    _chk(lib().dlt_swiglu_bwd(_p(gu), _p(da), _p(out), _p(s_out) if s_out is not None else None, M, twoI // 2, hk,
                              _stream()), "swiglu_bwd")
    return out


# ------------------------------------------------------------ cross-entropy
def cross_entropy_fwd_bwd(logits, targets, vocab, n_valid, grad_scale: float = 1.0):
    """Per-row loss; the logits buffer (bf16 or fp16) is overwritten by
    grad_scale * (softmax - onehot) / n_valid (fp16: grad_scale = the loss scale, so the
    gradient does not underflow)."""
    if logits.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.cross_entropy_fwd_bwd(logits, targets, vocab, n_valid, grad_scale)
    M, Vp = logits.shape
    hk = _req_act(logits, logits.dtype, "ce.logits")
    targets = targets.contiguous()
    if targets.dtype != torch.int64 or targets.numel() != M:
        raise ValueError("ce.targets must be int64 [M]")
    nv = n_valid.reshape(1).to(torch.int64).contiguous()
    loss = torch.empty(M, dtype=torch.float32, device=logits.device)
    _chk(lib().dlt_cross_entropy_fwd_bwd(_p(logits), _p(targets), _p(nv), _p(loss), M, Vp, vocab,
                                         float(grad_scale), hk, _stream()), "cross_entropy")
    return loss


# --------------------------------------------------------------- optimizer
_SUMSQ_PARTS = {}  # device -> 1024-float workspace of the two-stage (deterministic) reduction


def sumsq(x: torch.Tensor, out: torch.Tensor) -> None:
    """out[0] += sum(x**2), bitwise reproducible (fixed-order partials, no atomics)."""
    _req(x, torch.float32, "sumsq.x")
    _req(out, torch.float32, "sumsq.out")
    part = _SUMSQ_PARTS.get(x.device)
    if part is None:
        part = _SUMSQ_PARTS[x.device] = torch.empty(1024, dtype=torch.float32, device=x.device)
    _chk(lib().dlt_sumsq(_p(x), x.numel(), _p(part), _p(out), _stream()), "sumsq")


def clip_coef(sumsq_t: torch.Tensor, out: torch.Tensor, norm_mul: float, max_norm: float, scale_mul: float) -> None:
    _chk(lib().dlt_clip_coef(_p(sumsq_t), _p(out), norm_mul, max_norm, scale_mul, _stream()), "clip_coef")


def adamw_flat(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps, wd, step, gscale,
               zero_grad: bool = False):
    """One fused AdamW pass over flat fp32 buffers (+ the 16-bit shadow); ``zero_grad``:
    the gradient is zeroed in the same pass."""
    n = param.numel()
    for t, nm in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _req(t, torch.float32, "adamw." + nm, n)
    if shadow is not None and (shadow.dtype not in (torch.bfloat16, torch.float16) or shadow.numel() != n):
        raise ValueError("adamw.shadow must be bf16 or fp16 of the same numel")
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    f16 = shadow is not None and shadow.dtype == torch.float16
    if zero_grad:
        _chk(lib().dlt_adamw_ex(_p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), _p(shadow), n, lr, beta1, beta2,
                                eps, wd, lr / bc1, 1.0 / math.sqrt(bc2), _p(gscale), (1 if f16 else 0) | 2,
                                _stream()), "adamw")
        return
    fn = lib().dlt_adamw_f16 if f16 else lib().dlt_adamw
    _chk(fn(_p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), _p(shadow), n, lr, beta1, beta2, eps, wd,
            lr / bc1, 1.0 / math.sqrt(bc2), _p(gscale), _stream()), "adamw")


def add_bf16_into_f32(dst: torch.Tensor, src: torch.Tensor) -> bool:
    """dst (fp32) += src (bf16 or fp16) in one kernel; False (nothing launched) if the
    shapes or alignment do not fit the 8-wide vector path."""
    n = dst.numel()
    if (src.numel() != n or n % 8 or not dst.is_contiguous() or not src.is_contiguous()
            or dst.dtype != torch.float32 or src.dtype not in _HK or dst.data_ptr() % 16 or src.data_ptr() % 16):
        return False
    _chk(lib().dlt_add_bf16_f32(_p(dst), _p(src), n, _HK[src.dtype], _stream()), "add_bf16_f32")
    return True


def cast_bf16(x: torch.Tensor, y: torch.Tensor) -> None:
    _chk(lib().dlt_cast_bf16(_p(x), _p(y), x.numel(), _HK[y.dtype], _stream()), "cast_bf16")


# ---------------------------------------------------------------- wgrad GEMM
# the 256 x 128 tile forms of the hand GEMMs (hidden sizes 192 does not divide, e.g. the
# medium model's 1024); DLT_GEMM_BN128=0 leaves such shapes to hipBLASLt
_BN128 = os.environ.get("DLT_GEMM_BN128", "1") != "0"


def wgrad_bn(Nc: int) -> int:
    """dW column tile of the weight-gradient kernel: 192, else 128 (e.g. hidden 1024), else 0."""
    return 192 if Nc % 192 == 0 else (128 if _BN128 and Nc % 128 == 0 else 0)


def wgrad_fits(T: int, Nr: int, Nc: int) -> bool:
    """Shapes the 256 x 192 (or 256 x 128) weight-gradient kernel tiles (T in 128-token
    pairs; a last half row tile when Nr % 256 == 128)."""
    return T > 0 and T % 128 == 0 and Nr % 128 == 0 and wgrad_bn(Nc) > 0


def wgrad_splits(T: int, Nr: int, Nc: int, target: int = 256) -> int:
    """Split-K factor that brings tiles x splits closest to `target` workgroups (one per
    CU), capped by the number of 128-token pairs."""
    tiles = ((Nr + 255) // 256) * (Nc // wgrad_bn(Nc))
    return max(1, min(T // 128, (target + tiles // 2) // tiles))


def gemm_wgrad(dw: Optional[torch.Tensor], dy: torch.Tensor, x: torch.Tensor, splits: int = 0,
               part: Optional[torch.Tensor] = None) -> bool:
    """dw[Nr,Nc] (fp32) += dy[T,Nr]^T @ x[T,Nc] with the hand-written MFMA kernel
    (csrc/gemm_wgrad.hip).  splits == 0 picks the CU-filling split; with splits > 1 the
    fp32 partials go to `part` ([splits, Nr, Nc], allocated if None) and are summed into
    dw in fixed split order (deterministic).  dw = None with splits > 1: only the
    partials are written (the caller reduces them, e.g. straight into bf16).  dy / x:
    both bf16 or both fp16.  Returns False (nothing launched) when the shape does not tile."""
    T, Nr = dy.shape
    Nc = x.shape[1]
    if not wgrad_fits(T, Nr, Nc) or dy.stride(1) != 1 or x.stride(1) != 1 or dy.stride(0) % 8 or x.stride(0) % 8:
        return False
    if dw is None:
        if splits <= 1 or part is None or part.dtype != torch.float32 or part.numel() < splits * Nr * Nc \
                or not part.is_contiguous():
            raise ValueError("gemm_wgrad: partials-only mode needs splits > 1 and an fp32 part buffer")
    else:
        _req(dw, torch.float32, "wgrad.dw", Nr * Nc)
    if dy.dtype not in _WG_HK or x.dtype != dy.dtype or x.shape[0] != T:
        raise ValueError("gemm_wgrad: bf16 / fp16 dy[T,Nr] / x[T,Nc] of one dtype expected")
    if splits <= 0:
        splits = wgrad_splits(T, Nr, Nc)
    splits = min(splits, T // 128)
    if splits > 1 and (part is None or part.numel() < splits * Nr * Nc):
        part = torch.empty(splits * Nr * Nc, device=dw.device, dtype=torch.float32)
    _chk(lib().dlt_gemm_wgrad(_p(dy), _p(x), _p(dw) if dw is not None else None, _p(part) if splits > 1 else None,
                              T, Nr, Nc, dy.stride(0), x.stride(0), splits, _WG_HK[dy.dtype], _stream()),
         "gemm_wgrad")
    if splits > 1 and dw is not None:
        _chk(lib().dlt_splitk_acc(_p(part), _p(dw), Nr * Nc, splits, _stream()), "splitk_acc")
    return True


# operand format of the weight-gradient kernels (HK template parameter)
_WG_HK = {torch.bfloat16: 0, torch.float16: 1}

# DLT_WGRAD_SK_SHARES=n: n shares per column tile instead of 256 / column tiles (A/B knob)
_SK_SHARES = int(os.environ.get("DLT_WGRAD_SK_SHARES", "0"))


def gemm_wgrad_sk(dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor, shares: int = 0) -> bool:
    """dw[Nr,Nc] (fp32) += dy[T,Nr]^T @ x[T,Nc], stream-K form of the hand-written kernel
    (csrc/gemm_wgrad.hip k_gemm_wgrad_sk): one resident workgroup per CU walks an equal
    share of (row tile, token pair) work of one column tile; tiles split between shares
    are summed into dw in fixed share order (bitwise reproducible).  Pays off when a
    share is a sizable part of a tile (gate/up 6144 x 768 and lm_head 50304 x 768 at
    T = 32768: 275 / 2273 us vs 312 / 2422 for the best split-K, profiles/r3_wgrad.md).
    Returns False when the shape does not tile."""
    T, Nr = dy.shape
    Nc = x.shape[1]
    if not wgrad_fits(T, Nr, Nc) or dy.stride(1) != 1 or x.stride(1) != 1 or dy.stride(0) % 8 or x.stride(0) % 8:
        return False
    _req(dw, torch.float32, "wgrad_sk.dw", Nr * Nc)
    if dy.dtype not in _WG_HK or x.dtype != dy.dtype or x.shape[0] != T:
        raise ValueError("gemm_wgrad_sk: bf16 / fp16 dy[T,Nr] / x[T,Nc] of one dtype expected")
    shares = shares or _SK_SHARES
    n = int(lib().dlt_gemm_wgrad_sk_scratch(T, Nr, Nc, shares))
    part = torch.empty(n, device=dw.device, dtype=torch.float32)
    _chk(lib().dlt_gemm_wgrad_sk(_p(dy), _p(x), _p(dw), _p(part), T, Nr, Nc, dy.stride(0), x.stride(0), shares,
                                 _WG_HK[dy.dtype], _stream()), "gemm_wgrad_sk")
    return True


# ------------------------------------------------- projection GEMMs (csrc/gemm_bf16.hip)
# launch flags of the hand projection GEMMs; DLT_GEMM_FLAGS bit 256 = bounded persistence
# (each workgroup walks at most (flags >> 24) & 15 tiles, default 1, grid = tiles / that)
# instead of the persistent grid; DLT_GEMM_GRID=n caps the persistent grid at n
# (multiple of 8) workgroups (A/B knobs for overlapped schedules)
# Production flags (round 4): 1024 = LDS-transposed C stores (whole 192-byte row
# segments per store instruction: the plain epilogue's cycles -26 %), 12 = XCD row-band
# tile walk (an XCD keeps its A panels in its L2), 2048 = write-through (sc1) C stores
# (the C lines leave the XCD's L2 instead of evicting the operand panels: lm_head forward
# later K-iterations 6461 -> 4909 cycles); tools/cpp/gemm_stamps.cpp and
# profiles/r4_gemm_forward.md.  DLT_GEMM_FLAGS=n replaces them (bits 256 / 1024 / 2048 / 12).
_GB_DEFAULT_FLAGS = 2048 | 1024 | 12
_GB_FLAG_BITS = 256 | 1024 | 2048 | 4096 | 12 | (0xf << 24)  # (256 + bits 24-27: tiles per workgroup)
_GB_FLAGS = (int(os.environ.get("DLT_GEMM_FLAGS", str(_GB_DEFAULT_FLAGS))) & _GB_FLAG_BITS) | \
    ((min(int(os.environ.get("DLT_GEMM_GRID", "0")), 2040) // 8) << 16)
# launch flags of the FORWARD projection GEMMs only (plain / RoPE / SwiGLU epilogues),
# A/B knob for the two-chain window: DLT_GEMM_FWD_FLAGS=n replaces their flag bits (e.g.
# 256 | 3084: one tile per workgroup, grid = tiles) while the data gradients keep
# DLT_GEMM_FLAGS; the grid cap of gemm_grid_cap applies to both
_GB_FWD_OVERRIDE = os.environ.get("DLT_GEMM_FWD_FLAGS")


def _fwd_flags() -> int:
    if _GB_FWD_OVERRIDE is None:
        return _GB_FLAGS
    return (int(_GB_FWD_OVERRIDE) & _GB_FLAG_BITS) | (_GB_FLAGS & (0xff << 16))


def gemm_grid_cap(n: int) -> int:
    """Cap the persistent grid of the hand projection GEMMs at ``n`` workgroups (a
    multiple of 8; 0 = one per CU) for the launches that follow; returns the previous
    cap.  Each output tile is still computed whole by one workgroup, so results do not
    change.  The ``ffbb`` window sets 192: the other chain's kernels keep 64 CUs."""
    global _GB_FLAGS
    prev = 8 * ((_GB_FLAGS >> 16) & 0xff)
    _GB_FLAGS = (_GB_FLAGS & ~(0xff << 16)) | ((min(max(int(n), 0), 2040) // 8) << 16)
    return prev


def gemm_bf16_fits(M: int, N: int, K: int) -> bool:
    """Shapes the persistent MFMA kernel tiles exactly: 256 x 192 tiles, or 256 x 128 when
    192 does not divide N (plain store / data-gradient forms only)."""
    return M > 0 and M % 256 == 0 and (N % 192 == 0 or (_BN128 and N % 128 == 0)) and K % 128 == 0 and K >= 128


def gemm_bf16_fits192(M: int, N: int, K: int) -> bool:
    """Shapes the fused-epilogue forms (RoPE, SwiGLU, SwiGLU backward) tile: 256 x 192 only."""
    return gemm_bf16_fits(M, N, K) and N % 192 == 0


def gemm_bf16(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """C[M,N] = A[M,K] @ B[N,K]^T (bf16 or fp16 in/out, one format; fp32 accumulate) with
    the hand-written persistent MFMA kernel.  Returns None (nothing launched) when the
    shape does not tile (M % 256, N % 192, K % 128)."""
    M, K = a.shape
    N = b.shape[0]
    if not gemm_bf16_fits(M, N, K) or b.shape[1] != K:
        return None
    dt = a.dtype if a.dtype in _WG_HK else torch.bfloat16
    _req(a, dt, "gemm_bf16.a")
    _req(b, dt, "gemm_bf16.b")
    c = torch.empty(M, N, dtype=dt, device=a.device) if out is None else out
    _req(c, dt, "gemm_bf16.c", M * N)
    _chk(lib().dlt_gemm_bf16_tn(_p(a), _p(b), _p(c), M, N, K, K, K, N, _fwd_flags(), _WG_HK[dt], _stream()),
         "gemm_bf16")
    return c


def gemm_fw4_fits(M: int, N: int, K: int) -> bool:
    """Shapes the 4-wave 256 x 256 forward GEMM (csrc/gemm_fw4.hip) tiles."""
    return M > 0 and N > 0 and K > 0 and M % 256 == 0 and N % 128 == 0 and K % 64 == 0 and K >= 128


# launch flags of k_gemm_fw4 (csrc/gemm_fw4.hip): 1 = write-through (sc1) / 4 = nt C stores, 2 =
# row-major / 2048 = half-band tile order, 16 | 128 = SCHED 5, 4096 = two tiles per workgroup
_FW4_FLAGS = int(os.environ.get("DLT_GEMM_FW4_FLAGS", "148"))


def gemm_fw4(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
             flags: Optional[int] = None) -> Optional[torch.Tensor]:
    """C[M,N] = A[M,K] @ B[N,K]^T (bf16 or fp16 in/out, fp32 accumulate) with the 4-wave
    256 x 256 one-tile-per-workgroup MFMA kernel (128 x 128 per wave, AGPR accumulators).
    Returns None (nothing launched) when the shape does not tile (M % 256, N % 128, K % 64,
    K < 128)."""
    M, K = a.shape
    N = b.shape[0]
    if not gemm_fw4_fits(M, N, K) or b.shape[1] != K:
        return None
    hk = _req_act(a, a.dtype, "gemm_fw4.a")
    _req(b, a.dtype, "gemm_fw4.b")
    c = torch.empty(M, N, dtype=a.dtype, device=a.device) if out is None else out
    _req(c, a.dtype, "gemm_fw4.c", M * N)
    fl = _FW4_FLAGS if flags is None else flags
    rc = lib().dlt_gemm_fw4(_p(a), _p(b), _p(c), M, N, K, K, K, N, fl & ~1024, hk, None, 0, _stream())
    if rc == -1:
        return None  # a launch variant the shape does not take (two tiles per workgroup: tiles % 16)
    _chk(rc, "gemm_fw4")
    return c


def gemm_fw4_swiglu_fits(M: int, I2: int, K: int) -> bool:
    return gemm_fw4_fits(M, I2, K) and I2 % 256 == 0


def gemm_fw4_swiglu(x: torch.Tensor, wgu: torch.Tensor, gu_out: Optional[torch.Tensor] = None,
                    s_out: Optional[torch.Tensor] = None, flags: Optional[int] = None):
    """(gu[M, 2I], s[M, I]): gu = x @ Wgu^T (gate rows [0, I), up rows [I, 2I)) by the 4-wave
    k_gemm_fw4 with s = silu(gate) * up in its epilogue (csrc/gemm_fw4.hip, flags 1024;
    k_swiglu_fwd's arithmetic, same bits).  None if the shape does not tile (I % 128,
    M % 256, K % 64)."""
    M, K = x.shape
    I2 = wgu.shape[0]
    I = I2 // 2
    if not gemm_fw4_swiglu_fits(M, I2, K) or wgu.shape[1] != K:
        return None
    hk = _req_act(x, x.dtype, "gemm_fw4_swiglu.x")
    _req(wgu, x.dtype, "gemm_fw4_swiglu.w")
    gu = torch.empty(M, I2, dtype=x.dtype, device=x.device) if gu_out is None else gu_out
    s = torch.empty(M, I, dtype=x.dtype, device=x.device) if s_out is None else s_out
    _req(gu, x.dtype, "gemm_fw4_swiglu.gu", M * I2)
    _req(s, x.dtype, "gemm_fw4_swiglu.s", M * I)
    fl = (_FW4_FLAGS if flags is None else flags) & ~(16 | 128)
    if flags is not None and (flags & (16 | 128)) == (16 | 128):
        fl |= 16 | 128  # SCHED 5
    _chk(lib().dlt_gemm_fw4(_p(x), _p(wgu), _p(gu), M, I2, K, K, K, I2, (fl | 1024) & ~4096, hk, _p(s), I, _stream()),
         "gemm_fw4_swiglu")
    return gu, s


def gemm_qkv_rope(x: torch.Tensor, wqkv: torch.Tensor, S: int, cos: torch.Tensor, sin: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """qkv[M, 3H] = x @ Wqkv^T with NeoX RoPE applied to the q and k heads (head_dim 64,
    position of row m = m % S) in the GEMM epilogue -- the packed-QKV projection and
    ``rope_qk_inplace`` in one kernel.  cos/sin: [>= S, 32] fp32.  None if the shape
    does not tile (3H % 192, M % 256, K % 128)."""
    M, K = x.shape
    N = wqkv.shape[0]
    H = N // 3
    if (not gemm_bf16_fits192(M, N, K) or N % 3 or H % 64 or wqkv.shape[1] != K or M % S
            or cos.shape[-1] != 32 or cos.shape[0] < S):
        return None
    _req(x, torch.bfloat16, "gemm_qkv_rope.x")
    _req(wqkv, torch.bfloat16, "gemm_qkv_rope.w")
    _req(cos, torch.float32, "gemm_qkv_rope.cos")
    _req(sin, torch.float32, "gemm_qkv_rope.sin", cos.numel())
    c = torch.empty(M, N, dtype=torch.bfloat16, device=x.device) if out is None else out
    _req(c, torch.bfloat16, "gemm_qkv_rope.out", M * N)
    _chk(lib().dlt_gemm_bf16_qkv_rope(_p(x), _p(wqkv), _p(c), M, H, K, S, _p(cos), _p(sin), _fwd_flags(), _stream()),
         "gemm_qkv_rope")
    return c


def gemm_gu_swiglu(x: torch.Tensor, wgu: torch.Tensor, gu_out: Optional[torch.Tensor] = None,
                   s_out: Optional[torch.Tensor] = None):
    """(gu[M, 2I], s[M, I]) with gu = x @ Wgu^T (gate rows [0, I), up rows [I, 2I)) and
    s = silu(gate) * up computed in the GEMM epilogue.  None if the shape does not tile
    (I % 96, M % 256, K % 128)."""
    M, K = x.shape
    I2 = wgu.shape[0]
    I = I2 // 2
    if not gemm_bf16_fits192(M, I2, K) or I2 % 2 or I % 96 or wgu.shape[1] != K:
        return None
    _req(x, torch.bfloat16, "gemm_gu_swiglu.x")
    _req(wgu, torch.bfloat16, "gemm_gu_swiglu.w")
    gu = torch.empty(M, I2, dtype=torch.bfloat16, device=x.device) if gu_out is None else gu_out
    s = torch.empty(M, I, dtype=torch.bfloat16, device=x.device) if s_out is None else s_out
    _req(gu, torch.bfloat16, "gemm_gu_swiglu.gu", M * I2)
    _req(s, torch.bfloat16, "gemm_gu_swiglu.s", M * I)
    _chk(lib().dlt_gemm_bf16_gu_swiglu(_p(x), _p(wgu), _p(gu), _p(s), M, I, K, _fwd_flags(), _stream()), "gemm_gu_swiglu")
    return gu, s


def gemm_dgrad(dy: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """dX[M, Nout] = dY[M, Nred] @ W[Nred, Nout] with W read as stored (the data gradient
    of a projection y = x @ W^T) by the hand-written persistent MFMA kernel in its
    reduction-major-B form; bf16 or fp16 (all three tensors one dtype).  None (nothing
    launched) when the shape does not tile (M % 256, Nout % 192, Nred % 128)."""
    M, Nred = dy.shape
    Nout = w.shape[1]
    if not gemm_bf16_fits(M, Nout, Nred) or w.shape[0] != Nred:
        return None
    dt = dy.dtype
    if dt not in _WG_HK:
        raise ValueError("gemm_dgrad: bf16 / fp16 operands expected")
    _req(dy, dt, "gemm_dgrad.dy")
    _req(w, dt, "gemm_dgrad.w")
    c = torch.empty(M, Nout, dtype=dt, device=dy.device) if out is None else out
    _req(c, dt, "gemm_dgrad.out", M * Nout)
    _chk(lib().dlt_gemm_bf16_nn(_p(dy), _p(w), _p(c), M, Nout, Nred, Nred, Nout, Nout, _GB_FLAGS, _WG_HK[dt],
                                _stream()), "gemm_dgrad")
    return c


def gemm_down_swiglu_bwd(dd: torch.Tensor, wdown: torch.Tensor, gu: torch.Tensor,
                         out: Optional[torch.Tensor] = None, s_out: Optional[torch.Tensor] = None
                         ) -> Optional[torch.Tensor]:
    """dgu[M, 2I] = SwiGLU backward of ds = dd[M, H] @ Wdown[H, I] (bf16-rounded) against
    the kept gu[M, 2I] -- the down projection's data gradient and ``swiglu_bwd`` in one
    kernel (same math and roundings as the unfused pair).  ``s_out`` [M, I] (optional):
    also writes s = silu(g) * u with the forward's bits (``swiglu_bwd``'s s_out).  None
    if it does not tile."""
    M, H = dd.shape
    I = wdown.shape[1]
    if not gemm_bf16_fits192(M, I, H) or wdown.shape[0] != H or tuple(gu.shape) != (M, 2 * I):
        return None
    dt = dd.dtype if dd.dtype in _WG_HK else torch.bfloat16  # bf16 or fp16, one format for all
    _req(dd, dt, "gemm_down_swiglu_bwd.dd")
    _req(wdown, dt, "gemm_down_swiglu_bwd.w")
    _req(gu, dt, "gemm_down_swiglu_bwd.gu")
    c = torch.empty(M, 2 * I, dtype=dt, device=dd.device) if out is None else out
    _req(c, dt, "gemm_down_swiglu_bwd.out", M * 2 * I)
    if s_out is not None:
        _req(s_out, dt, "gemm_down_swiglu_bwd.s_out", M * I)
    _chk(lib().dlt_gemm_bf16_down_swiglu_bwd(_p(dd), _p(wdown), _p(gu), _p(c), _p(s_out), M, I, H, _GB_FLAGS,
                                             _WG_HK[dt], _stream()), "gemm_down_swiglu_bwd")
    return c


def scale_bf16(x: torch.Tensor, scale: torch.Tensor, out: Optional[torch.Tensor] = None,
               mul: float = 1.0) -> torch.Tensor:
    """y = x * scale * mul with a device scalar (no host sync) and a host factor, x bf16
    or fp16; falls back for odd sizes."""
    if x.dtype == torch.float32:
        from . import hip_f32
        return hip_f32.scale(x, scale, out=out, mul=mul)
    hk = _req_act(x, x.dtype, "scale_bf16.x")
    s = scale.reshape(1).float().contiguous()
    if x.numel() % 8:
        y = (x.float() * s * mul).to(x.dtype)
        return y if out is None else out.copy_(y)
    y = torch.empty_like(x) if out is None else out
    _req(y, x.dtype, "scale_bf16.out", x.numel())
    _chk(lib().dlt_scale_bf16(_p(x), _p(y), x.numel(), _p(s), float(mul), hk, _stream()), "scale_bf16")
    return y
