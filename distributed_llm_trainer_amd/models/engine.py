"""Hand-scheduled forward/backward executor for the GPT block stack.

The reference runs the model through PyTorch autograd with dozens of small ATen
kernels per layer (``gpt.py:388-455``; op list in SURVEY §2.5).  This engine instead
issues a fixed schedule of fused HIP kernels + hipBLASLt GEMMs per layer and writes
weight gradients straight into fp32 flat gradient buffers ("main grads"), which is
what lets the DDP/FSDP runtimes in ``parallel/`` overlap RCCL collectives with the
remaining backward at layer granularity (hooks below) instead of relying on
autograd-hook bucketing.

Per layer (M = B*S rows, residual stream kept in fp32 like the reference's DDP
autocast path):

  fwd:  x,n1   = add_dropout_rmsnorm(r, d_prev)        [fused kernel]
        qkv    = n1 @ Wqkv^T                             [GEMM, N = 3H]
        qkv    = rope_qk(qkv)  (q, k rotated in place)   [fused kernel]
        o,lse  = flash_attention(qkv; causal, dropout)   [MFMA kernel, reads the packed
                                                          [M, 3H] GEMM output directly]
        a      = o @ Wo^T                                [GEMM]
        x2,n2  = add_dropout_rmsnorm(x, a)               [fused kernel]
        gu     = n2 @ Wgu^T                              [GEMM, N = 2I]
        s      = silu(g) * u                             [fused kernel]
        d      = s @ Wdown^T                             [GEMM]  -> (x2, d) to next layer
  head: xf,nf  = add_dropout_rmsnorm(x2, d); logits = nf @ E^T; CE + dlogits in place.

  The attention backward writes dq/dk/dv straight into the packed [M, 3H] gradient
  with the inverse RoPE rotation applied in its epilogue (no repack kernel).

Dropout masks are pure functions of (seed, micro-step, layer, site, index)
(``ops/rng.py``), so activation checkpointing just re-runs the layer forward.
Checkpointing is selective by default (``DLT_AC_SELECTIVE=0``: the reference's whole-
block recompute from the block input): besides the block input the forward keeps the
attention output o (bf16), its LSE + keep bits and the mid-block residual x2 (fp32),
so the backward recomputes only norm -> QKV GEMM -> RoPE and norm -> gate/up GEMM ->
SwiGLU, and skips the attention forward and the o / down GEMMs -- 31 % of the block's
GEMM FLOPs plus the attention kernels, for ~3.5x the saved bytes of the block input.

Micro-step pipelining (:meth:`GPTEngine.train_window`): within a gradient-accumulation
window the forward of micro-step k+1 does not depend on the backward of micro-step k
(weights only change at the optimizer step), so the two are issued block by block on
two HIP streams and the GPU overlaps them -- the small-N GEMMs, the 1.5-waves/SIMD
attention grid and the memory-bound norm/SwiGLU kernels of one chain fill the CUs the
other leaves idle.  The reference runs the micro-steps strictly one after the other
(``ddp_trainer.py:322-345``).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional

import torch

from ..ops import rng


def _drain(gen):
    """Run a generator to completion and return its return value."""
    while True:
        try:
            next(gen)
        except StopIteration as stop:
            return stop.value


@dataclass
class LayerWeights:
    wqkv: torch.Tensor   # [3H, H] compute dtype (rows: q | k | v)
    wo: torch.Tensor     # [H, H]
    wgu: torch.Tensor    # [2I, H] (rows: gate | up)
    wdown: torch.Tensor  # [H, I]
    ln1: torch.Tensor    # [H]
    ln2: torch.Tensor    # [H]


@dataclass
class LayerGrads:
    wqkv: torch.Tensor   # fp32, accumulated in place
    wo: torch.Tensor
    wgu: torch.Tensor
    wdown: torch.Tensor
    ln1: torch.Tensor
    ln2: torch.Tensor


@dataclass
class HeadWeights:
    embed: torch.Tensor      # [V or Vp, H] gather table (fp32 master or gathered bf16)
    lm_head: torch.Tensor    # [Vp, H] compute dtype, rows >= V are zero
    norm: torch.Tensor       # [H]


@dataclass
class HeadGrads:
    embed: torch.Tensor      # [Vp, H] fp32 (tied: lm_head wgrad + embedding scatter-add)
    norm: torch.Tensor       # [H] fp32


class ParamProvider:
    """Interface the engine uses to fetch weights / gradient sinks and fire hooks.

    Implemented by ``parallel.flat.FlatParamStore`` (single GPU / DDP) and by
    ``parallel.fsdp.FSDPRuntime`` (sharded units).  Unit ids: ``"head"`` for the
    root unit (embedding, tied lm_head, final norm) and ``0..L-1`` for blocks.
    """

    def layer(self, i: int) -> LayerWeights: ...
    def layer_grads(self, i: int) -> LayerGrads: ...
    def head(self) -> HeadWeights: ...
    def head_grads(self) -> HeadGrads: ...

    # hooks -- default no-ops
    def pre_forward(self, unit) -> None: pass
    def post_forward(self, unit) -> None: pass
    def pre_backward(self, unit) -> None: pass
    def post_backward(self, unit) -> None: pass


def shift_targets(labels: torch.Tensor) -> torch.Tensor:
    """labels [B,S] -> per-row targets [B*S]: labels[b, s+1], IGNORE at s = S-1.

    Equivalent to the reference's ``logits[:, :-1]`` / ``labels[:, 1:]`` shift
    (``gpt.py:451-453``) without materialising shifted logits.
    """
    B, S = labels.shape
    t = torch.full((B, S), -100, dtype=torch.int64, device=labels.device)
    t[:, :-1] = labels[:, 1:]
    return t.reshape(-1)


@dataclass
class _LayerCache:
    x: torch.Tensor
    rstd1: Any = None
    n1: Any = None
    q: Any = None      # packed path: the roped [M, 3H] qkv (k, v = None)
    k: Any = None
    v: Any = None
    o: Any = None
    lse: Any = None
    x2: Any = None
    rstd2: Any = None
    n2: Any = None
    gu: Any = None
    s: Any = None


@dataclass
class _StepState:
    ids: torch.Tensor
    B: int
    S: int
    micro: int
    train: bool
    recompute: bool
    caches: List[_LayerCache] = field(default_factory=list)
    slot: int = 0          # micro-step index within the gradient-accumulation window
    defer: bool = False    # weight grads deferred to the last micro-step of the window
    last: bool = True
    xf: Any = None
    rstdf: Any = None
    nf: Any = None
    dlogits: Any = None
    ce_scale: float = 1.0
    head_key: int = 0   # which per-stream lm_head buffers (chunk logits, fp32 wgrad) it uses
    head_rows: Any = None  # the lm_head row chunks [(r0, r1), ...] (chunked head)
    dnf: Any = None     # early head: d(final norm output), computed in the forward
    head_acc: Any = None  # chunked head: this micro-step's fp32 lm_head weight gradient
    d_last: Any = None  # bf16 d of last layer (input of final norm)


class GPTEngine:
    def __init__(self, cfg, provider: ParamProvider, ops, act_dtype=torch.bfloat16,
                 seed: int = 1234, eps: float = 1e-6, gemm=None):
        self.cfg = cfg
        self.provider = provider
        self.ops = ops
        self.act_dtype = act_dtype
        self.seed = int(seed) & 0xFFFFFFFF
        self.eps = eps
        self.micro_counter = 0
        # fp16: the cross-entropy gradient is stored pre-multiplied by this factor (the
        # trainer's loss scale) so it does not underflow; the backward divides it out
        # where it applies dloss (the lm_head weight / data gradients)
        self.ce_grad_scale = 1.0
        self.gemm = gemm or _TorchGemm()
        self._rope = {}
        # dropout probabilities (zeroed in eval mode)
        self.p_attn = float(cfg.attention_dropout)
        self.p_hidden = float(cfg.dropout)
        # deferred weight gradients (see set_accumulation)
        self.acc_slot, self.acc_slots, self.defer = 0, 1, False
        # which weight gradients a deferred window defers (the others run per micro-step):
        # all by default; the memory-lean mode defers none (per-chain weight gradients)
        self.defer_roles = frozenset(self.ROLES)
        self.defer_layers = int(os.environ.get("DLT_DEFER_LAYERS", "0"))  # see _deferred
        self._slots = {}
        # dY-operand slot ring (ffbb window, see _window_ffbb): 0 = one slot per layer
        self._ring = 0
        self._ring_done = {}
        # DLT_S_RING=1: with the dY ring on, the SwiGLU output s (the down projection's
        # weight-gradient operand) joins it too -- the backward rewrites it (same bits; the
        # fused down-dgrad epilogue's s_out) and the forward's copy is a temporary: R slots
        # instead of one [2M, I] slot per layer, -1.8 GB at the headline shape.  Off by
        # default since the SwiGLU backward moved into the down-dgrad GEMM epilogue, where
        # the extra s stores cost the step 1.2-1.5 % (785.2k vs 797.1k tok/s, three same-box
        # pairs; profiles/r4_memory_lean.md)
        self.s_ring = os.environ.get("DLT_S_RING", "0") == "1"
        # memory-first (--memory_first): when the down projection's weight gradient runs in
        # each micro-step's own backward (not deferred), the SwiGLU output s is not kept
        # from the forward; the SwiGLU backward (fused into the down data gradient)
        # rewrites it from the kept gu with the forward's arithmetic -- same bits -- for
        # the down weight gradient (-100 MB per layer per 16k-token chain)
        self.s_refill = os.environ.get("DLT_S_REFILL", "0") == "1"
        # lm_head + cross-entropy in row chunks (head_chunks > 0; 0 = the window's logits
        # stay resident for ONE lm_head weight-gradient GEMM over all its rows, on the
        # side stream during the backward).  Per micro-step, for each chunk of rows:
        # logits GEMM, CE (gradient in place), the lm_head data gradient and the weight
        # gradient into a private fp32 buffer, added to the tied embedding gradient after
        # the micro-step's embedding scatter-add.  In train_window (dloss known up front)
        # the forward runs all of it ("early head") through ONE [M / chunks, V] logits
        # buffer instead of a [GA * M, V] window slot: headline peak 21.4 -> 19.0 GB, but
        # -3.5 % tok/s (the lm_head weight gradient no longer overlaps the backward;
        # profiles/r4_memory.md), so it is the memory-lean modes' choice (the DDP trainer
        # sets 2 with --memory_lean).  DLT_HEAD_CHUNKS=n overrides.
        env_chunks = os.environ.get("DLT_HEAD_CHUNKS")
        self.head_chunks_env = env_chunks is not None
        self.head_chunks = max(0, int(env_chunks)) if env_chunks is not None else 0
        # ... and the micro-steps of a window share ONE chunk logits buffer (DLT_HEAD_SHARE,
        # default on): a micro-step's early head waits for the previous one's (a device-side
        # event wait; the other chain's layers keep the GPU busy meanwhile)
        self.head_share = os.environ.get("DLT_HEAD_SHARE", "1") != "0"
        self._head_lg = {}   # head_key (0 when shared) -> chunk logits buffer
        self._head_lg_ev = None  # shared buffer: the last early head's completion event
        self._head_accs = {}  # head_key -> fp32 [V, H] weight-gradient buffer
        self._side = None  # weight-gradient side stream (lazily created)
        self._mask_side = None  # attention keep-bit side stream
        self._pipe = None  # second compute stream of train_window
        self.queue_placement = None  # how the side streams were placed (_place_streams)
        self.last_window = None  # schedule of the last train_window ("ffbb" | "fb")
        self.window_auto = None  # trial state of the timed fb / ffbb choice under collectives
        # attention straight on the packed [M, 3H] QKV GEMM output (RoPE in place,
        # inverse RoPE in the backward epilogue); DLT_PACKED_QKV=0 -> split q/k/v copies
        self.packed_qkv = (hasattr(ops, "attention_fwd_packed")
                           and os.environ.get("DLT_PACKED_QKV", "1") != "0")
        # last layers of the deferred-wgrad backward whose weight gradients run on the
        # current stream instead of the side stream (see _backward_gen)
        self.main_wgrad_layers = int(os.environ.get("DLT_MAIN_WGRAD_LAYERS", "1"))
        # micro-step fusion (set_loss_segments): a training forward of B rows holds this
        # many micro-steps of B / n rows each, every one with its own loss normalisation
        self.loss_segments = 1
        # activation checkpointing: keep o / lse / x2 too and skip the attention forward
        # and the o / down GEMMs in the recompute (see the module docstring)
        self.selective_recompute = os.environ.get("DLT_AC_SELECTIVE", "1") != "0"
        # ... and, within this many bytes of kept GEMM outputs, the packed QKV and gate/up
        # GEMM outputs as well, so the recompute reduces to the norms and SwiGLU (sized for
        # 288 GB of HBM: GPT-2 small/medium/xl keep both; see _ac_keep)
        # (default: a third of the GPU's memory -- 96 GB of MI355X's 288 GB: FSDP xl then
        # keeps both GEMM outputs, 55.6k -> 61.3k tok/s at 68.8 -> 88.6 GB; 48 GB off-GPU)
        env_budget = os.environ.get("DLT_AC_BUDGET_GB")
        if env_budget is not None:
            self.ac_budget = float(env_budget) * 1e9
        elif torch.cuda.is_available():
            self.ac_budget = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory / 3.0
        else:
            self.ac_budget = 48e9
        # attention keep-bit masks (1 bit per causal score, two layouts) are kept from the
        # forward for the backward while one micro-step's masks of all layers fit in this
        # budget; beyond it (long context: 3.2 GB per layer at S = 32768, nh 12) the
        # backward regenerates each layer's bits (one extra VALU kernel per layer)
        self.attn_mask_budget = float(os.environ.get("DLT_ATTN_MASK_BUDGET_GB", "32")) * 1e9

    def set_loss_segments(self, n: int) -> None:
        """Declare that each training forward carries ``n`` fused micro-steps.

        The rows split into ``n`` equal segments; each segment's cross-entropy is a mean
        over ITS valid targets, and the forward's loss is the mean of the segment
        losses -- so a chain of F fused micro-steps contributes exactly what F separate
        micro-steps contribute to the reference's ``sum_k loss_k / GA`` (also with
        ignore_index rows, whose count differs per micro-step)."""
        self.loss_segments = max(1, int(n))

    # ------------------------------------------------------- grad accumulation
    def set_accumulation(self, slot: int, n_slots: int, defer: bool = True) -> None:
        """Declare micro-step ``slot`` of an ``n_slots``-step accumulation window.

        With ``defer`` the GEMM inputs of every weight gradient (the normed/attention/
        SwiGLU activations and the output gradients) are written by their producing
        kernels straight into per-layer ``[n_slots*M, N]`` buffers, and each weight
        gradient is ONE GEMM over all ``n_slots*M`` rows at the last micro-step instead
        of ``n_slots`` GEMMs over M rows: same sum, but the K=B*S reductions of the
        small [768 x 768]-class outputs run ~1.4x faster at 4x the length (measured,
        tools/wgrad_m_test.py).  Memory: ~250 MB per layer per micro-step (small).
        """
        self.acc_slot, self.acc_slots = int(slot), int(n_slots)
        # A one-micro-step window defers too (DLT_DEFER_GA1=0: inline wgrads): the slot
        # buffers then let the weight-gradient GEMMs run on the side stream, overlapped
        # with the next layer's dgrad chain (attention/norm/SwiGLU backward).
        self.defer = bool(defer) and (n_slots > 1 or os.environ.get("DLT_DEFER_GA1", "1") != "0")

    # slot-buffer name -> the weight gradient it feeds (X or dY operand)
    _SLOT_ROLE = {"n1": "qkv", "dqkv": "qkv", "o": "o", "da": "o", "n2": "gu", "dgu": "gu", "s": "down", "dd": "down",
                  "lg": "head", "nf": "head"}
    ROLES = ("qkv", "o", "gu", "down", "head")

    def _deferred(self, st, role: str, layer=None) -> bool:
        if role == "head" and self.head_chunks > 0:
            return False  # the chunked head computes its weight gradient per micro-step
        d = st.defer and role in self.defer_roles
        # defer_layers > 0: only layers below it defer their roles (a memory / speed dial
        # between "none" and a whole role, e.g. --memory_first --defer_roles o); the
        # ffbb dY ring assumes whole roles, so it ignores the dial
        if d and layer is not None and 0 < self.defer_layers <= layer and not self._ring:
            return False
        return d

    def _sb(self, st, layer, name: str, M: int, N: int, device):
        """The micro-step's slice of a slot buffer when ``name``'s weight gradient is
        deferred, else None (the producing kernel allocates as usual)."""
        if not self._deferred(st, self._SLOT_ROLE[name], layer):
            return None
        return self._slot_buf(st, layer, name, M, N, device)[0]

    # slot buffers written by the backward (the dY operands of the deferred weight gradients)
    _DY_SLOTS = frozenset(("dqkv", "da", "dgu", "dd"))

    def _ring_name(self, name: str) -> bool:
        return name in self._DY_SLOTS or (name == "s" and self.s_ring)

    def _s_in_ring(self, st) -> bool:
        """The SwiGLU output lives in the slot ring (written by the backward), not in a
        per-layer slot from the forward."""
        return bool(self._ring) and self.s_ring and self._deferred(st, "down")

    def _refill_s(self, st) -> bool:
        """s is rewritten by the backward instead of kept (s_refill, see __init__)."""
        return self.s_refill and not st.recompute and not self._deferred(st, "down")

    def _slot_buf(self, st, layer, name: str, M: int, N: int, device):
        # ffbb ring: the dY operands of layer i live in ring slot i % R (see _window_ffbb)
        key = (("ring", layer % self._ring), name) if self._ring and self._ring_name(name) else (layer, name)
        buf = self._slots.get(key)
        if buf is None or buf.shape != (self.acc_slots * M, N) or buf.device != device:
            if buf is not None and buf.is_cuda:
                # slot buffers are shared by the compute, pipeline and weight-gradient
                # streams without record_stream: retire every user before reuse
                torch.cuda.synchronize(buf.device)
            buf = torch.empty(self.acc_slots * M, N, dtype=self.act_dtype, device=device)
            self._slots[key] = buf
        return buf[st.slot * M:(st.slot + 1) * M], buf

    def release_slots(self) -> None:
        bufs = list(self._slots.values()) + list(self._head_lg.values()) + list(self._head_accs.values())
        if any(b.is_cuda for b in bufs):
            torch.cuda.synchronize()
        self._slots.clear()
        self._head_lg.clear()
        self._head_accs.clear()
        self._head_lg_ev = None

    # ---------------------------------------------------------------- chunked head
    def _head_rows(self, M: int, nseg: int):
        """Row chunks of the lm_head (never straddling a loss segment)."""
        seg = M // nseg
        per = max(1, self.head_chunks // nseg)
        while per > 1 and seg % per:
            per -= 1
        step = seg // per
        return [(k * seg + j * step, k * seg + (j + 1) * step) for k in range(nseg) for j in range(per)]

    def _head_buf(self, cache: dict, key, shape, dtype, device):
        buf = cache.get(key)
        if buf is None or tuple(buf.shape) != tuple(shape) or buf.dtype != dtype or buf.device != device:
            if buf is not None and buf.is_cuda:
                torch.cuda.synchronize(buf.device)  # shared across streams without record_stream
            buf = torch.empty(shape, dtype=dtype, device=device)
            cache[key] = buf
        return buf

    def _nf_scaled(self, nf, dloss, inv_ce, out=None):
        if nf.dtype in (torch.bfloat16, torch.float16):
            return self.ops.scale_bf16(nf, dloss, out=out, mul=inv_ce)
        r = nf * (dloss * inv_ce)
        return out.copy_(r) if out is not None else r

    def _head_chunk_bwd(self, dl, w, dnf_out, acc, nfs, first: bool) -> None:
        """One row chunk of the lm_head backward: dnf rows = dl @ E, acc (+)= dl^T @ nfs."""
        self.gemm.linear_dgrad(dl, w, out=dnf_out)
        if first:
            acc.zero_()
        self.gemm.wgrad_acc(acc, dl, nfs)

    # ---------------------------------------------------------------- helpers
    def rope(self, S: int, device):
        key = (S, str(device))
        if key not in self._rope:
            self._rope[key] = self.ops.rope_tables(self.cfg.head_dim, max(S, self.cfg.max_seq_len), device=device)
        return self._rope[key]

    def _keys(self, micro: int, layer: int):
        return (rng.site_key(self.seed, micro, layer, rng.SITE_ATTN),
                rng.site_key(self.seed, micro, layer, rng.SITE_RESID),
                rng.site_key(self.seed, micro, layer, rng.SITE_MLP))

    # ---------------------------------------------------------------- forward
    def _attn_mask_async(self, B, S, p, key, dev):
        """(mask, ready-event) built on a side stream (opt-in, ``DLT_MASK_STREAM=1``), or
        (None, None) to let the attention launch build it inline.  Measured neutral on
        the headline config (the GPU is saturated either way), so off by default."""
        if (p <= 0.0 or dev.type != "cuda" or not hasattr(self.ops, "attention_dropout_mask")
                or os.environ.get("DLT_MASK_STREAM", "0") != "1"):
            return None, None
        if self._mask_side is None:
            self._mask_side = torch.cuda.Stream(dev)
        main = torch.cuda.current_stream()
        # allocated from the side stream's own pool: no wait on main needed, so the
        # masks of later layers can be produced while earlier layers still compute
        with torch.cuda.stream(self._mask_side):
            mask = self.ops.attention_dropout_mask(B, self.cfg.num_heads, S, p, key, device=dev)
            ev = torch.cuda.Event()
            ev.record()
        mask.record_stream(main)
        return mask, ev

    def _ac_keep(self, M: int):
        """(keep_qkv, keep_gu, keep_rest) under activation checkpointing: tensors kept
        instead of recomputed, greedily by recompute time saved per byte -- the QKV GEMM
        output, the gate/up GEMM output, then the two normed inputs and the SwiGLU output
        (memory-bound recomputes: 3 bytes of traffic per byte kept) -- while every layer of
        the two micro-steps a pipelined window holds fits in ``ac_budget``.  With all
        three nothing is recomputed.  Whole-block recompute (``DLT_AC_SELECTIVE=0``) keeps
        nothing."""
        if not self.selective_recompute:
            return False, False, False
        cfg = self.cfg
        per_layer_chains = cfg.num_layers * 2 * (2 if self.act_dtype == torch.bfloat16 else 4)
        qkv = M * 3 * cfg.hidden_size * per_layer_chains
        gu = M * 2 * cfg.intermediate_size * per_layer_chains
        rest = M * (2 * cfg.hidden_size + cfg.intermediate_size) * per_layer_chains
        keep_qkv = qkv <= self.ac_budget
        keep_gu = keep_qkv and qkv + gu <= self.ac_budget
        keep_rest = keep_gu and qkv + gu + rest <= self.ac_budget and os.environ.get("DLT_AC_KEEP_REST", "1") != "0"
        return keep_qkv, keep_gu, keep_rest

    def _layer_forward(self, st: _StepState, i: int, r, d, key_d: int, p_d: float,
                       save: bool):
        ops, gm, cfg = self.ops, self.gemm, self.cfg
        B, S = st.B, st.S
        w = self.provider.layer(i)
        pa = self.p_attn if st.train else 0.0
        ph = self.p_hidden if st.train else 0.0
        k_attn, k_resid, k_mlp = self._keys(st.micro, i)
        cos, sin = self.rope(S, r.device)

        M, H, I = B * S, cfg.hidden_size, cfg.intermediate_size
        dv = r.device
        sb = lambda name, n: self._sb(st, i, name, M, n, dv)  # noqa: E731
        # attention keep-bits depend only on the RNG key: build them on a side stream
        # so the VALU-only hashing overlaps the norm + QKV GEMM + RoPE below
        mask, mask_ev = self._attn_mask_async(B, S, pa, k_attn, dv)
        x, n1, rstd1 = ops.add_dropout_rmsnorm_fwd(r, d, w.ln1, self.eps, p_d, key_d, self.act_dtype,
                                                   y_out=sb("n1", H))
        fused_rope = self.packed_qkv and hasattr(gm, "linear_rope")
        if fused_rope:  # QKV GEMM with RoPE on q/k in its epilogue (when that races faster)
            qkv = gm.linear_rope(n1, w.wqkv, B, S, cfg.num_heads, cos, sin, ops)
        else:
            qkv = gm.linear(n1, w.wqkv)
        if mask is not None:
            torch.cuda.current_stream().wait_event(mask_ev)
        kw = {"mask": mask} if mask is not None else {}
        if pa > 0.0 and getattr(ops, "backend", "") == "hip" and getattr(ops, "attn_backend", "hip") in ("hip", "gemm"):
            # keep this layer's keep bits for the backward only within the memory budget.
            # The masks (two layouts, 1 bit per causal score: 8 * B * nh * S * ceil(S/32) B)
            # grow with S^2, the saved block input (M * H * 4 B) with S: under activation
            # checkpointing they are kept only while they cost at most as much as that
            # input (S <= ~1k at GPT-2 shapes), so turning recompute on never keeps MORE
            # than it saves (at S = 16k the masks are ~16x the input); the backward then
            # regenerates them (one VALU kernel per layer, bit-identical bits).
            mask_bytes = 8 * B * cfg.num_heads * S * ((S + 31) // 32)
            keep = mask_bytes * cfg.num_layers <= self.attn_mask_budget
            if st.recompute:
                keep = keep and mask_bytes <= M * H * 4
            kw["store_mask"] = keep
        if self.packed_qkv:
            if not fused_rope:
                ops.rope_qk_inplace(qkv, B, S, cfg.num_heads, cos, sin)
            o, lse = ops.attention_fwd_packed(qkv, B, S, cfg.num_heads, pa, k_attn, out=sb("o", H), **kw)
            q, k, v = qkv, None, None
        else:
            q, k, v = ops.rope_qkv_fwd(qkv, B, S, cfg.num_heads, cos, sin)
            o, lse = ops.attention_fwd(q, k, v, pa, k_attn, True, out=sb("o", H), **kw)
        del qkv
        a = gm.linear(o, w.wo)
        x2, n2, rstd2 = ops.add_dropout_rmsnorm_fwd(x, a, w.ln2, self.eps, ph, k_resid, self.act_dtype,
                                                    y_out=sb("n2", H))
        del a
        s_ring = self._s_in_ring(st)  # s is a temporary: the backward refills its ring slot
        s_slot = None if s_ring else sb("s", I)
        if hasattr(gm, "linear_swiglu"):  # gate/up GEMM with SwiGLU in its epilogue (when faster)
            gu, s = gm.linear_swiglu(n2, w.wgu, ops, s_out=s_slot)
        else:
            gu = gm.linear(n2, w.wgu)
            s = ops.swiglu_fwd(gu, out=s_slot)
        d_out = gm.linear(s, w.wdown)
        if s_ring or self._refill_s(st):
            s = None
        if save:
            c = _LayerCache(x=x, rstd1=rstd1, n1=n1, q=q, k=k, v=v, o=o, lse=lse,
                            x2=x2, rstd2=rstd2, n2=n2, gu=gu, s=s)
        elif st.recompute:
            if self.selective_recompute:
                keep_qkv, keep_gu, keep_rest = self._ac_keep(M)
                c = _LayerCache(x=x, o=o, lse=lse, x2=x2)
                if keep_qkv and self.packed_qkv:
                    c.q = q
                if keep_gu:
                    c.gu = gu
                if keep_rest and keep_qkv and self.packed_qkv:  # nothing left to recompute
                    c.n1, c.rstd1, c.n2, c.rstd2, c.s = n1, rstd1, n2, rstd2, s
            else:
                c = _LayerCache(x=x)
        else:
            c = None
        return x2, d_out, c

    def _layer_recompute(self, st: _StepState, i: int, c: _LayerCache) -> _LayerCache:
        """Activation-checkpoint recompute of layer ``i`` for the backward.  Whole-block
        recompute from the saved input, or (selective, the default) only the tensors the
        backward reads that were not kept: n1 / q(k, v) and n2 / gu / s (the QKV and
        gate/up GEMMs are skipped when the forward kept their outputs, _ac_keep).  Same kernels on
        the same inputs as the forward, so every recomputed tensor is bit-identical."""
        if c.o is None:
            return self._layer_forward(st, i, c.x, None, 0, 0.0, save=True)[2]
        if c.n1 is not None and c.s is not None and c.q is not None and c.gu is not None:
            return c  # the forward kept everything (_ac_keep within the budget)
        ops, gm, cfg = self.ops, self.gemm, self.cfg
        B, S = st.B, st.S
        w = self.provider.layer(i)
        cos, sin = self.rope(S, c.x.device)
        M, H, I = B * S, cfg.hidden_size, cfg.intermediate_size
        dv = c.x.device
        sb = lambda name, n: self._sb(st, i, name, M, n, dv)  # noqa: E731
        _, n1, rstd1 = ops.add_dropout_rmsnorm_fwd(c.x, None, w.ln1, self.eps, 0.0, 0, self.act_dtype,
                                                   y_out=sb("n1", H))
        if c.q is not None:  # QKV output kept by the forward (_ac_keep)
            qkv = c.q
            q, k, v = qkv, None, None
        elif self.packed_qkv and hasattr(gm, "linear_rope"):
            qkv = gm.linear_rope(n1, w.wqkv, B, S, cfg.num_heads, cos, sin, ops)
            q, k, v = qkv, None, None
        elif self.packed_qkv:
            qkv = gm.linear(n1, w.wqkv)
            ops.rope_qk_inplace(qkv, B, S, cfg.num_heads, cos, sin)
            q, k, v = qkv, None, None
        else:
            qkv = gm.linear(n1, w.wqkv)
            q, k, v = ops.rope_qkv_fwd(qkv, B, S, cfg.num_heads, cos, sin)
        del qkv
        _, n2, rstd2 = ops.add_dropout_rmsnorm_fwd(c.x2, None, w.ln2, self.eps, 0.0, 0, self.act_dtype,
                                                   y_out=sb("n2", H))
        s_ring = self._s_in_ring(st)  # the backward writes s into its ring slot
        if c.gu is not None:  # gate/up output kept by the forward (_ac_keep)
            gu = c.gu
            s = None if s_ring else ops.swiglu_fwd(gu, out=sb("s", I))
        elif hasattr(gm, "linear_swiglu"):
            gu, s = gm.linear_swiglu(n2, w.wgu, ops, s_out=None if s_ring else sb("s", I))
        else:
            gu = gm.linear(n2, w.wgu)
            s = None if s_ring else ops.swiglu_fwd(gu, out=sb("s", I))
        if s_ring:
            s = None
        return _LayerCache(x=c.x, rstd1=rstd1, n1=n1, q=q, k=k, v=v, o=c.o, lse=c.lse,
                           x2=c.x2, rstd2=rstd2, n2=n2, gu=gu, s=s)

    def forward(self, ids: torch.Tensor, targets: Optional[torch.Tensor], train: bool,
                recompute: bool = False, return_logits: bool = False,
                need_backward: Optional[bool] = None):
        """Returns (loss or None, logits or None, state for backward or None)."""
        return _drain(self._forward_gen(ids, targets, train, recompute, return_logits, need_backward))

    def _forward_gen(self, ids, targets, train, recompute=False, return_logits=False, need_backward=None,
                     acc=None, head_dloss=None):
        """Generator form of :meth:`forward`: yields after every block so the window
        scheduler (:meth:`train_window`) can interleave it with another micro-step's
        backward; the return value is forward's tuple.  ``acc`` = (slot, n_slots,
        defer) overrides the engine-global accumulation state.  ``head_dloss`` (the
        backward's dloss, known up front in train_window): run the chunked lm_head
        backward here ("early head", see head_chunks)."""
        B, S = ids.shape
        if need_backward is None:
            need_backward = torch.is_grad_enabled()
        need_bwd = bool(need_backward) and train and targets is not None
        if train:
            micro = self.micro_counter
            self.micro_counter += 1
        else:
            micro = 0
        st = _StepState(ids=ids, B=B, S=S, micro=micro, train=train, recompute=recompute)
        slot, n_slots, defer = acc if acc is not None else (self.acc_slot, self.acc_slots, self.defer)
        if need_bwd and defer:
            st.slot, st.defer, st.last = slot, True, slot == n_slots - 1
        st.head_key = slot % 2  # micro-steps of a window alternate between two streams by parity
        prov = self.provider
        ph = self.p_hidden if train else 0.0

        prov.pre_forward("head")
        hw = prov.head()
        r = self.ops.embedding_fwd(ids, hw.embed)
        d, key_d, p_d = None, 0, 0.0
        for i in range(self.cfg.num_layers):
            prov.pre_forward(i)
            save = need_bwd and not recompute
            r_new, d_new, c = self._layer_forward(st, i, r, d, key_d, p_d, save)
            if need_bwd:
                st.caches.append(c)
            prov.post_forward(i)
            r, d = r_new, d_new
            key_d, p_d = self._keys(micro, i)[2], ph
            yield
        hw = prov.head()
        xf, nf, rstdf = self.ops.add_dropout_rmsnorm_fwd(r, d, hw.norm, self.eps, p_d, key_d, self.act_dtype)
        st.d_last = None
        loss, logits = None, None
        V, Vp = self.cfg.vocab_size, hw.lm_head.shape[0]
        if targets is not None:
            rows = B * S
            nseg = self.loss_segments if (train and B % self.loss_segments == 0) else 1
            # fused micro-steps: per-segment normalisation (see set_loss_segments); the
            # gradient of (1/nseg) * mean_k: the CE kernel divides by its count argument
            segs = [(k * rows // nseg, (k + 1) * rows // nseg) for k in range(nseg)]
            if nseg == 1:
                nvs = [(targets != -100).sum()]
                norms = nvs
            else:
                nvs = [(targets[a:b] != -100).sum() for a, b in segs]
                norms = [nv * nseg for nv in nvs]
            chunked = need_bwd and self.head_chunks > 0
            if chunked:
                st.head_rows = self._head_rows(rows, nseg)
            if chunked and head_dloss is not None:
                # early head: per row chunk, logits -> CE (gradient in place) -> the lm_head
                # data gradient and weight gradient, through one chunk-sized logits buffer
                H = self.cfg.hidden_size
                rc = max(b - a for a, b in st.head_rows)
                lg_buf = self._head_buf(self._head_lg, 0 if self.head_share else st.head_key, (rc, Vp), nf.dtype,
                                        nf.device)
                if self.head_share and self._head_lg_ev is not None:
                    torch.cuda.current_stream().wait_event(self._head_lg_ev)
                hacc = self._head_buf(self._head_accs, st.head_key, tuple(hw.lm_head.shape), torch.float32,
                                      nf.device)
                dnf = torch.empty(rows, H, dtype=nf.dtype, device=nf.device)
                nfs = self._nf_scaled(nf, head_dloss.reshape(()).float(), 1.0 / self.ce_grad_scale)
                parts = []
                for ci, (a, b) in enumerate(st.head_rows):
                    lg = self.gemm.linear(nf[a:b], hw.lm_head, out=lg_buf[:b - a])
                    parts.append(self.ops.cross_entropy_fwd_bwd(lg, targets[a:b], V, norms[a * nseg // rows],
                                                                self.ce_grad_scale))
                    self._head_chunk_bwd(lg, hw.lm_head, dnf[a:b], hacc, nfs[a:b], ci == 0)
                del nfs
                if self.head_share and lg_buf.is_cuda:
                    self._head_lg_ev = torch.cuda.Event()
                    self._head_lg_ev.record()
                row_loss = parts[0] if len(parts) == 1 else torch.cat(parts)
                st.dnf, st.head_acc = dnf, hacc
            else:
                # [M, Vp]; with the window-deferred head (head_chunks 0) the logits
                # (-> dlogits) of every micro-step stay resident for ONE lm_head wgrad GEMM
                lg_out = self._sb(st, "head", "lg", rows, Vp, nf.device)
                lg = self.gemm.linear(nf, hw.lm_head, out=lg_out)
                if nseg == 1:
                    row_loss = self.ops.cross_entropy_fwd_bwd(lg, targets, V, norms[0], self.ce_grad_scale)
                else:
                    row_loss = torch.cat([self.ops.cross_entropy_fwd_bwd(lg[a:b], targets[a:b], V, norms[k],
                                                                         self.ce_grad_scale)
                                          for k, (a, b) in enumerate(segs)])
                if need_bwd:
                    st.dlogits = lg  # now holds ce_grad_scale * d(mean loss)/d(logits)
            if nseg == 1:
                loss = row_loss.sum() / nvs[0].clamp(min=1).float()
            else:
                loss = torch.stack([row_loss[a:b].sum() / nvs[k].clamp(min=1).float()
                                    for k, (a, b) in enumerate(segs)]).mean()
            if need_bwd:
                st.ce_scale = self.ce_grad_scale
                st.xf, st.rstdf, st.nf = xf, rstdf, nf
        if return_logits or targets is None:
            lg2 = self.gemm.linear(nf, hw.lm_head)
            logits = lg2[:, :V].reshape(B, S, V)
        prov.post_forward("head")
        return loss, logits, (st if need_bwd else None)

    # --------------------------------------------------------------- backward
    def _wgrad_stream(self, dev):
        """Side HIP stream for the deferred weight-gradient GEMMs (None = run inline).

        Only with a provider whose gradient hooks are stream-safe (the flat store /
        DDP runtime) and a GEMM backend with per-stream workspaces."""
        if not self._side_wanted(dev):
            return None
        self._place_streams(dev)
        return self._side

    def _side_wanted(self, dev) -> bool:
        return (dev.type == "cuda" and os.environ.get("DLT_WGRAD_STREAM", "1") != "0"
                and getattr(self.provider, "side_stream_hooks", False) and getattr(self.gemm, "stream_safe", False))

    def _place_streams(self, dev) -> None:
        """Create the weight-gradient and pipeline streams, each on a hardware queue that
        dispatches independently of the current stream's and of each other's.

        HIP binds a stream to a hardware queue at its first dispatch, round-robin, and a
        queue that shares a command-processor pipe with another cannot dispatch while the
        other's kernel is still placing workgroups -- a big GEMM holds the pipe for most of
        its run, so two chains on such queues serialise (the ffbb window fell from 800k to
        693k tok/s when a communicator's streams shifted the engine's queues, and to 696k
        with one idle stream created first: profiles/r5_stream_queues.md).
        DLT_QUEUE_PROBE=1 probes each new stream: a long many-workgroup kernel on an
        already placed stream, a one-workgroup kernel on the candidate; if the candidate's
        kernel cannot finish before the long one does, the candidate is parked (its queue
        stays taken) and the next stream, bound to the next queue, is tried.  Opt-in: on a
        forced RCCL rank the probe found no blocked pair, yet ffbb still collapsed (706k)
        and binding the side streams before the communicator's first collective cost fb
        9 % (718k vs 789k), so by default the streams stay unbound until their first use
        and collectives keep the fb window.  DLT_QUEUE_PAD=n creates n idle streams first
        (forced RCCL rank, ffbb: 797k with n = 3)."""
        if self._pipe is not None:
            return
        want_side = self._side_wanted(dev)
        pad = os.environ.get("DLT_QUEUE_PAD")
        if pad is None and self.window_auto is not None:
            pad = "3"  # the timed fb / ffbb choice (window_schedule): ffbb's measured placement
        if pad is not None or os.environ.get("DLT_QUEUE_PROBE", "0") != "1":
            _queue_pad(dev, int(pad or 0))
            # created unbound: each binds its hardware queue at its first dispatch
            self._side = torch.cuda.Stream(dev) if want_side else None
            self._pipe = torch.cuda.Stream(dev)
            self.queue_placement = {"probe": False, "pads": int(pad or 0), "verified": False}
            return
        main = torch.cuda.current_stream(dev)
        big = torch.zeros(64 << 20, dtype=torch.float32, device=dev)  # 256 MiB: ~16k workgroups per pass
        tiny = torch.zeros(8, dtype=torch.float32, device=dev)

        def fresh():
            st = torch.cuda.Stream(dev)
            with torch.cuda.stream(st):
                tiny.add_(0.0)  # first dispatch: binds the hardware queue
            return st

        def blocked(a, b) -> bool:
            votes = 0
            for _ in range(3):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                with torch.cuda.stream(a):
                    e0.record()
                    big.add_(1.0)
                    big.add_(1.0)
                    e2.record()
                b.wait_event(e0)
                with torch.cuda.stream(b):
                    tiny.add_(1.0)
                    e1.record()
                torch.cuda.synchronize(dev)
                votes += e0.elapsed_time(e1) > 0.5 * e0.elapsed_time(e2)
            return votes >= 2

        torch.cuda.synchronize(dev)
        placed, parked, verified = [main], 0, True
        chosen = []
        for _ in range(2 if want_side else 1):
            for attempt in range(4):
                st = fresh()
                if not any(blocked(p, st) for p in placed):
                    break
                if attempt == 3:
                    verified = False  # keep the last candidate anyway
                    break
                _QUEUE_PAD.append(st)
                parked += 1
            placed.append(st)
            chosen.append(st)
        self._side, self._pipe = (chosen[0], chosen[1]) if want_side else (None, chosen[0])
        del big, tiny
        self.queue_placement = {"probe": True, "pads": parked, "verified": verified}

    def _head_wgrad_buf(self, like: torch.Tensor) -> torch.Tensor:
        """Persistent fp32 buffer for the window's lm_head weight gradient."""
        buf = getattr(self, "_lmbuf", None)
        if buf is None or buf.shape != like.shape or buf.device != like.device or buf.dtype != like.dtype:
            if buf is not None and buf.is_cuda:
                torch.cuda.synchronize(buf.device)
            buf = torch.empty_like(like)
            self._lmbuf = buf
        return buf

    def backward(self, st: _StepState, dloss: torch.Tensor) -> None:
        _drain(self._backward_gen(st, dloss))

    def _backward_gen(self, st: _StepState, dloss: torch.Tensor, prev: Optional[dict] = None,
                      mine: Optional[dict] = None, ready: Optional[list] = None):
        """Generator form of :meth:`backward` (yields after every block).

        ``prev`` / ``mine`` (overlapped backwards, see train_window): the progress events
        of the previous micro-step's backward, and the dict this backward records its own
        into -- "norm" after the final-norm weight gradient, layer ``i`` after every
        gradient layer ``i`` shares with the other micro-steps (norm weights, per-micro-
        step weight gradients), "embed" after the embedding scatter-add.  Every write
        into a shared gradient buffer waits for the previous backward's matching event,
        so the accumulation order -- and every bit of the result -- is the sequential
        one.  Each wait is issued after ``prev`` recorded the event (the window scheduler
        keeps ``prev`` at least one block ahead).  ``ready``: events after the forwards of
        the window's other micro-steps (streams this backward's window-wide lm_head
        weight gradient does not otherwise wait for)."""
        ops, gm, cfg, prov = self.ops, self.gemm, self.cfg, self.provider

        def wait_prev(unit):
            if prev is not None:
                torch.cuda.current_stream().wait_event(prev[unit])

        def mark(unit):
            if mine is not None:
                ev = torch.cuda.Event()
                ev.record()
                mine[unit] = ev
        B, S = st.B, st.S
        L = cfg.num_layers
        ph = self.p_hidden if st.train else 0.0
        pa = self.p_attn if st.train else 0.0
        dloss = dloss.reshape(()).float()

        prov.pre_backward("head")
        hw, hg = prov.head(), prov.head_grads()
        M, H, I = B * S, cfg.hidden_size, cfg.intermediate_size
        dev = st.nf.device
        # deferred roles: one GEMM over the window at the last micro-step (side stream);
        # the others (defer_roles) run in every micro-step's own backward, inline
        dfr = {r: self._deferred(st, r) for r in self.ROLES}
        win = st.last and any(dfr.values())  # this backward runs the window's deferred GEMMs
        side = self._wgrad_stream(dev) if win else None
        inv_ce = 1.0 / st.ce_scale  # the pre-scaled CE gradient (fp16), see ce_grad_scale
        head_ev = None
        head_add = None  # the window's lm_head weight gradient, added after the scatter-adds
        head_taken = False  # ... or by the DDP runtime after its own reduction (head_wgrad_ready)
        head_late = None  # overlapped backwards: the per-micro-step head wgrad waits for "embed"
        head_acc = None  # chunked head: this micro-step's lm_head weight gradient (fp32)
        if st.dnf is not None:
            # early head (train_window): the forward already ran the lm_head backward
            dnf, head_acc = st.dnf, st.head_acc
            st.dnf = st.head_acc = None
        elif st.head_rows is not None:
            # chunked head from the kept logits (autograd path): the same chunk GEMMs, in
            # the same order, as the early head -- the same bits
            dnf = torch.empty(M, H, dtype=st.nf.dtype, device=dev)
            head_acc = self._head_buf(self._head_accs, st.head_key, tuple(hw.lm_head.shape), torch.float32, dev)
            nfs = self._nf_scaled(st.nf, dloss, inv_ce)
            for ci, (a, b) in enumerate(st.head_rows):
                self._head_chunk_bwd(st.dlogits[a:b], hw.lm_head, dnf[a:b], head_acc, nfs[a:b], ci == 0)
            del nfs
        else:
            # lm_head: dnf = dlogits @ E ; dE += dlogits^T @ (nf * dloss)
            dnf = gm.linear_dgrad(st.dlogits, hw.lm_head)
            nf_out = self._sb(st, "head", "nf", M, H, dev)
            if prev is None and mine is not None and _TEST_DELAY_FIRST_BWD:
                # race test hook (DLT_TEST_DELAY_FIRST_BWD=cycles): the first overlapped backward
                # writes its nf slot late, so a reader that does not wait for it sees stale data
                torch.cuda._sleep(_TEST_DELAY_FIRST_BWD)
            nf_scaled = self._nf_scaled(st.nf, dloss, inv_ce, out=nf_out)
            if nf_out is not None:
                # the window's lm_head weight gradient (the last backward, side stream) reads
                # every micro-step's nf slot: "nf" marks this one written, chained through the
                # previous backwards' marks (they run on other streams, a backward apart)
                if prev is not None and "nf" in prev:
                    torch.cuda.current_stream().wait_event(prev["nf"])
                mark("nf")
            if not dfr["head"]:
                if prev is not None:
                    head_late = (st.dlogits, nf_scaled)
                else:
                    gm.wgrad_acc(hg.embed, st.dlogits, nf_scaled)
            elif st.last:
                # ONE [Vp, H] wgrad GEMM over all GA*M rows of the window (K = 32768 instead
                # of 4 x 8192), on the weight-gradient stream so it overlaps the layer
                # backward.  It goes to its own buffer, added into the embedding gradient
                # after the last scatter-add (head_done): the same order in every schedule
                # (sequential, pipelined, overlapped), so it may run whenever its operands exist.
                lg_all = self._slot_buf(st, "head", "lg", M, hw.lm_head.shape[0], dev)[1]
                nf_all = self._slot_buf(st, "head", "nf", M, H, dev)[1]
                head_add = self._head_wgrad_buf(hg.embed)

                def issue_head():
                    head_add.zero_()
                    gm.wgrad_acc(head_add, lg_all, nf_all)
                if side is not None:
                    ev = torch.cuda.Event()
                    ev.record()  # after this backward's nf mark, which follows every earlier one
                    side.wait_event(ev)
                    for e in ready or ():
                        side.wait_event(e)
                    with torch.cuda.stream(side):
                        issue_head()
                        head_ev = torch.cuda.Event()
                        head_ev.record()
                else:
                    issue_head()
                # a data-parallel provider may take the lm_head part over now (its own early
                # all-reduce, added after the embedding part's reduction: parallel/ddp.py)
                take = getattr(getattr(prov, "hooks", None), "head_wgrad_ready", None)
                if take is not None and take(head_add, side):
                    head_taken = True
        st.dlogits = None
        key_last = self._keys(st.micro, L - 1)[2]
        # The side stream lags the dgrad chain by a few layers' worth of weight-gradient
        # GEMMs; the last ``n_main`` layers' wgrads run on the current stream instead, so
        # the two queues drain together once the dgrad chain is done.  Their gradient
        # hooks (DDP bucket launches) are issued at the end, after joining the side
        # stream, so a bucket never reads a gradient still being written on another
        # stream.  Only for providers whose hooks can be delayed (the flat DDP store).
        n_main = self.main_wgrad_layers if (side is not None and getattr(prov, "late_post_backward_ok", False)) else 0
        late = []
        # DDP store: the head gradient hook may run before layer 0's weight gradients
        early_head = getattr(prov, "late_post_backward_ok", False)

        def head_done():
            # embedding (tied with lm_head): scatter-add, then the head gradient hook
            if head_ev is not None:
                torch.cuda.current_stream().wait_event(head_ev)
            wait_prev("embed")
            if head_late is not None:
                gm.wgrad_acc(hg.embed, *head_late)
            ops.embedding_bwd(st.ids, g_x2n if early_head else g_x2, hg.embed)
            if head_add is not None and not head_taken:
                hg.embed.add_(head_add)
            if head_acc is not None:
                hg.embed.add_(head_acc)
            mark("embed")
            prov.post_backward("head")

        def sb(layer, name, n):
            return self._sb(st, layer, name, M, n, dev)

        def full(layer, name, n):
            return self._slot_buf(st, layer, name, M, n, dev)[1]

        wait_prev("norm")
        g_x2, g_d = ops.rmsnorm_bwd(dnf, st.xf, st.rstdf, hw.norm, None, hg.norm,
                                    ph, key_last, dy_scale=dloss, want_ddelta=True, ddelta_out=sb(L - 1, "dd", H),
                                    dy_mul=inv_ce)
        mark("norm")
        del dnf
        cos, sin = self.rope(S, g_x2.device)

        for i in reversed(range(L)):
            prov.pre_backward(i)
            wait_prev(i)
            if self._ring:
                # dY ring: this block writes layer i's dgu / da / dqkv (slot i % R) and layer
                # i-1's dd (slot (i-1) % R); their previous occupants are layers i+R and
                # i-1+R, whose window weight gradients were issued (side stream, in layer
                # order) by the last backward before this block was issued
                j = i - 1 + self._ring
                if j < L and any(self._deferred(st, self._SLOT_ROLE[n]) for n in self._DY_SLOTS):
                    # the window's last backward records it after issuing layer j's
                    # weight gradients; B1 runs one block behind B0 and R >= 2, so it must
                    # exist by now -- a missing event means the issue order changed and
                    # this block would overwrite operands still being read
                    ev = self._ring_done.get(j)
                    if ev is None:
                        raise RuntimeError(f"dY ring: layer {j}'s weight gradients not issued before layer {i} "
                                           "reuses its slot (window issue order changed?)")
                    torch.cuda.current_stream().wait_event(ev)
            c = st.caches[i]
            if st.recompute:
                # Re-run (part of) the layer forward from the saved tensors; masks replay exactly.
                c = self._layer_recompute(st, i, c)
            w, gr = prov.layer(i), prov.layer_grads(i)
            k_attn, k_resid, k_mlp = self._keys(st.micro, i)
            # MLP
            # s ring: the SwiGLU backward also rewrites s (the down wgrad operand) into
            # layer i's ring slot, from the same gu with the forward's arithmetic
            s_kw = {"s_out": sb(i, "s", I)} if self._s_in_ring(st) else {}
            s_new = None
            if self._refill_s(st) and c.gu is not None:
                s_new = torch.empty(M, I, dtype=c.gu.dtype, device=c.gu.device)
                s_kw = {"s_out": s_new}
            if hasattr(gm, "linear_dgrad_swiglu"):  # down dgrad with the SwiGLU backward in its epilogue (when faster)
                dgu = gm.linear_dgrad_swiglu(g_d, w.wdown, c.gu, ops, out=sb(i, "dgu", 2 * I), **s_kw)
            else:
                ds = gm.linear_dgrad(g_d, w.wdown)
                dgu = ops.swiglu_bwd(c.gu, ds, out=sb(i, "dgu", 2 * I), **s_kw)
                del ds
            dn2 = gm.linear_dgrad(dgu, w.wgu)
            dx2, da = ops.rmsnorm_bwd(dn2, c.x2, c.rstd2, w.ln2, g_x2, gr.ln2, ph, k_resid,
                                      ddelta_out=sb(i, "da", H))
            del dn2
            # attention
            do = gm.linear_dgrad(da, w.wo)
            if c.k is None:  # packed: dq/dk/dv land in [M, 3H] with the inverse RoPE applied
                dqkv = ops.attention_bwd_packed(c.q, c.o, do, c.lse, pa, k_attn, B, S, cfg.num_heads, cos, sin,
                                                out=sb(i, "dqkv", 3 * H))
                del do
            else:
                dq, dk, dv = ops.attention_bwd(c.q, c.k, c.v, c.o, do, c.lse, pa, k_attn, True)
                del do
                dqkv = ops.rope_qkv_bwd(dq, dk, dv, cos, sin, out=sb(i, "dqkv", 3 * H))
                del dq, dk, dv
            dn1 = gm.linear_dgrad(dqkv, w.wqkv)
            key_prev = self._keys(st.micro, i - 1)[2] if i > 0 else 0
            p_prev = ph if i > 0 else 0.0
            g_x2n, g_dn = ops.rmsnorm_bwd(dn1, c.x, c.rstd1, w.ln1, dx2, gr.ln1, p_prev, key_prev,
                                          want_ddelta=(i > 0), ddelta_out=sb(i - 1, "dd", H) if i > 0 else None)
            del dn1, dx2
            if i == 0 and early_head:
                # The head bucket (tied embedding + every norm weight) is final once the
                # embedding scatter-add is done: issue its all-reduce now, so it overlaps
                # the last layers' weight-gradient GEMMs instead of trailing the step.
                head_done()
            # weight gradients (fp32 accumulate into the main-grad buffers)
            side_ctx = None
            # deferred: one GEMM per weight over the whole accumulation window.  The
            # slot buffers are persistent, so these can run on a side stream
            # concurrently with the next layer's dgrad chain (the small-output
            # wgrads leave most CUs idle); the layer's gradient hook (DDP
            # bucket all-reduce) is issued from the same stream.
            dfl = {r: self._deferred(st, r, i) for r in self.ROLES}  # this layer's deferred roles
            if win:
                if side is not None and i >= n_main:
                    ev = torch.cuda.Event()
                    ev.record()
                    side.wait_event(ev)
                    side_ctx = torch.cuda.stream(side)
                    side_ctx.__enter__()
                if dfl["down"]:
                    _wgrad(gm, gr.wdown, full(i, "dd", H), full(i, "s", I))
                if dfl["gu"]:
                    _wgrad(gm, gr.wgu, full(i, "dgu", 2 * I), full(i, "n2", H))
                if dfl["o"]:
                    _wgrad(gm, gr.wo, full(i, "da", H), full(i, "o", H))
                if dfl["qkv"]:
                    _wgrad(gm, gr.wqkv, full(i, "dqkv", 3 * H), full(i, "n1", H))
                if self._ring:
                    ev = torch.cuda.Event()
                    ev.record()
                    self._ring_done[i] = ev
            if not all(dfl.values()):  # the per-micro-step ones, on this backward's stream
                if side_ctx is not None:
                    side_ctx.__exit__(None, None, None)
                if not dfl["down"]:
                    _wgrad(gm, gr.wdown, g_d, c.s if s_new is None else s_new)
                if not dfl["gu"]:
                    _wgrad(gm, gr.wgu, dgu, c.n2)
                if not dfl["o"]:
                    _wgrad(gm, gr.wo, da, c.o)
                if not dfl["qkv"]:
                    _wgrad(gm, gr.wqkv, dqkv, c.n1)
                if side_ctx is not None:
                    # the gradient hook goes out from the side stream, after both halves
                    ev = torch.cuda.Event()
                    ev.record()
                    side.wait_event(ev)
                    side_ctx = torch.cuda.stream(side)
                    side_ctx.__enter__()
            del dgu, da, dqkv
            g_x2, g_d = g_x2n, g_dn
            st.caches[i] = None
            try:
                if i < n_main:
                    late.append(i)
                else:
                    prov.post_backward(i)
            finally:
                if side_ctx is not None:
                    side_ctx.__exit__(None, None, None)
            mark(i)
            yield
        if not early_head:
            head_done()
        if late:
            torch.cuda.current_stream().wait_stream(side)
            for i in late:
                prov.post_backward(i)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)

    # ------------------------------------------------------ pipelined window
    def window_schedule(self, GA: int, defer: bool, cuda: bool = True):
        """(overlapped backwards?, "ffbb" | "fb") for a window of GA chains.

        Overlapped backwards: providers that allow them (``overlap_backward_ok``: the flat
        DDP store, the FSDP runtime), ``DLT_BWD_OVERLAP=0`` turns them off.  ffbb (two
        chains only, needs overlap) is the default when every weight gradient is deferred
        (the memory-lean modes keep fb: both forwards' activations live at once cost ~5 GB;
        FSDP's per-micro-step weight gradients: measured no faster, 1.5x the memory), the
        model is GPT-2-small-sized (small +0.9-1.1 %, medium -1.3 %: its larger GEMMs fill
        the GPU alone, two forwards only contend).  With gradient collectives a
        communicator's streams shift the engine's hardware queues (ffbb 693k vs fb 789k tok/s
        on one forced RCCL rank as placed by default, 797.5-798.0k with three idle streams
        created first: profiles/r5_stream_queues.md), so the schedule is chosen by timing
        (_auto_window / _auto_enter, default; DLT_WINDOW_AUTO=0 keeps fb, DLT_QUEUE_PROBE=1
        uses the opt-in placement probe instead).
        ``DLT_WINDOW_SCHED=fb|ffbb`` overrides (profiles/r3_window_ffbb.md)."""
        overlap = (cuda and GA > 1 and getattr(self.provider, "overlap_backward_ok", False)
                   and os.environ.get("DLT_BWD_OVERLAP", "1") != "0")
        hooks = getattr(self.provider, "hooks", None)
        comm = bool(getattr(hooks, "collectives", False) or getattr(self.provider, "collectives", False))
        eligible = (overlap and GA == 2 and defer and self.defer_roles == frozenset(self.ROLES)
                    and self.cfg.hidden_size <= 768)
        auto = None
        if eligible and comm and "DLT_WINDOW_SCHED" not in os.environ:
            eligible = False
            if os.environ.get("DLT_QUEUE_PROBE") == "1":
                self._place_streams(torch.device("cuda", torch.cuda.current_device()))
                eligible = bool(self.queue_placement and self.queue_placement["verified"])
            elif os.environ.get("DLT_WINDOW_AUTO", "1") != "0":
                auto = self._auto_window()
        sched = auto or os.environ.get("DLT_WINDOW_SCHED", "ffbb" if eligible else "fb")
        if not (overlap and GA == 2 and sched == "ffbb"):
            sched = "fb"
        return overlap, sched

    # Timed choice between the fb and ffbb windows under gradient collectives (default;
    # DLT_WINDOW_AUTO=0 keeps fb).  With collectives ffbb depends on which hardware queues
    # the communicator's streams leave the engine's (profiles/r5_stream_queues.md): on one
    # forced RCCL rank it ran 693k tok/s as placed by default and 797.5-798.0k with three
    # idle streams created ahead of the engine's (DLT_QUEUE_PAD=3, the default here), fb
    # 787-790k -- unknown on a multi-GPU node.  So the first pipelined windows run fb,
    # ffbb, fb, ffbb; at the entry of the next window each schedule's best step time (GPU
    # events at consecutive window entries, i.e. the whole step) is max-reduced over the
    # ranks and every rank keeps the faster schedule -- the same decision everywhere, taken
    # at the same point of the collective sequence.
    _AUTO_TRIALS = ("fb", "ffbb", "fb", "ffbb")

    def _auto_window(self) -> str:
        """The schedule of the next window while the choice is open, then the decision."""
        a = self.window_auto
        if a is None:
            a = self.window_auto = {"events": [], "decided": None, "ms": None}
        if a["decided"] is not None:
            return a["decided"]
        return self._AUTO_TRIALS[min(len(a["events"]), len(self._AUTO_TRIALS) - 1)]

    def _auto_enter(self, dev) -> bool:
        """Window entry while the timed choice is open: stamp it; after the last trial,
        decide.  True when the decision was just taken (the caller re-reads the schedule)."""
        a = self.window_auto
        if a is None or a["decided"] is not None or dev.type != "cuda":
            return False
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(dev))
        a["events"].append(ev)
        n = len(self._AUTO_TRIALS)
        if len(a["events"]) <= n:
            return False
        ev.synchronize()
        t = [a["events"][i].elapsed_time(a["events"][i + 1]) for i in range(n)]
        best = [min(t[i] for i in range(n) if self._AUTO_TRIALS[i] == k) for k in ("fb", "ffbb")]
        import torch.distributed as dist
        # over the gradient collectives' own group (the DDP runtime's pg; FSDP, whose shard
        # and replica groups together span every rank: None = WORLD): every rank of that
        # group takes the same pipelined-window path, so all of them reach this reduction
        # at the same point of their collective sequence
        pg = getattr(getattr(self.provider, "hooks", None), "pg", None)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(pg) > 1:
            v = torch.tensor(best, dtype=torch.float32, device=dev if dist.get_backend(pg) == "nccl" else "cpu")
            dist.all_reduce(v, op=dist.ReduceOp.MAX, group=pg)
            best = v.tolist()
        fb, ffbb = (float(x) for x in best)
        a["decided"] = "ffbb" if ffbb < fb else "fb"
        a["ms"] = {"fb": round(fb, 3), "ffbb": round(ffbb, 3)}
        a["events"] = []
        return True

    def _window_ffbb(self, micro_ids, micro_targets, dloss, recompute, defer, sync_hook, before_last,
                     serial=False):
        """Two-chain window F0 || F1 | B0 || B1 (see train_window).  ``serial``: the same
        block order with both chains on the current stream (the trainers' first step,
        whose GEMM races must time on a quiet GPU) -- same kernels, same results, and
        the same dY slot ring, so the first step does not need per-layer dY slots."""
        dev = micro_ids[0].device
        self.set_accumulation(0, 2, defer=defer)
        main = torch.cuda.current_stream(dev)
        if serial:
            p0 = main
        else:
            self._place_streams(dev)
            p0 = self._pipe
        self.rope(micro_ids[0].shape[1], dev)
        self._wgrad_stream(dev)  # created before the fork
        p0.wait_stream(main)
        streams = [p0, main]
        # the hand projection GEMM's persistent grid leaves CUs to the other chain
        # (DLT_FFBB_GEMM_GRID, default 192 of 256 workgroups: +0.05-0.5 % in three same-box
        # A/Bs, docs/KERNELS.md; results unchanged, each output tile is still computed
        # whole by one workgroup)
        cap = int(os.environ.get("DLT_FFBB_GEMM_GRID", "192")) if not serial else 0
        prev_cap = self.ops.gemm_grid_cap(cap) if cap and hasattr(self.ops, "gemm_grid_cap") else None
        # The two backwards run a block apart and the last one issues each layer's window
        # weight gradients right after its own block, so a layer's dY operands (dqkv, da,
        # dgu, dd: ~650 MB per layer at the headline shape) are dead a few layers later:
        # they live in a ring of R slots instead of one slot per layer (DLT_SLOT_RING,
        # default 3; 0 = per layer).  A block waits for the weight gradients of the
        # layer whose slot it reuses.
        ring = int(os.environ.get("DLT_SLOT_RING", "3")) if defer else 0
        self._ring = ring if 2 <= ring < self.cfg.num_layers else 0
        self._ring_done = {}
        if self._ring:  # per-layer dY slots of an earlier schedule would only hold memory
            for key in [k for k in self._slots if self._ring_name(k[1]) and not isinstance(k[0], tuple)]:
                del self._slots[key]
        try:
            return self._window_ffbb_body(micro_ids, micro_targets, dloss, recompute, defer, sync_hook, before_last,
                                          main, p0, streams)
        finally:
            self._ring = 0
            self._ring_done = {}
            if prev_cap is not None:
                self.ops.gemm_grid_cap(prev_cap)

    def _window_ffbb_body(self, micro_ids, micro_targets, dloss, recompute, defer, sync_hook, before_last,
                          main, p0, streams):
        losses: List[Any] = [None, None]
        states: List[Any] = [None, None]
        ready: List[Any] = []
        # forwards: chain 0 first in every round (micro-step numbering = dropout streams)
        gens = [self._forward_gen(micro_ids[k], micro_targets[k], True, recompute, need_backward=True,
                                  acc=(k, 2, defer), head_dloss=dloss) for k in range(2)]
        live = [0, 1]
        while live:
            for k in list(live):
                with torch.cuda.stream(streams[k]):
                    try:
                        next(gens[k])
                    except StopIteration as stop:
                        live.remove(k)
                        losses[k], _, states[k] = stop.value
                        if k == 0:
                            ev = torch.cuda.Event()
                            ev.record()
                            ready.append(ev)
        prog: List[dict] = [dict(), dict()]
        bgens = [self._backward_gen(states[0], dloss, None, prog[0]),
                 self._backward_gen(states[1], dloss, prog[0], prog[1], ready=ready)]
        states = [None, None]
        if sync_hook is None and before_last is not None:
            raise ValueError("the ffbb window schedule needs sync_hook (per-block sync flag)")
        live = [0, 1]
        while live:  # B0 always issues its block first: B1's waits find B0's events recorded
            for k in list(live):
                if sync_hook is not None:
                    sync_hook(k == 1)
                with torch.cuda.stream(streams[k]):
                    try:
                        next(bgens[k])
                    except StopIteration:
                        live.remove(k)
        main.wait_stream(p0)
        return losses

    def train_window(self, micro_ids: List[torch.Tensor], micro_targets: List[torch.Tensor],
                     dloss: torch.Tensor, recompute: bool = False,
                     before_last: Optional[Callable[[], None]] = None, defer: bool = True,
                     sync_hook: Optional[Callable[[bool], None]] = None, serial: bool = False) -> List[torch.Tensor]:
        """Forward + backward of a whole gradient-accumulation window.

        Schedule (GA = 4):  F0 | B0+F1 | B1+F2 | B2+F3 | B3, where "Bk+Fk+1" issues the
        blocks of the two chains alternately; micro-steps alternate between the current
        stream and the weight-gradient side stream, the last one on the current stream.
        A micro-step's forward and backward run on the same stream, so its activations
        never cross streams; what is shared
        (weights, slot buffers, RoPE tables, the ids) is read-only until the window
        ends or is produced before the fork.  The last backward first joins the other
        stream: its lm_head weight-gradient GEMM (beta = 1) and the DDP bucket
        all-reduces must see every micro-step's gradient.  Weight gradients are
        deferred (one GEMM per weight over the window), so before that point the
        chains only add into the norm-weight and embedding gradients, one backward
        after the other (deterministic kernels, no float atomics).

        ``dloss`` is d(total)/d(micro-step loss) (1/GA), ``before_last`` runs before
        the last backward is issued (the DDP runtime switches its sync on there).
        ``defer=False`` (the FSDP runtime, which reduce-scatters every micro-step) runs
        each micro-step's weight gradients in its own backward; the provider must then
        give every micro-step fresh gradient buffers (FSDP's per-micro-step full_grad),
        since two backwards may overlap on the GPU.
        Returns the GA micro-step losses (device scalars, unscaled).  Dropout streams,
        numerics and gradients are identical to running the micro-steps one by one.

        Overlapped backwards (flat DDP store, ``DLT_BWD_OVERLAP=1`` default): backward k
        does not wait for backward k-1 to finish, only -- per shared gradient buffer --
        for the matching progress event of it (final norm, each layer, the embedding;
        see _backward_gen), so the two backwards run concurrently a few layers apart,
        with the sequential accumulation order.  The schedule becomes
        F0 | B0+F1 | B0+B1 | B1 instead of F0 | B0+F1 | B1 (only the first forward and the
        tail of the last backward run without a partner).

        Two chains (the headline B8 x GA4 as 2 x 16), ``DLT_WINDOW_SCHED=ffbb`` (default with
        every weight gradient deferred; ``fb`` = the schedule above): F0 || F1,
        then B0 || B1 with B1 one block behind B0 (its per-buffer waits, above) -- no
        phase without a partner chain; chain 0 runs on a stream of its own, the weight
        gradients on the side stream.  ``sync_hook(last)`` is called before every
        backward block (the DDP runtime's per-micro-step sync flag; ``before_last`` is not
        used by this schedule).
        """
        GA = len(micro_ids)
        dev = micro_ids[0].device
        cuda = dev.type == "cuda"
        overlap, sched = self.window_schedule(GA, defer, cuda)
        if not serial and self._auto_enter(dev):
            overlap, sched = self.window_schedule(GA, defer, cuda)
        self.last_window = sched
        prog: List[dict] = [dict() for _ in range(GA)]
        if sched == "ffbb":
            return self._window_ffbb(micro_ids, micro_targets, dloss, recompute, defer, sync_hook, before_last,
                                     serial=serial)
        if serial:
            raise ValueError("serial=True is the single-stream form of the ffbb window only")
        self.set_accumulation(0, GA, defer=defer)
        main = pipe = None
        if cuda:
            main = torch.cuda.current_stream(dev)
            # The second chain runs on the weight-gradient side stream: the last
            # micro-step (the only one with weight-gradient GEMMs) is placed on the
            # current stream and joins the other chain before it starts, so the side
            # stream is idle by then.  Two streams in flight at any time, never three.
            pipe = self._wgrad_stream(dev)
            if pipe is None:
                self._place_streams(dev)
                pipe = self._pipe
            self.rope(micro_ids[0].shape[1], dev)  # lazily-built shared state: before the fork
            pipe.wait_stream(main)

        def stream_of(k):  # the last micro-step on the current stream, alternating backwards
            return main if (GA - 1 - k) % 2 == 0 else pipe

        def on(k):
            return torch.cuda.stream(stream_of(k)) if cuda else contextlib.nullcontext()

        def fwd(k):
            return self._forward_gen(micro_ids[k], micro_targets[k], True, recompute, need_backward=True,
                                     acc=(k, GA, defer), head_dloss=dloss)

        losses: List[Any] = [None] * GA
        states: List[Any] = [None] * GA
        with on(0):
            losses[0], _, states[0] = _drain(fwd(0))
        for k in range(GA):
            if k == GA - 1:
                if cuda and GA > 1 and not overlap:
                    main.wait_stream(pipe)
                if before_last is not None:
                    before_last()
            elif cuda and k > 0 and not overlap:
                # backward k starts after backward k-1 has finished on the other stream:
                # both add into the same norm / embedding gradients (fixed-order, non-atomic
                # kernels), so two backwards never overlap -- a backward still overlaps
                # the next micro-step's forward, which is what the pipelining is for.
                stream_of(k).wait_stream(stream_of(k - 1))
            # overlapped: backward k-1 is fully issued by now (its events exist)
            ev_args = (prog[k - 1] if k > 0 else None, prog[k]) if overlap else (None, None)
            running = [(k, self._backward_gen(states[k], dloss, *ev_args), False)]
            states[k] = None
            if k + 1 < GA:
                running.append((k + 1, fwd(k + 1), True))
            while running:
                for item in list(running):
                    j, gen, is_fwd = item
                    with on(j):
                        try:
                            next(gen)
                        except StopIteration as stop:
                            running.remove(item)
                            if is_fwd:
                                losses[j], _, states[j] = stop.value
        if overlap:  # the optimizer (current stream) must see every backward's gradients
            main.wait_stream(pipe)
        return losses


_TEST_DELAY_FIRST_BWD = int(os.environ.get("DLT_TEST_DELAY_FIRST_BWD", "0"))

_QUEUE_PAD = []  # streams that exist only to shift the engine streams' hardware queues


def _queue_pad(dev, n: int) -> None:
    """DLT_QUEUE_PAD=n (A/B knob, replaces the probe of Engine._place_streams): before the
    engine's side streams are created, n streams each dispatch one empty kernel, so the
    HIP runtime's round-robin assignment of hardware queues (at a stream's first dispatch)
    gives the engine's weight-gradient and pipeline streams queues n later."""
    if n <= 0 or _QUEUE_PAD or torch.device(dev).type != "cuda":
        return
    for _ in range(n):
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            torch.cuda._sleep(1)
        _QUEUE_PAD.append(st)
    torch.cuda.synchronize(dev)


def _wgrad(gm, dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    """A layer weight gradient: accumulated into the provider's fp32 buffer, or written
    once per micro-step into a bf16 reduce-scatter buffer (FSDPRuntime.bf16_grads)."""
    if dw.dtype in (torch.bfloat16, torch.float16):
        gm.wgrad_set(dw, dy, x)
    else:
        gm.wgrad_acc(dw, dy, x)


class _TorchGemm:
    """Plain library GEMMs (hipBLASLt on ROCm via torch.matmul).

    NOT stream-safe on the GPU: torch keeps one hipBLASLt handle per thread, and
    hipBLASLt GEMMs in flight concurrently on two streams through one handle can
    deadlock the gfx950 stream-K kernels (see ops/csrc_gemm/gemm_planner.cpp), so with
    this backend the engine runs no side-stream GEMMs and no micro-step pipelining.

    ``wgrad_acc`` accumulates bf16 x bf16 products straight into the fp32 main-grad
    buffer with ``addmm(..., out_dtype=float32)`` when available (no bf16 round trip,
    no separate add kernel); otherwise falls back to matmul + add_.
    """

    stream_safe = False

    def __init__(self):
        self._fp32_out_ok = None

    @staticmethod
    def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        if out is not None:
            return torch.matmul(x, w.t(), out=out)
        return torch.matmul(x, w.t())

    @staticmethod
    def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        if out is not None:
            return torch.matmul(dy, w, out=out)
        return torch.matmul(dy, w)

    @staticmethod
    def wgrad_set(dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
        """dw (bf16, overwritten) = dy^T @ x (the FSDP bf16 send-buffer mode)."""
        dw2 = dw.view(dy.shape[1], x.shape[1])
        if dw2.dtype not in (torch.bfloat16, torch.float16) or not dw2.is_contiguous():
            raise ValueError("wgrad_set output must be contiguous bf16 / fp16")
        torch.matmul(dy.t(), x, out=dw2)

    def wgrad_acc(self, dw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
        if dw.dtype in (torch.bfloat16, torch.float16):
            raise ValueError("wgrad_acc accumulates into fp32; use wgrad_set for a 16-bit gradient")
        dw2 = dw.view(dy.shape[1], x.shape[1])
        if dy.dtype == torch.float32:
            dw2.addmm_(dy.t(), x)
            return
        if self._fp32_out_ok is not False and dy.is_cuda:
            try:
                torch.addmm(dw2, dy.t(), x, out_dtype=torch.float32, out=dw2)
                self._fp32_out_ok = True
                return
            except (RuntimeError, TypeError):
                self._fp32_out_ok = False
        dw2.add_(torch.matmul(dy.t(), x))


class EngineFunction(torch.autograd.Function):
    """Autograd bridge: ``loss.backward()`` runs ``GPTEngine.backward``.

    Weight gradients are written into the provider's fp32 gradient buffers directly
    (the ``param.grad`` views); autograd only sees a dummy anchor input.
    """

    @staticmethod
    def forward(ctx, anchor, engine, ids, targets, recompute):
        loss, _, st = engine.forward(ids, targets, train=True, recompute=recompute,
                                    need_backward=True)
        ctx.engine = engine
        ctx.state = st
        return loss

    @staticmethod
    def backward(ctx, dloss):
        if ctx.state is not None:
            ctx.engine.backward(ctx.state, dloss)
            ctx.state = None
        return None, None, None, None, None
