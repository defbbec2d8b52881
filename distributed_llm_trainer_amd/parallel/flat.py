"""Flat parameter / gradient / shadow-weight storage for the single-GPU and DDP paths.

The reference keeps 110 separate fp32 parameter tensors, lets autocast re-cast each
weight to bf16 on every micro-step and lets the DDP Reducer copy
gradients into 25 MB buckets (K16).  Here every parameter is a *view* into one
contiguous fp32 master buffer laid out so that

* ``q|k|v`` rows of a layer are adjacent -> the packed ``[3H, H]`` QKV weight is a
  free view, likewise ``gate|up`` -> ``[2I, H]`` (one GEMM each instead of 3 and 2);
* a bf16 "shadow" buffer with the identical layout is written by the fused AdamW
  kernel, so GEMMs read bf16 weights with no per-step cast kernels;
* the embedding region is padded to ``vocab_size_padded`` rows (zero rows, zero
  grads) so the tied lm_head GEMM has an aligned N;
* gradients live in a flat fp32 buffer with the same layout: DDP all-reduces
  contiguous slices of it in place (zero-copy buckets), and clip/AdamW are single
  flat launches;
* all no-weight-decay params (the RMSNorm weights -- the reference's "norm"/"bias"
  rule, ``ddp_trainer.py:214-227``) are at the end, so weight decay is one boundary.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..models.engine import HeadGrads, HeadWeights, LayerGrads, LayerWeights, ParamProvider


@dataclass
class Segment:
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]


class FlatLayout:
    """Ordered segments of the flat buffer for one GPT model."""

    def __init__(self, cfg):
        self.cfg = cfg
        H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_layers
        V, Vp = cfg.vocab_size, cfg.vocab_size_padded
        segs: List[Segment] = []
        off = 0

        def add(name, shape, alloc=None):
            nonlocal off
            n = 1
            for s in shape:
                n *= s
            segs.append(Segment(name, off, n, tuple(shape)))
            off += alloc if alloc is not None else n

        self.layer_bounds: List[Tuple[int, int]] = []
        for i in range(L):
            start = off
            p = f"layers.{i}."
            add(p + "attention.q_proj.weight", (H, H))
            add(p + "attention.k_proj.weight", (H, H))
            add(p + "attention.v_proj.weight", (H, H))
            add(p + "attention.o_proj.weight", (H, H))
            add(p + "mlp.gate_proj.weight", (I, H))
            add(p + "mlp.up_proj.weight", (I, H))
            add(p + "mlp.down_proj.weight", (H, I))
            self.layer_bounds.append((start, off))
        self.embed_offset = off
        add("embed_tokens.weight", (V, H), alloc=Vp * H)
        self.decay_end = off
        for i in range(L):
            add(f"layers.{i}.input_layernorm.weight", (H,))
            add(f"layers.{i}.post_attention_layernorm.weight", (H,))
        add("norm.weight", (H,))
        self.total = off
        self.segments = segs
        self.by_name: Dict[str, Segment] = {s.name: s for s in segs}


class FlatParamStore(ParamProvider):
    # gradient hooks (DDP bucket launches) may be issued from the engine's
    # weight-gradient stream: they only enqueue collectives on the current stream
    side_stream_hooks = True
    # ... and may be delayed to the end of the backward (engine ``main_wgrad_layers``)
    late_post_backward_ok = True
    # two micro-steps' backwards may run concurrently, ordered per shared gradient buffer by
    # progress events (GPTEngine.train_window)
    overlap_backward_ok = True

    def __init__(self, model, device, compute_dtype=torch.bfloat16, grad_dtype=torch.float32):
        self.model = model
        self.cfg = model.config
        self.layout = FlatLayout(self.cfg)
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        lay = self.layout
        H = self.cfg.hidden_size
        self.flat = torch.zeros(lay.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(lay.total, dtype=grad_dtype, device=self.device)
        named = dict(model.named_parameters())
        with torch.no_grad():
            for seg in lay.segments:
                p = named[seg.name]
                self.flat[seg.offset:seg.offset + seg.numel].copy_(p.detach().reshape(-1))
        # re-home parameters as views (tied lm_head.weight is the same Parameter)
        for seg in lay.segments:
            p = named[seg.name]
            p.data = self.flat[seg.offset:seg.offset + seg.numel].view(seg.shape)
            p.grad = self.grad[seg.offset:seg.offset + seg.numel].view(seg.shape)
        if compute_dtype == torch.float32:
            self.shadow = self.flat
        else:
            self.shadow = self.flat.to(compute_dtype)
        self._build_views()
        # readers of the module's state see the weights of the last optimizer step, and a
        # load replaces them only after that step is applied (a pending update replayed
        # onto loaded weights would corrupt them with stale gradients and moments)
        model.register_state_dict_pre_hook(lambda *args, **kw: self.flush_pending())
        model.register_load_state_dict_pre_hook(lambda *args, **kw: self.flush_pending())

    # ----------------------------------------------------------------- views
    def _build_views(self):
        lay, cfg = self.layout, self.cfg
        H, I, Vp = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size_padded
        bn = lay.by_name

        def v(buf, name, rows, cols):
            s = bn[name]
            return buf[s.offset:s.offset + rows * cols].view(rows, cols)

        def vec(buf, name):
            s = bn[name]
            return buf[s.offset:s.offset + s.numel]

        self._layers, self._lgrads = [], []
        for i in range(cfg.num_layers):
            p = f"layers.{i}."
            self._layers.append(LayerWeights(
                wqkv=v(self.shadow, p + "attention.q_proj.weight", 3 * H, H),
                wo=v(self.shadow, p + "attention.o_proj.weight", H, H),
                wgu=v(self.shadow, p + "mlp.gate_proj.weight", 2 * I, H),
                wdown=v(self.shadow, p + "mlp.down_proj.weight", H, I),
                ln1=vec(self.flat, p + "input_layernorm.weight"),
                ln2=vec(self.flat, p + "post_attention_layernorm.weight")))
            self._lgrads.append(LayerGrads(
                wqkv=v(self.grad, p + "attention.q_proj.weight", 3 * H, H),
                wo=v(self.grad, p + "attention.o_proj.weight", H, H),
                wgu=v(self.grad, p + "mlp.gate_proj.weight", 2 * I, H),
                wdown=v(self.grad, p + "mlp.down_proj.weight", H, I),
                ln1=vec(self.grad, p + "input_layernorm.weight"),
                ln2=vec(self.grad, p + "post_attention_layernorm.weight")))
        e = bn["embed_tokens.weight"]
        self._head = HeadWeights(
            embed=self.flat[e.offset:e.offset + e.numel].view(e.shape),
            lm_head=self.shadow[e.offset:e.offset + Vp * H].view(Vp, H),
            norm=vec(self.flat, "norm.weight"))
        self._hgrads = HeadGrads(embed=self.grad[e.offset:e.offset + Vp * H].view(Vp, H),
                                 norm=vec(self.grad, "norm.weight"))

    def unit_ranges(self) -> Dict[object, List[Tuple[int, int]]]:
        """The flat ranges of each forward unit, in forward order: "head" (embedding / tied
        lm_head + the final norm; the embedding is read first) and layer i (its weights and
        its two norm weights).  Together they cover the buffer exactly once (the lazy
        optimizer step updates one unit at a time, training/optim.py LazyStep)."""
        lay, H = self.layout, self.cfg.hidden_size
        bn = lay.by_name
        fn = bn["norm.weight"]
        units: Dict[object, List[Tuple[int, int]]] = {"head": [(lay.embed_offset, lay.decay_end),
                                                               (fn.offset, fn.offset + fn.numel)]}
        for i, (a, b) in enumerate(lay.layer_bounds):
            n1 = bn[f"layers.{i}.input_layernorm.weight"]
            n2 = bn[f"layers.{i}.post_attention_layernorm.weight"]
            assert n2.offset == n1.offset + H
            units[i] = [(a, b), (n1.offset, n2.offset + H)]
        return units

    # pending lazy optimizer step (training/optim.py LazyStep): each unit's update is
    # launched by pre_forward(unit) of the next forward
    pending = None

    def flush_pending(self) -> None:
        """Apply every not-yet-applied unit of a pending lazy optimizer step, ordered before
        the current stream's later work (checkpoints, eval, state_dict readers)."""
        if self.pending is not None:
            self.pending.ensure_all()
            self.pending = None

    def discard_pending(self) -> None:
        """Drop a pending lazy optimizer step without applying it (its not-yet-applied
        units' gradients are zeroed, as the step would have done): the fp32 master was
        overwritten externally and is the truth now."""
        p = self.pending
        if p is not None:
            p.discard()
            self.pending = None

    def refresh_shadow(self) -> None:
        """Re-derive the bf16 shadow from the fp32 master (after load / external edits).
        The master is taken as final: a still-pending lazy step is discarded, never
        replayed on top of it (callers that want it applied flush before editing)."""
        self.discard_pending()
        if self.shadow is not self.flat:
            self.shadow.copy_(self.flat)

    def zero_grad(self) -> None:
        self.grad.zero_()

    # -------------------------------------------------------------- provider
    def layer(self, i):
        return self._layers[i]

    def layer_grads(self, i):
        return self._lgrads[i]

    def head(self):
        return self._head

    def head_grads(self):
        return self._hgrads

    def sync_grads_from_params(self) -> None:
        """Eager path: make sure every param.grad lives in (or is copied into) the flat
        grad buffer, and re-point it there."""
        named = dict(self.model.named_parameters())
        for seg in self.layout.segments:
            p = named[seg.name]
            view = self.grad[seg.offset:seg.offset + seg.numel].view(seg.shape)
            if p.grad is None:
                continue
            if p.grad.data_ptr() != view.data_ptr():
                view.copy_(p.grad)
                p.grad = view

    # ------------------------------------------------------------ hook fan-out
    hooks: Optional[object] = None

    def pre_forward(self, unit):
        if self.pending is not None:
            self.pending.ensure(unit)
        if self.hooks is not None:
            self.hooks.pre_forward(unit)

    def post_forward(self, unit):
        if self.hooks is not None:
            self.hooks.post_forward(unit)

    def pre_backward(self, unit):
        if self.hooks is not None:
            self.hooks.pre_backward(unit)

    def post_backward(self, unit):
        if self.hooks is not None:
            self.hooks.post_backward(unit)
