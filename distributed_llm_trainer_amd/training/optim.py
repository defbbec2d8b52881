"""Fused AdamW over flat parameter buffers, plus on-device gradient clipping.

Semantics follow ``torch.optim.AdamW`` (decoupled weight decay, bias correction,
eps outside the sqrt) exactly as the reference configures it:

* DDP trainer (``ddp_trainer.py:214-234``): two groups, weight decay on everything
  except names containing "bias"/"norm" -> here the flat layout puts all norm weights
  after ``decay_end`` so the two groups are two contiguous regions.
* FSDP trainer (``fsdp_trainer.py:334-343``): one group, weight decay on everything.

Differences by design: one kernel launch per region instead of
a per-tensor loop; the clip coefficient and the DDP 1/world averaging are computed on
the device and folded into the AdamW grad scale (no ``.item()`` host sync); the
kernel also refreshes the bf16 shadow weights used by the GEMMs.

``state_dict()`` emits the torch AdamW format (int param ids in param-group order,
``{step, exp_avg, exp_avg_sq}``) so checkpoints are interchangeable with the
reference's ``optimizer.state_dict()``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..ops import reference as ref


class FlatAdamW:
    def __init__(self, flat: torch.Tensor, grad: torch.Tensor, shadow: Optional[torch.Tensor],
                 regions: Sequence[Tuple[int, int, float]], lr: float, betas=(0.9, 0.95),
                 eps: float = 1e-8, param_map: Optional[List[List[Tuple[str, int, int, tuple]]]] = None):
        """``regions``: list of (start, end, weight_decay) -- one per param group.
        ``param_map``: per group, the (name, offset, numel, shape) of each parameter, in
        the reference's param order (used for state_dict compatibility)."""
        self.flat, self.grad = flat, grad
        self.shadow = shadow if (shadow is not None and shadow is not flat) else None
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.regions = list(regions)
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=wd, amsgrad=False,
                                  maximize=False, foreach=None, capturable=False, differentiable=False,
                                  fused=None, decoupled_weight_decay=True)
                             for (_, _, wd) in self.regions]
        self.param_map = param_map
        self.step_count = 0
        self.is_cuda = flat.is_cuda
        self._scale_buf = torch.zeros(2, dtype=torch.float32, device=flat.device)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=flat.device)
        self._ones = torch.tensor([0.0, 1.0], dtype=torch.float32, device=flat.device)

    # ----------------------------------------------------------- grad clipping
    def local_sumsq(self) -> torch.Tensor:
        self._sumsq.zero_()
        if self.is_cuda:
            from ..ops import hip
            hip.sumsq(self.grad, self._sumsq)
        else:
            self._sumsq += self.grad.float().pow(2).sum()
        return self._sumsq

    def compute_scale(self, max_norm: float, grad_div: float = 1.0, sumsq: Optional[torch.Tensor] = None
                      ) -> torch.Tensor:
        """Returns a device tensor [total_norm, grad_scale].  The stored grads are
        ``grad_div`` times the true gradient (e.g. a SUM all-reduce over ranks), the
        norm reported is that of the true gradient, and grad_scale = clip_coef/grad_div."""
        if sumsq is None:
            sumsq = self.local_sumsq()
        if self.is_cuda:
            from ..ops import hip
            hip.clip_coef(sumsq, self._scale_buf, 1.0 / grad_div, float(max_norm), 1.0 / grad_div)
        else:
            norm = torch.sqrt(sumsq.reshape(())) / grad_div
            coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones(())
            self._scale_buf[0] = norm
            self._scale_buf[1] = coef / grad_div
        return self._scale_buf

    # ------------------------------------------------------------------- step
    @torch.no_grad()
    def step(self, scale: Optional[torch.Tensor] = None) -> None:
        self.step_count += 1
        sc = scale if scale is not None else self._ones
        for (a, b, _), g in zip(self.regions, self.param_groups):
            if b <= a:
                continue
            self._apply_range(a, b, (g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]), self.step_count, sc,
                              zero_grad=False)

    def step_lazy(self, scale: Optional[torch.Tensor], units: Dict[object, List[Tuple[int, int]]],
                  mode: str = "inline") -> "LazyStep":
        """Record this step instead of running it: each unit's AdamW (and its gradient
        zeroing) is launched when the unit is next needed -- the engine's pre_forward hook
        of the next step (see :class:`LazyStep`).  Same per-element arithmetic, hyper-
        parameters snapshotted now, so the weights come out bitwise as :meth:`step`'s."""
        self.step_count += 1
        self._lazy = LazyStep(self, scale if scale is not None else self._ones, units, mode)
        return self._lazy

    # the last recorded lazy step (state_dict / load_state_dict apply it first, so the
    # moments reported or replaced are those of step_count)
    _lazy = None
    # the stream of LazyStep's "stream" mode, created once and reused by every step
    _lazy_stream = None

    def flush_lazy(self) -> None:
        if self._lazy is not None:
            self._lazy.ensure_all()
            self._lazy = None

    def _apply_range(self, a: int, b: int, hp, step: int, sc: torch.Tensor, zero_grad: bool) -> None:
        """AdamW over flat[a:b] with one group's hyperparameters ``hp`` = (lr, (b1, b2), eps, wd)."""
        lr, (b1, b2), eps, wd = hp
        sh = None if self.shadow is None else self.shadow[a:b]
        if self.is_cuda:
            from ..ops import hip
            hip.adamw_flat(self.flat[a:b], self.grad[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b], sh, lr, b1, b2,
                           eps, wd, step, sc, zero_grad=zero_grad)
        else:
            ref.adamw_step(self.flat[a:b], self.grad[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b], sh, lr, b1, b2,
                           eps, wd, step, sc[1])
            if zero_grad:
                self.grad[a:b].zero_()

    def zero_grad(self, set_to_none: bool = True) -> None:
        # grads are persistent flat views; "set_to_none" semantics = zero the buffer
        self.grad.zero_()

    # ------------------------------------------------------------- state dict
    def state_dict(self) -> Dict:
        self.flush_lazy()
        state, groups, idx = {}, [], 0
        pm = self.param_map or [[("flat", a, b - a, (b - a,))] for (a, b, _) in self.regions]
        for g, plist in zip(self.param_groups, pm):
            ids = []
            for (_name, off, n, shape) in plist:
                state[idx] = {"step": torch.tensor(float(self.step_count)),
                              "exp_avg": self.exp_avg[off:off + n].view(shape).detach().cpu().clone(),
                              "exp_avg_sq": self.exp_avg_sq[off:off + n].view(shape).detach().cpu().clone()}
                ids.append(idx)
                idx += 1
            gg = {k: v for k, v in g.items()}
            gg["params"] = ids
            groups.append(gg)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd: Dict) -> None:
        self.flush_lazy()
        pm = self.param_map or [[("flat", a, b - a, (b - a,))] for (a, b, _) in self.regions]
        st = sd["state"]
        steps = []
        with torch.no_grad():
            for g, sg, plist in zip(self.param_groups, sd["param_groups"], pm):
                for k in ("lr", "betas", "eps", "weight_decay"):
                    if k in sg:
                        g[k] = tuple(sg[k]) if k == "betas" else sg[k]
                for pid, (_name, off, n, shape) in zip(sg["params"], plist):
                    s = st.get(pid) if isinstance(st, dict) else None
                    if s is None:
                        s = st.get(str(pid)) if isinstance(st, dict) else None
                    if s is None:
                        continue
                    self.exp_avg[off:off + n].copy_(s["exp_avg"].reshape(-1).to(self.exp_avg))
                    self.exp_avg_sq[off:off + n].copy_(s["exp_avg_sq"].reshape(-1).to(self.exp_avg_sq))
                    stp = s.get("step", 0)
                    steps.append(int(stp.item() if torch.is_tensor(stp) else stp))
        if steps:
            self.step_count = max(steps)


class LazyStep:
    """A recorded optimizer step, applied unit by unit where the next forward needs it.

    The reference steps every parameter at the end of the step (``ddp_trainer.py:352-356``),
    a memory-bound pass with nothing to overlap (1.03 ms of a 41 ms step alone on the
    GPU, profiles/r4_step_breakdown_final.md).  Here the trainer records the step (clip
    scale, lr, betas, eps, wd, step count) and the flat store's ``pre_forward(unit)`` hook
    launches that unit's AdamW -- which also zeroes its gradient -- right before the
    unit's first use in the next forward:

    * ``inline``: on the stream of the first chain that reaches the unit; the other
      chain's stream waits for an event.  In the two-chain ``ffbb`` window a unit's
      update runs beside the other chain's previous layer.
    * ``stream``: every unit is issued at once, in forward order, on a stream of its own
      (one event per unit), so the updates run ahead beside the forward of both chains.

    Anything that reads the weights outside a training forward (checkpoint save, eval,
    decode, ``state_dict``) calls :meth:`ensure_all` first (the trainer does; the store's
    ``flush_pending``).  Units are disjoint flat ranges (:meth:`FlatParamStore.unit_ranges`).
    """

    def __init__(self, opt: FlatAdamW, scale: torch.Tensor, units: Dict[object, List[Tuple[int, int]]], mode: str):
        self.opt = opt
        self.step = opt.step_count
        self.scale = scale.detach().clone()  # the next step's compute_scale reuses the buffer
        self.hp = [(g["lr"], tuple(g["betas"]), g["eps"], g["weight_decay"]) for g in opt.param_groups]
        self.units = {u: list(r) for u, r in units.items()}
        self.mode = mode if opt.is_cuda else "inline"
        self.events: Dict[object, object] = {}
        self.done = set()
        self._stream = None
        covered = sorted(x for r in self.units.values() for x in r)
        pos = 0
        for a, b in covered:
            if a != pos:
                raise ValueError(f"lazy optimizer units leave [{pos}, {a}) of the flat buffer uncovered")
            pos = b
        if pos != opt.flat.numel():
            raise ValueError("lazy optimizer units do not cover the flat buffer")

    def _launch(self, unit) -> None:
        for (a, b) in self.units[unit]:
            for (ra, rb, _), hp in zip(self.opt.regions, self.hp):
                lo, hi = max(a, ra), min(b, rb)
                if hi > lo:
                    self.opt._apply_range(lo, hi, hp, self.step, self.scale, zero_grad=True)
        self.done.add(unit)

    def _issue_all_on_stream(self) -> None:
        cur = torch.cuda.current_stream()
        if self._stream is None:
            # one stream for every step (kept on the optimizer): a fresh torch.cuda.Stream
            # per step cycles through PyTorch's stream pool and would periodically alias
            # the engine's or RCCL's streams
            if self.opt._lazy_stream is None or self.opt._lazy_stream.device != cur.device:
                self.opt._lazy_stream = torch.cuda.Stream(cur.device)
            self._stream = self.opt._lazy_stream
        self._stream.wait_stream(cur)  # after the step's clip scale and the gradient all-reduces
        with torch.cuda.stream(self._stream):
            for u in self.units:
                self._launch(u)
                ev = torch.cuda.Event()
                ev.record()
                self.events[u] = ev

    def ensure(self, unit) -> None:
        """Make ``unit``'s update visible to the current stream (launching it if needed)."""
        if unit not in self.units:
            return
        if self.mode == "stream":
            if not self.events:
                self._issue_all_on_stream()
            torch.cuda.current_stream().wait_event(self.events[unit])
            return
        if unit in self.done:
            ev = self.events.get(unit)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            return
        self._launch(unit)
        if self.opt.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.events[unit] = ev

    def ensure_all(self) -> None:
        for u in self.units:
            self.ensure(u)

    def discard(self) -> None:
        """Give the step up: units not yet updated only get their gradients zeroed (what
        the update would also have done); units already launched stay applied."""
        if self.mode == "stream" and self.events:
            return  # every unit was issued with the first ensure
        for u, ranges in self.units.items():
            if u in self.done:
                continue
            for (a, b) in ranges:
                self.opt.grad[a:b].zero_()
            self.done.add(u)
        if self.opt._lazy is self:
            self.opt._lazy = None

    @property
    def complete(self) -> bool:
        return len(self.done) == len(self.units)


def flat_store_optimizer(store, lr: float, betas, eps: float, weight_decay: float,
                         split_no_decay: bool = True) -> FlatAdamW:
    """AdamW over a FlatParamStore; groups mirror the reference DDP (split) or FSDP (single)."""
    lay = store.layout
    model = store.model
    names = [n for n, _ in model.named_parameters()]
    by = lay.by_name

    def pm(filter_fn):
        out = []
        for n in names:
            if filter_fn(n):
                s = by[n]
                out.append((n, s.offset, s.numel, s.shape))
        return out

    if split_no_decay:
        regions = [(0, lay.decay_end, weight_decay), (lay.decay_end, lay.total, 0.0)]
        nd = lambda n: ("bias" in n) or ("norm" in n)  # noqa: E731 (reference rule)
        param_map = [pm(lambda n: not nd(n)), pm(nd)]
    else:
        regions = [(0, lay.total, weight_decay)]
        param_map = [pm(lambda n: True)]
    return FlatAdamW(store.flat, store.grad, store.shadow, regions, lr, betas, eps, param_map)
