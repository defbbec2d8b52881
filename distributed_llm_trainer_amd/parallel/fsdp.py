"""Fully-sharded data parallelism (ZeRO-3 / ZeRO-2 / DDP-equivalent / hybrid) for the
fused GPT executor, on RCCL collectives.

Parity target: ``torch.distributed.fsdp.FullyShardedDataParallel`` as configured by
the reference (``fsdp_trainer.py:158-332``; SURVEY §2.4 P2-P6, call stack §3.2):
one flat parameter per ``TransformerBlock`` plus a root unit holding the tied
embedding/lm_head and the final norm; fp32 master shards; bf16 all-gather before use;
reshard after forward (FULL_SHARD) or keep until backward (SHARD_GRAD_OP); bf16
reduce-scatter of gradients into the fp32 shard; optimizer on shards; optional CPU
offload of master params/optimizer (host AdamW); BACKWARD_PRE prefetch with at most
one gather in flight beyond the one being consumed (``limit_all_gathers``).

MI355X-specific design choices:

* Unit = one flat buffer laid out ``[q|k|v|o|gate|up|down|ln1|ln2]`` so the
  gathered bf16 buffer is directly the packed QKV / gate|up GEMM operands (no
  unflatten copies).  The root unit ``[embed(Vp rows)|norm]`` keeps the padded
  vocabulary rows so the gathered buffer IS the lm_head operand.
* The executor calls ``pre_forward/post_forward/pre_backward/post_backward`` per
  unit, so the next unit's all-gather is issued on RCCL's stream BEFORE the current
  unit's kernels run (forward prefetch) and, in backward, before the current unit's
  recompute+backward (BACKWARD_PRE).  Reduce-scatters are issued as soon as a unit's
  gradients are final and overlap the next unit's backward.
* Shards are padded to a multiple of 4 elements (16-byte aligned slices for the
  vectorised AdamW kernel); the shard's bf16 shadow (written by AdamW) is the
  all-gather input, so there is no per-step cast kernel.
* On one 8x MI355X node the all-gathers/reduce-scatters ride RCCL over the xGMI
  full mesh; block units are 18.9 MB (small) .. 81.9 MB (xl) bf16 -- large enough
  for RCCL to stripe over all 7 links.

Gradient semantics: gradients are SUMMED over ranks by the reduce-scatter (reduce in
``reduce_dtype``) and the 1/world averaging is folded into the AdamW scale, like
``parallel/ddp.py``.  ``sync_every_micro_step`` reproduces the reference, which
reduce-scatters on every micro-step (no ``no_sync``, Q15); turning it off keeps the
full-size fp32 unit gradients across micro-steps and reduce-scatters once.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..models.engine import HeadGrads, HeadWeights, LayerGrads, LayerWeights, ParamProvider

STRATEGIES = ("FULL_SHARD", "SHARD_GRAD_OP", "NO_SHARD", "HYBRID_SHARD")


def _add_bf16(dst: torch.Tensor, src: torch.Tensor) -> bool:
    """fp32 dst += bf16 src with the fused HIP kernel (ops/csrc/optim.hip)."""
    from ..ops import hip
    return hip.add_bf16_into_f32(dst, src)


@dataclass
class _Seg:
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]


class FlatUnit:
    """One FSDP unit: a flat parameter, its shard (views into the runtime's contiguous
    shard buffers), and its transient full buffers."""

    def __init__(self, uid, segs: List[_Seg], numel: int, world: int, rank: int, device, compute_dtype):
        self.uid = uid
        self.segs = segs
        self.numel = numel
        self.world = world
        self.rank = rank
        self.device = device
        per = -(-numel // world)
        per = ((per + 3) // 4) * 4
        self.shard = per
        self.padded = per * world
        self.compute_dtype = compute_dtype
        self.master = None   # fp32 shard (device, or pinned host with cpu_offload)
        self.grad = None     # fp32 shard grad
        self.shard_c = None  # compute-dtype shard on device = all-gather input (AdamW writes it)
        self.full: Optional[torch.Tensor] = None        # gathered compute-dtype params
        self.full_grad: Optional[torch.Tensor] = None   # full fp32 grads during backward
        self.ag_work = None
        self.rs_pending = []
        self.host_bufs = []      # cpu_offload: pinned staging buffers, one per pending reduce
        self.refs = 0            # chains (forward / backward of a micro-step) using `full`
        self.ready_ev = None     # HIP event: `full` is complete (recorded after the gather wait)
        self.norm_grad = None    # bf16-gradient mode: fp32 ln1 | ln2 gradients of the micro-step
        self.head_q = []         # root unit: gradient buffers of backwards issued but not yet reduced

    def local_slice(self) -> Tuple[int, int]:
        return self.rank * self.shard, (self.rank + 1) * self.shard


class FSDPRuntime(ParamProvider):
    # Overlapped backwards (GPTEngine.train_window): every micro-step gets fresh unit
    # gradient buffers (layer_grads / head_grads, reduced and dropped in post_backward), the
    # host issues the two backwards' hooks in sequential order, and the shard gradients
    # are only accumulated in finish() -- nothing two backwards write is shared.
    overlap_backward_ok = True

    def __init__(self, model, device, sharding_strategy: str = "FULL_SHARD", compute_dtype=torch.bfloat16,
                 reduce_dtype=torch.bfloat16, cpu_offload: bool = False, backward_prefetch: str = "BACKWARD_PRE",
                 limit_all_gathers: bool = True, sync_every_micro_step: bool = True, process_group=None,
                 replicate_group=None):
        strat = sharding_strategy.upper()
        if strat not in STRATEGIES:
            raise ValueError(f"unknown sharding strategy {sharding_strategy!r}; choose from {STRATEGIES}")
        self.model = model
        self.cfg = model.config
        self.device = torch.device(device)
        self.strategy = strat
        self.compute_dtype = compute_dtype
        self.reduce_dtype = reduce_dtype
        self.cpu_offload = cpu_offload
        self.prefetch = backward_prefetch.upper()
        self.limit_all_gathers = limit_all_gathers
        self.sync_every_micro_step = sync_every_micro_step
        self.sync = True
        self.dist = dist.is_initialized()
        self.pg = process_group
        self.rep_pg = replicate_group
        if strat == "HYBRID_SHARD" and self.dist and process_group is None:
            self.pg, self.rep_pg = _hybrid_groups()
        world = dist.get_world_size(self.pg) if self.dist else 1
        rank = dist.get_rank(self.pg) if self.dist else 0
        if strat == "NO_SHARD":
            self.shard_world, self.shard_rank = 1, 0
        else:
            self.shard_world, self.shard_rank = world, rank
        self.world = dist.get_world_size() if self.dist else 1
        # DLT_FORCE_COLLECTIVES=1 (see parallel/ddp.py): one rank still all-gathers and
        # reduce-scatters through the process group instead of aliasing its shard
        self.force = self.dist and self.world == 1 and os.environ.get("DLT_FORCE_COLLECTIVES") == "1"
        # Per-micro-step unit gradients straight in the reduce dtype: with bf16 reduction
        # on every micro-step (the reference's FSDP schedule) the weight-gradient GEMMs
        # write the bf16 send buffer directly (beta = 0, HipGemm.wgrad_set), the norm
        # weights accumulate in a tiny fp32 side buffer that is cast into it before the
        # reduce-scatter -- no fp32 zero / accumulate / cast passes over the unit.
        # (bf16, and fp16 under the fp16 policy: "bf16_grads" = 16-bit gradients in the
        # reduce dtype, which must equal the compute dtype the GEMM operands use)
        self.bf16_grads = (reduce_dtype in (torch.bfloat16, torch.float16) and reduce_dtype == compute_dtype
                           and sync_every_micro_step and self.device.type == "cuda"
                           and os.environ.get("DLT_FSDP_BF16_GRADS", "1") != "0")
        # limit_all_gathers (reference fsdp_trainer.py:296): at most this many prefetched
        # (issued ahead of use, not yet consumed) all-gathers in flight -- one per
        # micro-step chain (GPTEngine.train_window runs two chains)
        self.max_prefetch = 2 if limit_all_gathers else 1 << 30
        self._prefetched = set()
        self._rep_stream = None  # HYBRID_SHARD: replicate all-reduces off the compute stream
        self._d2h_stream = None  # cpu_offload: reduced shards copied to pinned host buffers
        self.units: Dict[object, FlatUnit] = {}
        self._build_units(model)
        self._free_module_params(model)
        self.hooks = None

    @property
    def collectives(self) -> bool:
        """True when all-gathers / reduce-scatters go through the process group (several
        ranks, or one rank with DLT_FORCE_COLLECTIVES=1): GPTEngine.window_schedule then
        keeps the fb window."""
        return bool(self.dist and (self.world > 1 or self.force))

    # ------------------------------------------------------------------ build
    def _unit_layout(self, uid):
        cfg = self.cfg
        H, I, Vp = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size_padded
        segs, off = [], 0

        def add(name, shape, alloc=None):
            nonlocal off
            n = 1
            for s in shape:
                n *= s
            segs.append(_Seg(name, off, n, tuple(shape)))
            off += alloc if alloc is not None else n

        if uid == "head":
            add("embed_tokens.weight", (cfg.vocab_size, H), alloc=Vp * H)
            add("norm.weight", (H,))
        else:
            p = f"layers.{uid}."
            add(p + "attention.q_proj.weight", (H, H))
            add(p + "attention.k_proj.weight", (H, H))
            add(p + "attention.v_proj.weight", (H, H))
            add(p + "attention.o_proj.weight", (H, H))
            add(p + "mlp.gate_proj.weight", (I, H))
            add(p + "mlp.up_proj.weight", (I, H))
            add(p + "mlp.down_proj.weight", (H, I))
            add(p + "input_layernorm.weight", (H,))
            add(p + "post_attention_layernorm.weight", (H,))
        return segs, off

    @torch.no_grad()
    def _build_units(self, model):
        named = dict(model.named_parameters())
        order = list(range(self.cfg.num_layers)) + ["head"]
        for uid in order:
            segs, n = self._unit_layout(uid)
            self.units[uid] = FlatUnit(uid, segs, n, self.shard_world, self.shard_rank, self.device,
                                       self.compute_dtype)
        total = sum(u.shard for u in self.units.values())
        pdev = torch.device("cpu") if self.cpu_offload else self.device
        pin = self.cpu_offload and torch.cuda.is_available()
        self.master_flat = torch.zeros(total, dtype=torch.float32, device=pdev)
        self.grad_flat = torch.zeros(total, dtype=torch.float32, device=pdev)
        if pin:
            self.master_flat = self.master_flat.pin_memory()
            self.grad_flat = self.grad_flat.pin_memory()
        if self.compute_dtype == torch.float32 and not self.cpu_offload:
            self.shard_c_flat = self.master_flat  # fp32 policy: the master shard IS the all-gather input
        else:
            self.shard_c_flat = torch.zeros(total, dtype=self.compute_dtype, device=self.device)
        off = 0
        self.unit_offsets = {}
        for uid in order:
            u = self.units[uid]
            u.master = self.master_flat[off:off + u.shard]
            u.grad = self.grad_flat[off:off + u.shard]
            u.shard_c = self.shard_c_flat[off:off + u.shard]
            self.unit_offsets[uid] = (off, off + u.shard)
            off += u.shard
        for uid in order:
            u = self.units[uid]
            segs = u.segs
            full = torch.zeros(u.padded, dtype=torch.float32)
            for s in segs:
                full[s.offset:s.offset + s.numel].copy_(named[s.name].detach().reshape(-1).cpu())
            a, b = u.local_slice()
            u.master.copy_(full[a:b])
            u.shard_c.copy_(full[a:b].to(self.compute_dtype))

    def _free_module_params(self, model):
        """The module keeps tiny placeholders; real storage lives in the shards."""
        for p in model.parameters():
            p.data = torch.empty(0, dtype=p.dtype, device=self.device)
            p.grad = None

    # ---------------------------------------------------------- collectives
    def _prefetch(self, u: FlatUnit):
        """Issue an all-gather ahead of use, within the limit_all_gathers budget (a
        unit that does not get one is gathered synchronously when it is acquired)."""
        if u.full is not None:
            return
        self._prefetched = {x for x in self._prefetched if x.ag_work is not None and x.refs == 0}
        if len(self._prefetched) >= self.max_prefetch:
            return
        self._gather(u, async_op=True)
        if u.ag_work is not None:
            self._prefetched.add(u)

    def _gather(self, u: FlatUnit, async_op: bool):
        if u.full is not None and u.ag_work is None:
            return
        if u.full is None:
            if self.shard_world == 1 and not self.force:  # NO_SHARD: the "gathered" buffer IS the local replica
                u.full = u.shard_c
                return
            u.full = torch.empty(u.padded, dtype=self.compute_dtype, device=self.device)
            u.ag_work = dist.all_gather_into_tensor(u.full, u.shard_c, group=self.pg, async_op=async_op)
            if not async_op:
                u.ag_work = None

    def _wait_gather(self, u: FlatUnit):
        waited = False
        if u.full is None:
            self._gather(u, async_op=False)
            waited = True
        if u.ag_work is not None:
            u.ag_work.wait()
            u.ag_work = None
            waited = True
        if waited and u.full is not None and u.full.is_cuda:
            u.ready_ev = torch.cuda.Event()
            u.ready_ev.record()

    # Residency is reference-counted so that two chains (the forward of micro-step k+1
    # and the backward of micro-step k, interleaved on two HIP streams by
    # GPTEngine.train_window) can share a gathered unit: the buffer is resharded only
    # when the last user releases it, every user's stream waits for the gather's
    # completion event, and the buffer is recorded on every stream that read it.
    def _acquire(self, u: FlatUnit):
        self._prefetched.discard(u)
        self._wait_gather(u)
        if u.full is not None and u.full.is_cuda:
            cur = torch.cuda.current_stream(self.device)
            if u.ready_ev is not None:
                cur.wait_event(u.ready_ev)
            if u.full is not u.shard_c:
                u.full.record_stream(cur)
        u.refs += 1

    def _release(self, u: FlatUnit, reshard: bool):
        u.refs = max(0, u.refs - 1)
        if reshard and u.refs == 0:
            self._reshard(u)

    def _reshard(self, u: FlatUnit):
        if u.ag_work is not None:
            u.ag_work.wait()
            u.ag_work = None
        u.full = None
        u.ready_ev = None

    def _reduce(self, u: FlatUnit):
        """Sum full-size grads over ranks into this rank's fp32 shard grad (async)."""
        g = u.full_grad
        if self.shard_world == 1 and not (self.force and self.strategy != "NO_SHARD"):
            # the reduce-dtype copy also on one rank: it is what stays pending until
            # finish() (half the bytes of the fp32 full grad, which is freed here)
            t = g if self.reduce_dtype == torch.float32 else g.to(self.reduce_dtype)
            work = None
            if self.dist and (self.world > 1 or self.force):
                work = dist.all_reduce(t, group=self.pg if self.strategy != "NO_SHARD" else None, async_op=True)
            u.rs_pending.append(self._stage_host(u, work, t, None))
        else:
            src = g if self.reduce_dtype == torch.float32 else g.to(self.reduce_dtype)
            out = torch.empty(u.shard, dtype=src.dtype, device=self.device)
            work = dist.reduce_scatter_tensor(out, src, group=self.pg, async_op=True)
            if self.rep_pg is not None and self.strategy == "HYBRID_SHARD":
                # replicate all-reduce chained behind the reduce-scatter on a side stream:
                # overlaps the rest of the backward instead of running inside finish()
                if self._rep_stream is None:
                    self._rep_stream = torch.cuda.Stream(self.device) if out.is_cuda else None
                ctx = torch.cuda.stream(self._rep_stream) if self._rep_stream is not None else None
                if ctx is not None:
                    with ctx:
                        work.wait()  # device-side: the side stream waits for the reduce-scatter
                        out.record_stream(self._rep_stream)
                        work = dist.all_reduce(out, group=self.rep_pg, async_op=True)
                else:
                    work.wait()
                    work = dist.all_reduce(out, group=self.rep_pg, async_op=True)
            u.rs_pending.append(self._stage_host(u, work, out, src))
        u.full_grad = None

    def _stage_host(self, u: FlatUnit, work, out: torch.Tensor, src):
        """cpu_offload: copy the reduced shard to a pinned host buffer as soon as its
        collective completes -- on a copy stream that waits for it on the device, so the
        D2H transfer overlaps the rest of the backward instead of a blocking ``.cpu()`` per
        unit in finish(), which then only waits for the copy and adds on the host.
        Returns the rs_pending entry (work, out, src, host, event)."""
        if not (self.cpu_offload and out.is_cuda):
            return (work, out, src, None, None)
        if self._d2h_stream is None:
            self._d2h_stream = torch.cuda.Stream(self.device)
        k = len(u.rs_pending)
        n = min(out.numel(), u.shard)
        while len(u.host_bufs) <= k:
            u.host_bufs.append(None)
        host = u.host_bufs[k]
        if host is None or host.numel() != n or host.dtype != out.dtype:
            host = torch.empty(n, dtype=out.dtype, pin_memory=True)
            u.host_bufs[k] = host
        cur = torch.cuda.current_stream(self.device)
        self._d2h_stream.wait_stream(cur)  # `out` / the collective were issued from here
        with torch.cuda.stream(self._d2h_stream):
            if work is not None:
                work.wait()  # device-side: the copy stream waits for the collective
            host.copy_(out[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        out.record_stream(self._d2h_stream)
        return (None, out, src, host, ev)

    def _finish_reduce(self, u: FlatUnit):
        for work, out, _src, host, ev in u.rs_pending:
            if host is not None:  # cpu_offload: the staged D2H copy (see _stage_host)
                ev.synchronize()
                u.grad.add_(host)
                continue
            if work is not None:
                work.wait()
            if out.numel() != u.shard:  # NO_SHARD: full buffer == shard
                out = out[:u.shard]
            if out.is_cuda:  # produced on the backward's stream (maybe the pipeline stream)
                out.record_stream(torch.cuda.current_stream(out.device))
            if self.cpu_offload:
                u.grad.add_(out.cpu())
            elif not (out.is_cuda and out.dtype in (torch.bfloat16, torch.float16) and _add_bf16(u.grad, out)):
                u.grad.add_(out)  # add_ promotes the wire dtype inside the kernel
        u.rs_pending.clear()

    def finish(self):
        for u in self.units.values():
            self._finish_reduce(u)

    # ------------------------------------------------------------ provider
    def _view(self, u: FlatUnit, buf: torch.Tensor, name: str, rows: int = None, cols: int = None):
        for s in u.segs:
            if s.name == name:
                if rows is None:
                    return buf[s.offset:s.offset + s.numel]
                return buf[s.offset:s.offset + rows * cols].view(rows, cols)
        raise KeyError(name)

    def layer(self, i):
        u = self.units[i]
        self._wait_gather(u)
        H, I = self.cfg.hidden_size, self.cfg.intermediate_size
        p = f"layers.{i}."
        f = u.full
        return LayerWeights(wqkv=self._view(u, f, p + "attention.q_proj.weight", 3 * H, H),
                            wo=self._view(u, f, p + "attention.o_proj.weight", H, H),
                            wgu=self._view(u, f, p + "mlp.gate_proj.weight", 2 * I, H),
                            wdown=self._view(u, f, p + "mlp.down_proj.weight", H, I),
                            ln1=self._view(u, f, p + "input_layernorm.weight"),
                            ln2=self._view(u, f, p + "post_attention_layernorm.weight"))

    def layer_grads(self, i):
        u = self.units[i]
        H, I = self.cfg.hidden_size, self.cfg.intermediate_size
        if u.full_grad is None:
            if self.bf16_grads:  # every segment is written (not accumulated) once per micro-step
                u.full_grad = torch.empty(u.padded, dtype=self.reduce_dtype, device=self.device)
                if u.padded > u.numel:
                    u.full_grad[u.numel:].zero_()
                u.norm_grad = torch.zeros(2 * H, dtype=torch.float32, device=self.device)
            else:
                u.full_grad = torch.zeros(u.padded, dtype=torch.float32, device=self.device)
        p = f"layers.{i}."
        g = u.full_grad
        if g.dtype in (torch.bfloat16, torch.float16):
            ln1, ln2 = u.norm_grad[:H], u.norm_grad[H:]
        else:
            ln1 = self._view(u, g, p + "input_layernorm.weight")
            ln2 = self._view(u, g, p + "post_attention_layernorm.weight")
        return LayerGrads(wqkv=self._view(u, g, p + "attention.q_proj.weight", 3 * H, H),
                          wo=self._view(u, g, p + "attention.o_proj.weight", H, H),
                          wgu=self._view(u, g, p + "mlp.gate_proj.weight", 2 * I, H),
                          wdown=self._view(u, g, p + "mlp.down_proj.weight", H, I),
                          ln1=ln1, ln2=ln2)

    def head(self):
        u = self.units["head"]
        self._wait_gather(u)
        H, Vp = self.cfg.hidden_size, self.cfg.vocab_size_padded
        e = u.full[:Vp * H].view(Vp, H)
        return HeadWeights(embed=e, lm_head=e, norm=self._view(u, u.full, "norm.weight"))

    def head_grads(self):
        """A fresh root-unit gradient buffer per backward (FIFO): the two-chain window
        issues both backwards interleaved, each asks for its buffer at its start, and
        post_backward("head") reduces them in the same order."""
        u = self.units["head"]
        if self.sync_every_micro_step:
            g = torch.zeros(u.padded, dtype=torch.float32, device=self.device)
            u.head_q.append(g)
        else:  # accumulated over the micro-steps until the synchronising one
            if u.full_grad is None:
                u.full_grad = torch.zeros(u.padded, dtype=torch.float32, device=self.device)
            g = u.full_grad
        H, Vp = self.cfg.hidden_size, self.cfg.vocab_size_padded
        return HeadGrads(embed=g[:Vp * H].view(Vp, H), norm=self._view(u, g, "norm.weight"))

    # ------------------------------------------------------------------- hooks
    def _next(self, uid, forward: bool):
        L = self.cfg.num_layers
        if forward:
            if uid == "head":
                return 0 if L > 0 else None
            return uid + 1 if uid + 1 < L else None
        if uid == "head":
            return L - 1 if L > 0 else None
        return uid - 1 if uid - 1 >= 0 else None

    def pre_forward(self, uid):
        u = self.units[uid]
        self._acquire(u)
        nxt = self._next(uid, True)
        if nxt is not None:  # forward prefetch of the next unit
            self._prefetch(self.units[nxt])

    def post_forward(self, uid):
        # the root stays gathered until its backward (like FSDP's root unit)
        self._release(self.units[uid], reshard=uid != "head" and self.strategy in ("FULL_SHARD", "HYBRID_SHARD"))

    def pre_backward(self, uid):
        u = self.units[uid]
        self._acquire(u)
        if self.prefetch == "BACKWARD_PRE":
            nxt = self._next(uid, False)
            if nxt is not None and nxt != "head":
                self._prefetch(self.units[nxt])

    def post_backward(self, uid):
        u = self.units[uid]
        if u.full_grad is not None and u.full_grad.dtype in (torch.bfloat16, torch.float16) and uid != "head":
            # the norm-weight gradients (fp32 side buffer) into the bf16 send buffer
            H = self.cfg.hidden_size
            p = f"layers.{uid}."
            torch._foreach_copy_([self._view(u, u.full_grad, p + "input_layernorm.weight"),
                                  self._view(u, u.full_grad, p + "post_attention_layernorm.weight")],
                                 [u.norm_grad[:H], u.norm_grad[H:]])  # one multi-tensor launch
            u.norm_grad = None
        if uid == "head" and u.head_q:
            u.full_grad = u.head_q.pop(0)
        do_reduce = self.sync or self.sync_every_micro_step
        if do_reduce:
            self._reduce(u)
        self._release(u, reshard=self.strategy != "NO_SHARD")
        if uid != "head" and self.prefetch == "BACKWARD_POST":
            nxt = self._next(uid, False)
            if nxt is not None and nxt != "head":
                self._prefetch(self.units[nxt])

    def require_sync(self, flag: bool):
        self.sync = bool(flag)

    # ------------------------------------------------------------ optimizer
    def flat_views(self):
        """(master, grad, shard_c) per unit, in unit order."""
        return [(u.master, u.grad, u.shard_c) for u in self.units.values()]

    def zero_grad(self):
        self.grad_flat.zero_()
        for u in self.units.values():
            u.full_grad = None
            u.head_q.clear()

    def refresh_shadow(self):
        """Re-derive the device compute-dtype shards from the fp32 masters."""
        if self.shard_c_flat is not self.master_flat:
            self.shard_c_flat.copy_(self.master_flat.to(self.device).to(self.compute_dtype))

    # ------------------------------------------------------------ state dict
    def _is_rank0(self) -> bool:
        return not self.dist or dist.get_rank() == 0

    @torch.no_grad()
    def full_param_flat(self, uid, rank0_only: bool = False) -> Optional[torch.Tensor]:
        """Gather a unit's fp32 master params (FULL_STATE_DICT).  With ``rank0_only``
        (the reference's ``FullStateDictConfig(offload_to_cpu=True, rank0_only=True)``,
        ``fsdp_trainer.py:447``) only rank 0 gets the host copy; the other ranks take part
        in the device all-gather and return None."""
        return self.gather_shard_tensor(uid, self.units[uid].master, rank0_only=rank0_only)

    @torch.no_grad()
    def gather_shard_tensor(self, uid, shard: torch.Tensor, rank0_only: bool = False) -> Optional[torch.Tensor]:
        u = self.units[uid]
        src = shard.to(self.device).float()
        if self.shard_world == 1:
            return src.cpu() if (not rank0_only or self._is_rank0()) else None
        out = torch.empty(u.padded, dtype=torch.float32, device=self.device)
        dist.all_gather_into_tensor(out, src, group=self.pg)
        if rank0_only and not self._is_rank0():
            return None  # the device buffer is freed at once: no host copy on this rank
        return out.cpu()

    @torch.no_grad()
    def load_full_flat(self, uid, full: torch.Tensor) -> None:
        u = self.units[uid]
        a, b = u.local_slice()
        u.master.copy_(full[a:b].to(u.master.device))
        u.shard_c.copy_(full[a:b].to(self.device).to(self.compute_dtype))

    def state_dict_full(self, rank0_only: bool = False) -> Optional[Dict[str, torch.Tensor]]:
        """Reference-format fp32 state dict (gathers every unit; collective).  With
        ``rank0_only`` the other ranks return None and never hold a host copy."""
        sd = {}
        for uid, u in self.units.items():
            full = self.full_param_flat(uid, rank0_only=rank0_only)
            if full is None:
                continue
            for s in u.segs:
                sd[s.name] = full[s.offset:s.offset + s.numel].view(s.shape).clone()
        return sd if (not rank0_only or self._is_rank0()) else None


def _hybrid_groups():
    """(shard group = ranks of this node, replicate group = same local rank across nodes)."""
    import os
    world = dist.get_world_size()
    rank = dist.get_rank()
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    nnodes = max(1, world // local)
    shard_groups = [dist.new_group(list(range(n * local, (n + 1) * local))) for n in range(nnodes)]
    rep_groups = [dist.new_group(list(range(l, world, local))) for l in range(local)]
    return shard_groups[rank // local], rep_groups[rank % local]
