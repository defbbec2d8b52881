"""Data-parallel gradient reduction over RCCL (xGMI) with layer-granular overlap.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as used by the reference
(``ddp_trainer.py:167-172,329-332``).  What it does
differently, by design for an 8x MI355X xGMI full mesh:

* **Zero-copy buckets.** Gradients already live in one flat fp32 buffer
  (``parallel/flat.py``) whose layer regions are contiguous, so a bucket is a slice:
  no flatten/unflatten copy kernels.
* **Big buckets.** Default 64 MB (vs DDP's 25 MB / 1 MB first bucket).  A ring
  all-reduce over xGMI is per-link bound and RCCL spreads a large message over
  several channels/links; fewer, larger collectives amortise the ~10-20 us launch
  and protocol cost.  (small: 607 MB of fp32 grads -> ~10 buckets.)
* **Layer-granular overlap.** The fused executor calls ``post_backward(i)`` when
  layer i's weight gradients are final; the bucket whose lowest layer is i is then
  enqueued on RCCL's stream (async) while layer i-1's backward keeps computing.
* **no_sync.** Only the micro-step that calls ``require_sync(True)`` reduces
  (reference GA semantics, ``ddp_trainer.py:329-332``).
* **No per-step buffer broadcast.** The reference's DDP rebroadcasts the RoPE
  buffers every step (X3); they are deterministic, so we don't.
* **Averaging folded into the optimizer.** All-reduce uses SUM; the 1/world factor
  is applied inside the AdamW kernel together with the clip coefficient.
* Optional ``reduce_dtype=torch.bfloat16`` halves the bytes on the wire (the fp32
  accumulation buffer is kept; bf16 is only the transport).
* **Split head bucket.**  The tied embedding / lm_head gradient has two parts: the
  lm_head weight gradient (dense [Vp, H], one GEMM at the START of the window's last
  backward, ``GPTEngine`` deferred head) and the embedding scatter-add (at its END, only
  the rows of tokens in the batch).  The engine hands the lm_head part over
  (:meth:`head_wgrad_ready`): it is all-reduced right away, overlapped with the whole
  layer backward, and added in :meth:`finish`.  The embedding part is reduced row-sparse:
  the ranks agree on the union of their non-zero rows (one byte per row, MAX all-reduce)
  and all-reduce only those rows -- dense when the union covers over half of the rows
  (uniform random tokens at W = 8).  Before round 6 the whole 154 MB fp32 head bucket was
  reduced after the embedding backward with nothing left to overlap
  (``profiles/r5_comm_model.md``: 0.6-1.3 ms exposed at W = 8).
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


class DDPRuntime:
    def __init__(self, store, process_group=None, bucket_cap_mb: float = 64.0,
                 reduce_dtype: torch.dtype = torch.float32, broadcast_init: bool = True):
        self.store = store
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.reduce_dtype = reduce_dtype
        self.sync = True
        # DLT_FORCE_COLLECTIVES=1: issue every collective even on one rank, so a one-GPU
        # box runs the multi-GPU code path (RCCL kernels launched from the weight-gradient
        # stream, waits, the bucket schedule) with a result that must equal no collectives
        self.force = dist.is_initialized() and self.world == 1 and os.environ.get("DLT_FORCE_COLLECTIVES") == "1"
        self.launched = 0
        self.handles: List[Tuple[object, Optional[torch.Tensor], int, int]] = []
        # the lm_head part of the tied gradient taken over this step (head_wgrad_ready):
        # (work, buffer, transport tensor or None), added into the grad in finish()
        self.head_parts: List[Tuple[object, torch.Tensor, Optional[torch.Tensor]]] = []
        # row-sparse embedding reductions in flight: (work, rows, index, a, b, H)
        self.row_handles: List[Tuple[object, torch.Tensor, torch.Tensor, int, int, int]] = []
        self.split_head = os.environ.get("DLT_DDP_SPLIT_HEAD", "1") != "0"
        # row-sparse embedding part (opt-in): reduce only the union of non-zero rows when it
        # is at most this share of the rows.  Finding the union costs a host sync on its row
        # count at the end of every backward: -1 % on a forced-RCCL rank with synthetic
        # tokens (union = every row, dense anyway; tools/ab/r6/rccl_knobs.sh), so 0 = dense.
        self.sparse_rows_max = float(os.environ.get("DLT_DDP_SPARSE_ROWS", "0"))
        self.last_head = None  # how the last embedding bucket was reduced: "dense" / ("rows", U, Vp)
        lay = store.layout
        elem = store.grad.element_size()
        cap = max(1, int(bucket_cap_mb * 1024 * 1024 / elem))
        # buckets over layers, formed from the LAST layer downwards (backward order)
        self.fire_at = {}  # unit -> list of (start, end)
        L = len(lay.layer_bounds)
        i = L - 1
        while i >= 0:
            j = i
            end = lay.layer_bounds[i][1]
            while j > 0 and end - lay.layer_bounds[j - 1][0] <= cap:
                j -= 1
            start = lay.layer_bounds[j][0]
            self.fire_at.setdefault(j, []).append((start, end))
            i = j - 1
        # embedding (tied lm_head) + all norm weights: final after the embedding bwd
        self.fire_at.setdefault("head", []).append((lay.embed_offset, lay.total))
        self.embed_range = (lay.embed_offset, lay.decay_end)
        self.hidden = store.cfg.hidden_size
        self.buckets = [b for v in self.fire_at.values() for b in v]
        if broadcast_init and (self.world > 1 or self.force):
            self.broadcast_parameters()
        store.hooks = self

    # ------------------------------------------------------------------ init
    @torch.no_grad()
    def broadcast_parameters(self) -> None:
        """Rank 0's weights win (one flat broadcast instead of DDP's per-bucket X2).  A
        pending lazy optimizer step is applied first, so the broadcast carries final weights
        and nothing is replayed on top of them afterwards."""
        self.store.flush_pending()
        dist.broadcast(self.store.flat, src=0, group=self.pg)
        self.store.refresh_shadow()

    # ----------------------------------------------------------------- no_sync
    def require_sync(self, flag: bool) -> None:
        self.sync = bool(flag)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.sync
        self.sync = False
        try:
            yield
        finally:
            self.sync = old

    # ------------------------------------------------------------------- hooks
    def pre_forward(self, unit):
        pass

    def post_forward(self, unit):
        pass

    def pre_backward(self, unit):
        pass

    def post_backward(self, unit):
        if not self.sync or (self.world == 1 and not self.force):
            return
        for (a, b) in self.fire_at.get(unit, ()):
            if unit == "head" and self.head_parts:
                # the grad region holds only the embedding scatter-add (+ the norm weights)
                ea, eb = self.embed_range
                self._launch_rows(ea, eb, self.hidden)
                if b > eb:
                    self._launch(eb, b)
            else:
                self._launch(a, b)

    def head_wgrad_ready(self, buf: torch.Tensor, stream=None) -> bool:
        """The engine's lm_head weight gradient of this step's window ([Vp, H] fp32, a
        buffer of its own, ``stream`` = where it was computed): all-reduce it now and add it
        in :meth:`finish`.  Returns False (the engine adds it itself) when nothing is
        reduced this micro-step or the split is off (``DLT_DDP_SPLIT_HEAD=0``)."""
        if not (self.split_head and self.sync and (self.world > 1 or self.force)):
            return False
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        with ctx:
            self.launched += 1
            if self.reduce_dtype != buf.dtype:
                t = buf.to(self.reduce_dtype)
                h = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            else:
                t = None
                h = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        self.head_parts.append((h, buf, t))
        return True

    def _launch_rows(self, a: int, b: int, H: int) -> None:
        """All-reduce the rows of grad[a:b] (a [rows, H] matrix) that are non-zero on any
        rank; rows zero on every rank stay zero (their sum).  One byte per row is MAX-
        reduced first so every rank gathers the same rows (a host sync on the row count)."""
        if self.sparse_rows_max <= 0:  # dense (default): no union, no host sync
            self.last_head = "dense"
            self._launch(a, b)
            return
        g = self.store.grad[a:b].view(-1, H)
        touched = (g != 0).any(dim=1).to(torch.uint8)
        dist.all_reduce(touched, op=dist.ReduceOp.MAX, group=self.pg)
        idx = touched.nonzero().squeeze(1)
        if idx.numel() > self.sparse_rows_max * g.shape[0]:
            self.last_head = "dense"
            self._launch(a, b)
            return
        self.last_head = ("rows", int(idx.numel()), int(g.shape[0]))
        self.launched += 1
        rows = g.index_select(0, idx)
        if self.reduce_dtype != rows.dtype:
            rows = rows.to(self.reduce_dtype)
        h = dist.all_reduce(rows, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        self.row_handles.append((h, rows, idx, a, b, H))

    def _launch(self, a: int, b: int) -> None:
        self.launched += 1
        g = self.store.grad[a:b]
        if self.reduce_dtype != g.dtype:
            t = g.to(self.reduce_dtype)
            h = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            self.handles.append((h, t, a, b))
        else:
            h = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            self.handles.append((h, None, a, b))

    def reduce_all_now(self) -> None:
        """Synchronous fallback used by the eager (non-engine) path."""
        if self.world == 1 and not self.force:
            return
        for (a, b) in self.buckets:
            self._launch(a, b)
        self.finish()

    def finish(self) -> None:
        """Wait for every outstanding bucket (makes the current stream wait on RCCL), then
        add the reduced lm_head part of the tied gradient."""
        for (h, t, a, b) in self.handles:
            h.wait()
            if t is not None:
                if t.is_cuda:  # may have been allocated on the weight-gradient stream
                    t.record_stream(torch.cuda.current_stream(t.device))
                self.store.grad[a:b].copy_(t)
        self.handles.clear()
        for (h, rows, idx, a, b, H) in self.row_handles:
            h.wait()
            g = self.store.grad[a:b].view(-1, H)
            g.index_copy_(0, idx, rows.to(g.dtype))
        self.row_handles.clear()
        if self.head_parts:
            ea, eb = self.embed_range
            emb = self.store.grad[ea:eb].view_as(self.head_parts[0][1])
            for (h, buf, t) in self.head_parts:
                h.wait()
                if t is not None:
                    if t.is_cuda:
                        t.record_stream(torch.cuda.current_stream(t.device))
                    buf.copy_(t)
                # the engine's order without collectives: embedding scatter-add, then + lm_head part
                emb.add_(buf)
            self.head_parts.clear()

    @property
    def collectives(self) -> bool:
        """Whether bucket all-reduces are actually issued (world > 1, or forced on one rank)."""
        return self.world > 1 or self.force

    @property
    def grad_div(self) -> float:
        return float(self.world)
