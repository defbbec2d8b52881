"""KV-cached autoregressive decoding for ``GPT.generate`` on the engine path.

The reference's ``generate`` (``gpt.py:457-484``) re-runs the full forward over the
whole context for every new token (O(T^2) work).  Here the prompt is
prefilled once, per-layer K/V (already RoPE-rotated) are cached in preallocated
``[B, nh, max_seq_len, hd]`` buffers, and each new token costs one token's worth of
GEMV + attention.  Sampling semantics are the reference's: temperature, top-k
filtering (``logits < kth`` -> -inf), softmax, ``torch.multinomial``; contexts longer
than ``max_seq_len`` are cropped to the last ``max_seq_len`` tokens (the cache is then
re-prefilled on the cropped window so RoPE positions match the reference exactly).

Weights are read from the engine's provider (bf16 shadows on GPU / FSDP gathered
units), so generation works the same for single-GPU, DDP and FSDP-trained models.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F


class KVCache:
    def __init__(self, cfg, B: int, device, dtype):
        self.k = [torch.zeros(B, cfg.num_heads, cfg.max_seq_len, cfg.head_dim, device=device, dtype=dtype)
                  for _ in range(cfg.num_layers)]
        self.v = [torch.zeros_like(t) for t in self.k]
        self.len = 0


def _rms(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    # x [B, T, nh, hd] fp32; cos/sin [T, hd/2]
    half = x.shape[-1] // 2
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


@torch.no_grad()
def forward_cached(model, ids: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Append ``ids`` [B, T] at positions cache.len.. ; returns last-position logits [B, V]."""
    eng = model.engine
    cfg = model.config
    prov = eng.provider
    dt = eng.act_dtype
    B, T = ids.shape
    p0 = cache.len
    nh, hd = cfg.num_heads, cfg.head_dim
    cos_t, sin_t = eng.rope(max(cfg.max_seq_len, p0 + T), ids.device)
    cos, sin = cos_t[p0:p0 + T].float(), sin_t[p0:p0 + T].float()
    prov.pre_forward("head")
    hw = prov.head()
    h = hw.embed.index_select(0, ids.reshape(-1)).float().view(B, T, -1)
    scale = 1.0 / math.sqrt(hd)
    for i in range(cfg.num_layers):
        prov.pre_forward(i)
        w = prov.layer(i)
        n1 = _rms(h, w.ln1, eng.eps).to(dt)
        qkv = torch.matmul(n1, w.wqkv.t()).float().view(B, T, 3, nh, hd)
        q = _rope(qkv[:, :, 0], cos, sin)
        k = _rope(qkv[:, :, 1], cos, sin)
        v = qkv[:, :, 2]
        cache.k[i][:, :, p0:p0 + T] = k.transpose(1, 2).to(dt)
        cache.v[i][:, :, p0:p0 + T] = v.transpose(1, 2).to(dt)
        K = cache.k[i][:, :, :p0 + T].float()
        Vv = cache.v[i][:, :, :p0 + T].float()
        qh = q.to(dt).float().transpose(1, 2)  # [B, nh, T, hd]
        s = torch.matmul(qh, K.transpose(-2, -1)) * scale
        if T > 1:
            qpos = torch.arange(p0, p0 + T, device=ids.device)[:, None]
            kpos = torch.arange(0, p0 + T, device=ids.device)[None, :]
            s = s.masked_fill(kpos > qpos, float("-inf"))
        pr = torch.softmax(s, dim=-1)
        o = torch.matmul(pr, Vv).transpose(1, 2).reshape(B, T, nh * hd).to(dt)
        h = h + torch.matmul(o, w.wo.t()).float()
        n2 = _rms(h, w.ln2, eng.eps).to(dt)
        gu = torch.matmul(n2, w.wgu.t()).float()
        I = cfg.intermediate_size
        a = (F.silu(gu[..., :I]) * gu[..., I:]).to(dt)
        h = h + torch.matmul(a, w.wdown.t()).float()
        prov.post_forward(i)
    hw = prov.head()
    nf = _rms(h[:, -1], hw.norm, eng.eps).to(dt)
    logits = torch.matmul(nf, hw.lm_head.t())[:, :cfg.vocab_size].float()
    prov.post_forward("head")
    cache.len = p0 + T
    return logits


class DecodeGraph:
    """The one-token decode step captured once as a HIP graph and replayed per token.

    Decode is launch-bound (~200 small kernels per token for GPT-2 small); a graph
    replay issues them with one call.  Everything inside has a fixed shape: the token
    ids and the position are device tensors, the new K/V row is written with
    ``index_copy_`` at the position, and attention runs over the whole preallocated
    cache with a ``key_pos > pos`` mask (a few extra MB per layer per token, far cheaper
    than the launches it saves).  Used by ``kv_cached_generate`` on a GPU with a
    single-process parameter store (FSDP gathers are collectives: not captured).
    """

    def __init__(self, model, cache: KVCache, pos: int, sample: Optional[dict] = None):
        """``sample`` (fused step only): dict(temperature, top_k, seed, hist, hist_base) --
        the graph then also draws the next token (ops ``dec_sample``) into ``self.ids`` and
        ``hist`` and advances the device position, so generation is one replay per token
        with no host round trip."""
        self.model, self.cache = model, cache
        cfg = model.config
        dev = cache.k[0].device
        B = cache.k[0].shape[0]
        self.ids = torch.zeros(B, 1, dtype=torch.long, device=dev)
        self.pos = torch.full((1,), pos, dtype=torch.long, device=dev)
        self.kpos = torch.arange(cfg.max_seq_len, device=dev)
        # fused HIP step (ops/csrc/decode.hip): 5 kernels per layer instead of ~25 ATen ops
        self.fused = _fused_ok(model, B)
        if self.fused:
            H, I = cfg.hidden_size, cfg.intermediate_size
            self.h = torch.empty(B, H, dtype=torch.float32, device=dev)
            self.qb = torch.empty(B, H, dtype=torch.bfloat16, device=dev)
            self.ob = torch.empty(B, H, dtype=torch.bfloat16, device=dev)
            self.sb = torch.empty(B, I, dtype=torch.bfloat16, device=dev)
            self.lg = torch.empty(B, cfg.vocab_size, dtype=torch.float32, device=dev)
        self.sample = sample if self.fused else None
        if self.sample is not None:
            self.sample_ws = model.engine.ops.dec_sample_workspace(B, dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm up allocations / library plans outside the capture
            for _ in range(2):
                # the sampling step advances the device position: restart every warm-up
                # step at ``pos`` so none writes K/V at pos + 1 (== max_seq_len when the
                # prompt fills all but one slot)
                self.pos.fill_(pos)
                self._step()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = self._step()
        self.pos.fill_(pos)  # the warm-up steps advanced it (sampling graph)

    def _step_fused(self) -> torch.Tensor:
        model, cache = self.model, self.cache
        eng, cfg = model.engine, model.config
        ops, prov = eng.ops, eng.provider
        cos_t, sin_t = eng.rope(cfg.max_seq_len, self.ids.device)
        hw = prov.head()
        self.h.copy_(hw.embed.index_select(0, self.ids.view(-1)))
        scale = 1.0 / math.sqrt(cfg.head_dim)
        for i in range(cfg.num_layers):
            w = prov.layer(i)
            ops.dec_norm_qkv(self.h, w.ln1, eng.eps, w.wqkv, cos_t, sin_t, self.pos, self.qb, cache.k[i], cache.v[i],
                             cfg.num_heads)
            ops.dec_attn(self.qb, cache.k[i], cache.v[i], self.pos, self.ob, scale)
            ops.dec_gemv_res(self.ob, w.wo, self.h)
            ops.dec_norm_gu(self.h, w.ln2, eng.eps, w.wgu, self.sb)
            ops.dec_gemv_res(self.sb, w.wdown, self.h)
        ops.dec_norm_head(self.h, hw.norm, eng.eps, hw.lm_head, self.lg, cfg.vocab_size)
        if self.sample is not None:
            sm = self.sample
            ops.dec_sample(self.lg, sm["temperature"], sm["top_k"], sm["seed"], self.pos, self.ids, sm["hist"],
                           sm["hist_base"], ws=self.sample_ws)
            ops.dec_advance(self.pos)
        return self.lg

    def _step(self) -> torch.Tensor:
        if self.fused:
            return self._step_fused()
        model, cache = self.model, self.cache
        eng, cfg = model.engine, model.config
        prov, dt = eng.provider, eng.act_dtype
        B = self.ids.shape[0]
        nh, hd = cfg.num_heads, cfg.head_dim
        cos_t, sin_t = eng.rope(cfg.max_seq_len, self.ids.device)
        cos = cos_t.index_select(0, self.pos).float()
        sin = sin_t.index_select(0, self.pos).float()
        hw = prov.head()
        h = hw.embed.index_select(0, self.ids.view(-1)).float().view(B, 1, -1)
        scale = 1.0 / math.sqrt(hd)
        masked = (self.kpos > self.pos)[None, None, None, :]
        for i in range(cfg.num_layers):
            w = prov.layer(i)
            n1 = _rms(h, w.ln1, eng.eps).to(dt)
            qkv = torch.matmul(n1, w.wqkv.t()).float().view(B, 1, 3, nh, hd)
            q = _rope(qkv[:, :, 0], cos, sin)
            k = _rope(qkv[:, :, 1], cos, sin)
            cache.k[i].index_copy_(2, self.pos, k.transpose(1, 2).to(dt))
            cache.v[i].index_copy_(2, self.pos, qkv[:, :, 2].transpose(1, 2).to(dt))
            qh = q.to(dt).transpose(1, 2)  # [B, nh, 1, hd]; bf16 GEMVs straight on the bf16 cache
            s_ = torch.matmul(qh, cache.k[i].transpose(-2, -1)).float() * scale
            pr = torch.softmax(s_.masked_fill(masked, float("-inf")), dim=-1)
            o = torch.matmul(pr.to(dt), cache.v[i]).transpose(1, 2).reshape(B, 1, nh * hd)
            h = h + torch.matmul(o, w.wo.t()).float()
            n2 = _rms(h, w.ln2, eng.eps).to(dt)
            gu = torch.matmul(n2, w.wgu.t()).float()
            I = cfg.intermediate_size
            h = h + torch.matmul((F.silu(gu[..., :I]) * gu[..., I:]).to(dt), w.wdown.t()).float()
        nf = _rms(h[:, -1], hw.norm, eng.eps).to(dt)
        return torch.matmul(nf, hw.lm_head.t())[:, :cfg.vocab_size].float()

    def __call__(self, ids: torch.Tensor) -> torch.Tensor:
        """Append ``ids`` [B, 1] at position cache.len; returns logits [B, V] (graph-owned:
        consume before the next call)."""
        self.ids.copy_(ids)
        self.pos.fill_(self.cache.len)
        self.graph.replay()
        self.cache.len += 1
        return self.logits


DEC_LDS_MAX = 160 * 1024  # bytes of LDS per workgroup on gfx950


def _fused_ok(model, B: int) -> bool:
    """The fused HIP decode step applies: HIP ops, a supported batch, head_dim 64, and
    the LDS its kernels need fits one CU: ``k_dec_attn`` keeps all ``max_seq_len``
    scores of a (batch, head) in LDS (maxS * 4 + 1056 B: max_seq_len <= ~40.7k), the
    norm + GEMV kernels one normed bf16 row per batch entry (``dec_lds`` in decode.hip).
    Beyond that ``DecodeGraph`` captures the ATen step instead."""
    ops = model.engine.ops
    cfg = model.config
    attn_lds = cfg.max_seq_len * 4 + 8 * 4 + 4 * 64 * 4
    norm_lds = B * cfg.hidden_size * 2 + B * 4 * 4 + B * 16 * 4
    return (hasattr(ops, "dec_norm_qkv") and B in getattr(ops, "DECODE_BATCHES", ())
            and cfg.head_dim == 64 and attn_lds <= DEC_LDS_MAX and norm_lds <= DEC_LDS_MAX
            and os.environ.get("DLT_DECODE_FUSED", "1") != "0")


def _graph_ok(model, device) -> bool:
    import os
    from ..parallel.flat import FlatParamStore
    return (device.type == "cuda" and os.environ.get("DLT_DECODE_GRAPH", "1") != "0"
            and isinstance(model.engine.provider, FlatParamStore))


def _reset(cache: KVCache) -> KVCache:
    cache.len = 0
    return cache


@torch.no_grad()
def kv_cached_generate(model, input_ids: torch.Tensor, max_new_tokens: int = 100, temperature: float = 1.0,
                       top_k: int = 50) -> torch.Tensor:
    cfg = model.config
    eng = model.engine
    B = input_ids.shape[0]
    cache = KVCache(cfg, B, input_ids.device, eng.act_dtype)
    ctx = input_ids[:, -cfg.max_seq_len:]
    logits = forward_cached(model, ctx, cache)
    out = input_ids
    n_dev = min(max_new_tokens - 1, cfg.max_seq_len - cache.len)
    if (n_dev > 0 and temperature > 0 and _graph_ok(model, input_ids.device) and _fused_ok(model, B)
            and os.environ.get("DLT_DECODE_DEVICE_LOOP", "1") != "0"):
        # first token from the prefill logits (ATen sampling), then one graph replay per
        # token: the fused step samples on the device and feeds itself (no host round trip)
        lg = logits / temperature
        if top_k > 0:
            v, _ = torch.topk(lg, min(top_k, lg.size(-1)))
            lg = lg.masked_fill(lg < v[:, [-1]], float("-inf"))
        nxt = torch.multinomial(F.softmax(lg, dim=-1), num_samples=1)
        hist = torch.empty(B, n_dev, dtype=torch.long, device=input_ids.device)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())  # torch's generator: manual_seed reproducible
        graph = DecodeGraph(model, cache, cache.len,
                            sample=dict(temperature=float(temperature), top_k=int(top_k), seed=seed, hist=hist,
                                        hist_base=cache.len + 1))
        graph.ids.copy_(nxt)
        for _ in range(n_dev):
            graph.graph.replay()
        cache.len += n_dev
        out = torch.cat([out, nxt, hist], dim=1)
        if n_dev == max_new_tokens - 1:
            return out
        # context window full: continue on the host path (re-prefill cropping)
        logits = forward_cached(model, out[:, -cfg.max_seq_len:], _reset(cache))
        max_new_tokens -= n_dev + 1
    graph = DecodeGraph(model, cache, cache.len) if (_graph_ok(model, input_ids.device)
                                                    and cache.len < cfg.max_seq_len and max_new_tokens > 1) else None
    for step in range(max_new_tokens):
        lg = logits / temperature
        if top_k > 0:
            v, _ = torch.topk(lg, min(top_k, lg.size(-1)))
            lg = lg.masked_fill(lg < v[:, [-1]], float("-inf"))
        probs = F.softmax(lg, dim=-1)
        nxt = torch.multinomial(probs, num_samples=1)
        out = torch.cat([out, nxt], dim=1)
        if step == max_new_tokens - 1:
            break
        if cache.len + 1 <= cfg.max_seq_len:
            logits = graph(nxt) if graph is not None else forward_cached(model, nxt, cache)
        else:  # context window full: re-prefill the cropped window (reference cropping semantics)
            cache.len = 0
            logits = forward_cached(model, out[:, -cfg.max_seq_len:], cache)
    return out
