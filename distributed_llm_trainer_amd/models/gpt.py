"""LLaMA-style "GPT-2" model with the reference's module tree and state-dict keys.

Parity target: ``/root/reference/src/models/gpt.py`` -- RMSNorm (``:22-67``), NeoX
RoPE (``:70-147``), causal self-attention with separate bias-free q/k/v/o
(``:150-242``), SwiGLU MLP (``:245-283``), pre-norm block (``:286-316``), tied
``lm_head`` (``:339-342``), N(0, 0.02) init (``:380-385``), shifted CE loss
(``:449-453``), top-k sampling ``generate`` (``:457-484``).

Two execution paths share the same ``nn.Parameter`` objects:

* **eager path** (this file): plain PyTorch modules.  It is the numerics oracle for
  the tests and the CPU "plumbing" path (BASELINE.json configs[0]).
* **engine path** (``enable_engine``): parameters are re-homed into flat fp32
  buffers (``parallel/flat.py``) and forward/backward run through the hand-scheduled
  fused executor (``models/engine.py``) whose hot ops are the HIP/CDNA4 kernels in
  ``ops/csrc``.  On GPU this is the only path the trainers use; the fused loss path
  never materialises the ``[B, S, V]`` logits, so ``forward`` returns
  ``(None, loss)`` when called with labels during training.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from .config import GPTConfig


class RMSNorm(nn.Module):
    def __init__(self, hidden_size: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.eps = eps

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        rms = torch.rsqrt(x.pow(2).mean(dim=-1, keepdim=True) + self.eps)
        return x * rms * self.weight


class RotaryPositionEmbedding(nn.Module):
    """NeoX-style RoPE.  The cos/sin caches are persistent buffers because the
    reference checkpoint format carries them (``rotary_emb.{inv_freq,cos_cached,sin_cached}``)."""

    def __init__(self, dim: int, max_seq_len: int = 2048, base: int = 10000):
        super().__init__()
        self.dim = dim
        self.max_seq_len = max_seq_len
        self.base = base
        inv_freq = 1.0 / (base ** (torch.arange(0, dim, 2).float() / dim))
        self.register_buffer("inv_freq", inv_freq)
        self._build_cache(max_seq_len)

    def _build_cache(self, seq_len: int) -> None:
        t = torch.arange(seq_len, device=self.inv_freq.device).float()
        freqs = torch.outer(t, self.inv_freq)
        emb = torch.cat((freqs, freqs), dim=-1)
        self.register_buffer("cos_cached", emb.cos())
        self.register_buffer("sin_cached", emb.sin())

    def forward(self, x: torch.Tensor, seq_len: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if seq_len > self.cos_cached.shape[0]:
            # (the reference rebuilds on every long call because it never updates
            # max_seq_len; we rebuild once and keep the larger cache)
            self._build_cache(seq_len)
        return self.cos_cached[:seq_len], self.sin_cached[:seq_len]


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    half = x.shape[-1] // 2
    return torch.cat([-x[..., half:], x[..., :half]], dim=-1)


def apply_rotary_pos_emb(q, k, cos, sin):
    return q * cos + rotate_half(q) * sin, k * cos + rotate_half(k) * sin


class CausalSelfAttention(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        self.config = config
        self.num_heads = config.num_heads
        self.head_dim = config.hidden_size // config.num_heads
        h = config.hidden_size
        self.q_proj = nn.Linear(h, h, bias=False)
        self.k_proj = nn.Linear(h, h, bias=False)
        self.v_proj = nn.Linear(h, h, bias=False)
        self.o_proj = nn.Linear(h, h, bias=False)
        self.attn_dropout = nn.Dropout(config.attention_dropout)
        self.resid_dropout = nn.Dropout(config.dropout)
        self.rotary_emb = RotaryPositionEmbedding(self.head_dim, config.max_seq_len)
        self.use_flash = config.use_flash_attention

    def forward(self, hidden_states: torch.Tensor, attention_mask: Optional[torch.Tensor] = None):
        B, S, _ = hidden_states.shape
        q = self.q_proj(hidden_states).view(B, S, self.num_heads, self.head_dim).transpose(1, 2)
        k = self.k_proj(hidden_states).view(B, S, self.num_heads, self.head_dim).transpose(1, 2)
        v = self.v_proj(hidden_states).view(B, S, self.num_heads, self.head_dim).transpose(1, 2)
        cos, sin = self.rotary_emb(q, S)
        q, k = apply_rotary_pos_emb(q, k, cos[None, None], sin[None, None])
        if self.use_flash:
            out = F.scaled_dot_product_attention(
                q, k, v, attn_mask=None,
                dropout_p=self.config.attention_dropout if self.training else 0.0, is_causal=True)
        else:
            scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(self.head_dim)
            mask = torch.triu(torch.ones(S, S, device=hidden_states.device, dtype=torch.bool), diagonal=1)
            scores = scores.masked_fill(mask[None, None], float("-inf"))
            probs = F.softmax(scores, dim=-1, dtype=torch.float32).to(scores.dtype)
            out = self.attn_dropout(probs) @ v
        out = out.transpose(1, 2).contiguous().view(B, S, -1)
        return self.resid_dropout(self.o_proj(out))


class MLP(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        self.gate_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.up_proj = nn.Linear(config.hidden_size, config.intermediate_size, bias=False)
        self.down_proj = nn.Linear(config.intermediate_size, config.hidden_size, bias=False)
        self.dropout = nn.Dropout(config.dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.dropout(self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x)))


class TransformerBlock(nn.Module):
    """Pre-norm block; the FSDP wrap unit and the activation-checkpoint unit."""

    def __init__(self, config: GPTConfig, layer_idx: int):
        super().__init__()
        self.layer_idx = layer_idx
        self.input_layernorm = RMSNorm(config.hidden_size)
        self.attention = CausalSelfAttention(config)
        self.post_attention_layernorm = RMSNorm(config.hidden_size)
        self.mlp = MLP(config)

    def forward(self, hidden_states, attention_mask=None):
        h = hidden_states + self.attention(self.input_layernorm(hidden_states), attention_mask)
        return h + self.mlp(self.post_attention_layernorm(h))


class GPT(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        self.config = config
        self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size)
        self.layers = nn.ModuleList([TransformerBlock(config, i) for i in range(config.num_layers)])
        self.norm = RMSNorm(config.hidden_size)
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size, bias=False)
        self.lm_head.weight = self.embed_tokens.weight  # tied
        self.gradient_checkpointing = config.gradient_checkpointing
        self.apply(self._init_weights)
        self.engine = None
        self.store = None
        self._anchor = None

    def _init_weights(self, module):
        if isinstance(module, nn.Linear):
            torch.nn.init.normal_(module.weight, mean=0.0, std=self.config.initializer_range)
            if module.bias is not None:
                torch.nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            torch.nn.init.normal_(module.weight, mean=0.0, std=self.config.initializer_range)

    # ------------------------------------------------------------ engine path
    def enable_engine(self, provider=None, ops=None, act_dtype=None, seed: int = 1234,
                      compute_dtype=None):
        """Switch to the fused executor.  Builds a FlatParamStore unless a provider
        (e.g. the FSDP runtime) is given.  Returns the engine."""
        from ..models.engine import GPTEngine
        from .. import ops as ops_mod
        dev = next(self.parameters()).device
        if act_dtype is None:
            act_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        if compute_dtype is None:
            compute_dtype = act_dtype
        if provider is None:
            from ..parallel.flat import FlatParamStore
            provider = FlatParamStore(self, dev, compute_dtype=compute_dtype)
            self.store = provider
        if ops is None:
            # bf16 / fp16 run the 16-bit HIP kernels (csrc/common.h HK), fp32 (the
            # reference / debug mode, --mixed_precision fp32) the fp32 ones (csrc/fp32.hip);
            # GEMMs go through the planner (hipBLASLt fp32 GEMMs in fp32 mode)
            ops = ops_mod.for_device(dev, head_dim=self.config.head_dim, act_dtype=act_dtype)
        gemm = None
        if dev.type == "cuda" and ops.backend == "hip":
            import os
            from ..ops import gemm as gemm_mod
            if os.environ.get("DLT_GEMM", "planner") == "planner" and gemm_mod.available():
                gemm = gemm_mod.HipGemm()
        self.engine = GPTEngine(self.config, provider, ops, act_dtype=act_dtype, seed=seed, gemm=gemm)
        self._anchor = torch.zeros((), device=dev, requires_grad=True)
        return self.engine

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None):
        """(logits [B, S, V], loss or None), as the reference (``gpt.py:388-455``).

        Divergence on the engine path: a TRAINING forward with labels (``self.training``
        and grad enabled) returns ``(None, loss)`` -- the fused lm_head + cross-entropy
        turns the logits buffer into dloss/dlogits in place, so full [B, S, V] logits are
        never materialised for the caller.  Eval mode, ``torch.no_grad()`` or a call
        without labels returns the logits as the reference does."""
        if self.engine is not None:
            return self._engine_forward(input_ids, labels)
        h = self.embed_tokens(input_ids)
        for layer in self.layers:
            if self.gradient_checkpointing and self.training:
                h = checkpoint(layer, h, attention_mask, use_reentrant=False)
            else:
                h = layer(h, attention_mask)
        h = self.norm(h)
        logits = self.lm_head(h)
        loss = None
        if labels is not None:
            shift_logits = logits[..., :-1, :].contiguous()
            shift_labels = labels[..., 1:].contiguous()
            loss = F.cross_entropy(shift_logits.view(-1, self.config.vocab_size), shift_labels.view(-1))
        return logits, loss

    def _engine_forward(self, input_ids, labels):
        from .engine import EngineFunction, shift_targets
        eng = self.engine
        if labels is None:
            _, logits, _ = eng.forward(input_ids, None, train=self.training, need_backward=False)
            return logits, None
        targets = shift_targets(labels)
        recompute = bool(self.gradient_checkpointing)
        if self.training and torch.is_grad_enabled():
            loss = EngineFunction.apply(self._anchor, eng, input_ids, targets, recompute)
            return None, loss
        loss, logits, _ = eng.forward(input_ids, targets, train=self.training, need_backward=False,
                                      return_logits=True)
        return logits, loss

    # ------------------------------------------------------------ generation
    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, max_new_tokens: int = 100,
                 temperature: float = 1.0, top_k: int = 50) -> torch.Tensor:
        """Top-k sampling with the reference's semantics (``gpt.py:457-484``).

        With the engine enabled this uses the KV-cached decoder in
        ``eval/decode.py`` (one token per step instead of a full re-forward)."""
        self.eval()
        flush = getattr(getattr(self.engine, "provider", None), "flush_pending", None)
        if flush is not None:  # a recorded (lazy) optimizer step: the decoder reads every unit
            flush()
        if self.engine is not None:
            from ..eval.decode import kv_cached_generate
            return kv_cached_generate(self, input_ids, max_new_tokens, temperature, top_k)
        for _ in range(max_new_tokens):
            idx = input_ids if input_ids.size(1) <= self.config.max_seq_len else input_ids[:, -self.config.max_seq_len:]
            logits, _ = self(idx)
            logits = logits[:, -1, :] / temperature
            if top_k > 0:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = float("-inf")
            probs = F.softmax(logits, dim=-1)
            nxt = torch.multinomial(probs, num_samples=1)
            input_ids = torch.cat([input_ids, nxt], dim=1)
        return input_ids


def count_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
