"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the CPU reference.

The reference relies on PyTorch's stateful Philox generator (``nn.Dropout``,
``gpt.py:168-169,234,240,253,282``) and on ``torch.utils.checkpoint`` saving and
restoring that state so recompute replays the same masks.  The
MI355X engine instead derives every mask from a pure function of
``(seed, site-key, element index)``:

* no RNG state has to be saved/restored for activation checkpointing -- a recompute
  regenerates identical masks by construction;
* forward and backward kernels regenerate masks instead of storing them
  (the attention mask alone would be B*nh*S*S bytes per layer);
* the CPU reference below reproduces the exact same bits, so GPU kernels can be
  checked against it with dropout ON.

Hash: Chris Wellons' ``lowbias32`` integer finaliser; one hash feeds TWO elements
(16 random bits each), which halves the integer-multiply work inside the attention
kernels.  Element ``i`` of a dropout site with key ``k`` uses
``h = lowbias32(k ^ (i >> 1))`` and is kept iff ``((h >> 16*(i & 1)) & 0xFFFF) >= thr``
with ``thr = round(p * 65536)`` (p is realised to within 1e-5); kept values are
scaled by ``1/(1-p)``.
"""
from __future__ import annotations

import torch

MASK32 = 0xFFFFFFFF

# Dropout "sites" inside one transformer layer; combined with the layer index and a
# per-micro-step counter into a 32-bit key on the host.
SITE_ATTN = 1
SITE_RESID = 2
SITE_MLP = 3


def lowbias32(x: int) -> int:
    x &= MASK32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & MASK32
    x ^= x >> 15
    x = (x * 0x846CA68B) & MASK32
    x ^= x >> 16
    return x


def site_key(seed: int, step: int, layer: int, site: int) -> int:
    """32-bit key for one dropout site of one layer in one micro-step."""
    k = lowbias32(seed ^ 0x9E3779B9)
    k = lowbias32(k ^ (step * 0x85EBCA6B & MASK32))
    k = lowbias32(k ^ ((layer * 16 + site) * 0xC2B2AE35 & MASK32))
    return k


def keep_threshold(p: float) -> int:
    """16-bit threshold: keep iff 16 random bits >= threshold.  p=0 -> 0 (always keep)."""
    if p <= 0.0:
        return 0
    return min(int(round(p * 65536.0)), 65536)


def lowbias32_t(x: torch.Tensor) -> torch.Tensor:
    """Vectorised lowbias32 on int64 tensors holding uint32 values (low 32 bits exact)."""
    x = x & MASK32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & MASK32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & MASK32
    x = x ^ (x >> 16)
    return x


def keep_mask(numel_shape, key: int, p: float, device=None, index: torch.Tensor = None) -> torch.Tensor:
    """Boolean keep-mask for a contiguous tensor of ``numel_shape`` (flat element index)."""
    if index is None:
        n = 1
        for s in numel_shape:
            n *= int(s)
        index = torch.arange(n, device=device, dtype=torch.int64).view(*numel_shape)
    h = lowbias32_t((index >> 1) ^ (key & MASK32))
    bits = (h >> ((index & 1) * 16)) & 0xFFFF
    return bits >= keep_threshold(p)


def attn_keep_mask(bh: int, seq_q: int, seq_k: int, key: int, p: float, device=None) -> torch.Tensor:
    """Keep-mask [bh, Sq, Sk] for attention probabilities.

    Per (batch*head) the key is re-mixed: ``kbh = lowbias32(key + bh*0x9E3779B9)``,
    element (i, j) uses index ``i*Sk + j``.
    """
    bidx = torch.arange(bh, device=device, dtype=torch.int64)
    kbh = lowbias32_t(key + bidx * 0x9E3779B9).view(bh, 1, 1)
    ij = torch.arange(seq_q * seq_k, device=device, dtype=torch.int64).view(1, seq_q, seq_k)
    h = lowbias32_t((ij >> 1) ^ kbh)
    bits = (h >> ((ij & 1) * 16)) & 0xFFFF
    return bits >= keep_threshold(p)
