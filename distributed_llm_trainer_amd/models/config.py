"""Model hyper-parameters (``GPTConfig``) and the GPT-2-named presets.

Parity target: ``src/models/config.py:6-102`` of the reference.  Same field names,
defaults and the four ``gpt2_*`` presets, so YAML / pickled configs from the
reference map 1:1 onto this class.

Intentional divergences (documented in SURVEY.md §7.1 / Appendix A):

* ``num_parameters()`` returns the *true* parameter count of the LLaMA-style block
  (RMSNorm + SwiGLU + RoPE + tied head).  The reference formula
  (``config.py:81-102``) assumes a classic GPT-2 layout and under-reports; it is kept
  as ``num_parameters_legacy()`` for comparison (Q4).
* ``activation`` is kept for schema compatibility; as in the reference it is not read
  by the model (the MLP is SwiGLU, ``gpt.py:245-283``).
* ``vocab_size_padded`` is the lm_head GEMM width used internally by the fused MI355X
  path (multiple of 64 so the bf16 weight rows stay 128-B aligned for MFMA tiles);
  the state dict still carries exactly ``vocab_size`` rows.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, fields
from typing import Any, Dict, Optional


@dataclass
class GPTConfig:
    """Configuration for the GPT model.  Defaults are the "GPT-2 124M" preset."""

    # Model architecture
    vocab_size: int = 50257
    hidden_size: int = 768
    num_layers: int = 12
    num_heads: int = 12
    intermediate_size: Optional[int] = None  # defaults to 4 * hidden_size
    max_seq_len: int = 1024

    # Regularization
    dropout: float = 0.1
    attention_dropout: float = 0.1

    # Initialization
    initializer_range: float = 0.02

    # Activation (schema-compat only; the block is SwiGLU like the reference)
    activation: str = "gelu"

    # Optimization flags
    use_flash_attention: bool = False
    gradient_checkpointing: bool = False

    def __post_init__(self) -> None:
        if self.intermediate_size is None:
            self.intermediate_size = 4 * self.hidden_size
        assert self.hidden_size % self.num_heads == 0, (
            f"hidden_size ({self.hidden_size}) must be divisible by num_heads ({self.num_heads})"
        )

    # ------------------------------------------------------------------ presets
    @classmethod
    def gpt2_small(cls) -> "GPTConfig":
        """"GPT-2 124M" preset (151,862,784 real parameters)."""
        return cls(vocab_size=50257, hidden_size=768, num_layers=12, num_heads=12)

    @classmethod
    def gpt2_medium(cls) -> "GPTConfig":
        """"GPT-2 355M" preset (454,166,528 real parameters)."""
        return cls(vocab_size=50257, hidden_size=1024, num_layers=24, num_heads=16)

    @classmethod
    def gpt2_large(cls) -> "GPTConfig":
        """"GPT-2 774M" preset (1,008,140,800 real parameters)."""
        return cls(vocab_size=50257, hidden_size=1280, num_layers=36, num_heads=20)

    @classmethod
    def gpt2_xl(cls) -> "GPTConfig":
        """"GPT-2 1.5B" preset (2,046,646,400 real parameters, 25 heads)."""
        return cls(vocab_size=50257, hidden_size=1600, num_layers=48, num_heads=25)

    @classmethod
    def from_preset(cls, name: str) -> "GPTConfig":
        name = name.lower().replace("gpt2-", "").replace("gpt2_", "")
        table = {"small": cls.gpt2_small, "medium": cls.gpt2_medium,
                 "large": cls.gpt2_large, "xl": cls.gpt2_xl}
        if name not in table:
            raise ValueError(f"unknown model preset {name!r}; choose from {sorted(table)}")
        return table[name]()

    # ------------------------------------------------------------- derived
    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def vocab_size_padded(self) -> int:
        return ((self.vocab_size + 63) // 64) * 64

    def num_parameters(self) -> int:
        """True trainable parameter count (tied embedding counted once)."""
        h, i = self.hidden_size, self.intermediate_size
        per_layer = 4 * h * h + 3 * h * i + 2 * h
        return self.vocab_size * h + self.num_layers * per_layer + h

    def num_parameters_legacy(self) -> int:
        """The reference's classic-GPT-2 estimate (``config.py:81-102``), kept for parity."""
        embed = self.vocab_size * self.hidden_size
        pos = self.max_seq_len * self.hidden_size
        layer = 4 * self.hidden_size ** 2 + 2 * self.hidden_size * self.intermediate_size + 4 * self.hidden_size
        return embed + pos + self.num_layers * layer + 2 * self.hidden_size

    def flops_per_token(self, seq_len: Optional[int] = None, causal: bool = True,
                        recompute: bool = False) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd; +1 fwd with recompute).

        Attention score/value FLOPs are counted for the causal half when ``causal``.
        """
        s = seq_len or self.max_seq_len
        h, i, L, v = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        dense = 2 * (4 * h * h + 3 * h * i) * L + 2 * h * v
        attn = 2 * 2 * s * h * L * (0.5 if causal else 1.0)
        fwd = dense + attn
        return fwd * (4.0 if recompute else 3.0)

    # ------------------------------------------------------------- (de)serialise
    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "GPTConfig":
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})
