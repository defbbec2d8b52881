"""OpenWebText loaders (API parity with ``src/data/openwebtext.py:13-181``), incl. ``.gz``
inputs and the reference's path fallback (``:147-155``: toggle the ``.gz`` suffix)."""
from __future__ import annotations

import os
from typing import Optional

from torch.utils.data import DataLoader

from .text import StreamingTextDataset, TextDataConfig, TokenizedTextDataset, create_text_dataloader

OpenWebTextConfig = TextDataConfig


class OpenWebTextDataset(TokenizedTextDataset):
    pass


class OpenWebTextIterableDataset(StreamingTextDataset):
    pass


def resolve_path(path: str) -> str:
    if os.path.exists(path):
        return path
    cand = path[:-3] if path.endswith(".gz") else f"{path}.gz"
    if os.path.exists(cand):
        return cand
    raise FileNotFoundError(f"OpenWebText file not found: {path}")


def create_openwebtext_dataloader(path: str, batch_size: int, seq_len: int, distributed: bool = False,
                                  rank: int = 0, world_size: int = 1, tokenizer_name: str = "gpt2",
                                  max_tokens: Optional[int] = None, streaming: bool = False,
                                  cache_max_tokens: Optional[int] = None, num_workers: int = 2,
                                  tokenizer=None, **kw):
    path = resolve_path(path)
    return create_text_dataloader(path, batch_size, seq_len, distributed, rank, world_size, tokenizer_name,
                                  max_tokens, streaming, cache_max_tokens, num_workers, tokenizer, **kw)
