"""TinyStories loaders (API parity with ``src/data/tinystories.py:11-161``)."""
from __future__ import annotations

from typing import Optional

from torch.utils.data import DataLoader

from .text import StreamingTextDataset, TextDataConfig, TokenizedTextDataset, create_text_dataloader

TinyStoriesConfig = TextDataConfig


class TinyStoriesDataset(TokenizedTextDataset):
    """Map-style: whole file tokenised once, non-overlapping ``seq_len`` windows."""


class TinyStoriesIterableDataset(StreamingTextDataset):
    """Streaming: line-sharded over rank x worker, LRU tokenisation cache."""


def create_tinystories_dataloader(path: str, batch_size: int, seq_len: int, distributed: bool = False,
                                  rank: int = 0, world_size: int = 1, tokenizer_name: str = "gpt2",
                                  max_tokens: Optional[int] = None, streaming: bool = False,
                                  cache_max_tokens: Optional[int] = None, num_workers: int = 2,
                                  tokenizer=None, **kw):
    return create_text_dataloader(path, batch_size, seq_len, distributed, rank, world_size, tokenizer_name,
                                  max_tokens, streaming, cache_max_tokens, num_workers, tokenizer, **kw)
