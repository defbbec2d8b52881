"""Shared text-dataset machinery behind the TinyStories / OpenWebText loaders.

Parity target: ``src/data/tinystories.py:11-161`` and ``src/data/openwebtext.py:13-181``
(map-style: whole file tokenised once, non-overlapping ``seq_len`` windows returned as
1-tuples; streaming: line-sharded over ``rank x worker``, token buffer cut into
``seq_len`` chunks, ``max_tokens`` cap, LRU tokenisation cache, transparent ``.gz``).

Fixes: the streaming token cache is consulted BEFORE encoding
(Q9 -- the reference encodes first, so its cache never saves work), and the
map-style dataset can be backed by a pre-tokenised ``.bin`` token file read through
the native memory-mapped loader (``data/native.py``) instead of re-tokenising.
"""
from __future__ import annotations

import gzip
import io
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Iterator, List, Optional

import torch
from torch.utils.data import DataLoader, Dataset, DistributedSampler, IterableDataset, get_worker_info

from .tokenizer import get_tokenizer


@dataclass
class TextDataConfig:
    path: str
    seq_len: int
    tokenizer_name: str = "gpt2"
    max_tokens: Optional[int] = None
    streaming: bool = False
    cache_max_tokens: Optional[int] = None


def open_text(path: str):
    if path.endswith(".gz"):
        return io.TextIOWrapper(gzip.open(path, "rb"), encoding="utf-8")
    return open(path, "r", encoding="utf-8")


class TokenizedTextDataset(Dataset):
    """Whole file -> token ids -> fixed, non-overlapping windows of ``seq_len``."""

    def __init__(self, cfg: TextDataConfig, tokenizer=None):
        self.cfg = cfg
        self.tokenizer = tokenizer or get_tokenizer(cfg.tokenizer_name)
        with open_text(cfg.path) as f:
            text = f.read()
        ids = self.tokenizer.encode(text)
        if cfg.max_tokens is not None:
            ids = ids[: cfg.max_tokens]
        if len(ids) < cfg.seq_len:
            raise ValueError(f"Not enough tokens ({len(ids)}) for seq_len={cfg.seq_len} in {cfg.path}")
        self.tokens = torch.tensor(ids, dtype=torch.long)

    def __len__(self) -> int:
        return (len(self.tokens) - 1) // self.cfg.seq_len

    def __getitem__(self, idx: int):
        s = idx * self.cfg.seq_len
        return (self.tokens[s:s + self.cfg.seq_len],)


class _LRU:
    def __init__(self, max_tokens: Optional[int]):
        self.max_tokens = max_tokens
        self.d: "OrderedDict[str, List[int]]" = OrderedDict()
        self.size = 0
        self.hits = 0
        self.misses = 0

    def get(self, key: str):
        v = self.d.get(key)
        if v is not None:
            self.d.move_to_end(key)
            self.hits += 1
        else:
            self.misses += 1
        return v

    def put(self, key: str, ids: List[int]) -> None:
        if not self.max_tokens or len(ids) > self.max_tokens:
            return
        self.d[key] = ids
        self.size += len(ids)
        while self.size > self.max_tokens and self.d:
            _, old = self.d.popitem(last=False)
            self.size -= len(old)


class StreamingTextDataset(IterableDataset):
    """Line-sharded streaming tokenisation (shard = rank*workers + worker_id)."""

    def __init__(self, cfg: TextDataConfig, rank: int = 0, world_size: int = 1, tokenizer=None):
        self.cfg = cfg
        self.rank = rank
        self.world_size = world_size
        self.tokenizer = tokenizer or get_tokenizer(cfg.tokenizer_name)
        self.cache = _LRU(cfg.cache_max_tokens)

    def _encode(self, line: str) -> List[int]:
        ids = self.cache.get(line)
        if ids is None:
            ids = self.tokenizer.encode(line)
            self.cache.put(line, ids)
        return ids

    def __iter__(self) -> Iterator[torch.Tensor]:
        info = get_worker_info()
        nw, wid = (info.num_workers, info.id) if info is not None else (1, 0)
        shards = self.world_size * nw
        shard = self.rank * nw + wid
        buf: List[int] = []
        produced = 0
        S = self.cfg.seq_len
        with open_text(self.cfg.path) as f:
            for li, line in enumerate(f):
                if li % shards != shard:
                    continue
                line = line.strip()
                if not line:
                    continue
                buf.extend(self._encode(line))
                while len(buf) >= S:
                    if self.cfg.max_tokens is not None and produced + S > self.cfg.max_tokens:
                        return
                    yield torch.tensor(buf[:S], dtype=torch.long)
                    produced += S
                    buf = buf[S:]


def create_text_dataloader(path: str, batch_size: int, seq_len: int, distributed: bool = False, rank: int = 0,
                           world_size: int = 1, tokenizer_name: str = "gpt2", max_tokens: Optional[int] = None,
                           streaming: bool = False, cache_max_tokens: Optional[int] = None,
                           num_workers: int = 2, tokenizer=None, seed: int = 0, device=None):
    if path.endswith(".bin") and os.environ.get("DLT_NATIVE_DATA", "1") != "0":
        from ..runtime import loader as nl
        if nl.available():
            tb = 4 if os.environ.get("DLT_TOKEN_DTYPE", "uint16") == "uint32" else 2
            return nl.NativeTokenLoader(path, seq_len, batch_size, token_bytes=tb, max_tokens=max_tokens,
                                        rank=rank if distributed else 0, world_size=world_size if distributed else 1,
                                        seed=seed, device=device)
    cfg = TextDataConfig(path=path, seq_len=seq_len, tokenizer_name=tokenizer_name, max_tokens=max_tokens,
                         streaming=streaming, cache_max_tokens=cache_max_tokens)
    if path.endswith(".bin"):
        from .native import TokenFileDataset
        dataset = TokenFileDataset(path, seq_len, max_tokens=max_tokens)
        sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank) if distributed else None
        shuffle = sampler is None
    elif streaming:
        dataset = StreamingTextDataset(cfg, rank=rank, world_size=world_size, tokenizer=tokenizer)
        sampler, shuffle = None, False
    else:
        dataset = TokenizedTextDataset(cfg, tokenizer=tokenizer)
        sampler = DistributedSampler(dataset, num_replicas=world_size, rank=rank) if distributed else None
        shuffle = sampler is None
    return DataLoader(dataset, batch_size=batch_size, sampler=sampler, shuffle=shuffle, drop_last=True,
                      pin_memory=torch.cuda.is_available(), num_workers=num_workers)
