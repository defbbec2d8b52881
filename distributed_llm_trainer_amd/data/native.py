"""Pre-tokenised token files (``.bin``: flat little-endian uint16/uint32 token ids).

Map-style dataset of non-overlapping ``seq_len`` windows over a memory-mapped token
file, so multi-GB corpora are never loaded or re-tokenised per run (the reference
tokenises the whole text file in every process, ``tinystories.py:30-33``).  When the
native runtime library (``runtime/_dlt_runtime.so``) is built, window batches are
gathered by its multi-threaded C++ reader into pinned memory; otherwise numpy memmap
slicing is used (same bytes, same order).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset


def write_token_file(path: str, ids, dtype=np.uint16) -> None:
    arr = np.asarray(ids, dtype=dtype)
    arr.tofile(path)


class TokenFileDataset(Dataset):
    def __init__(self, path: str, seq_len: int, max_tokens: Optional[int] = None, dtype=None):
        self.path = path
        self.seq_len = seq_len
        if dtype is None:
            dtype = np.uint32 if os.environ.get("DLT_TOKEN_DTYPE", "uint16") == "uint32" else np.uint16
        self.tokens = np.memmap(path, dtype=dtype, mode="r")
        n = len(self.tokens)
        if max_tokens is not None:
            n = min(n, max_tokens)
        if n < seq_len:
            raise ValueError(f"Not enough tokens ({n}) for seq_len={seq_len} in {path}")
        self.n = n

    def __len__(self) -> int:
        return (self.n - 1) // self.seq_len

    def __getitem__(self, idx: int):
        s = idx * self.seq_len
        return (torch.from_numpy(np.asarray(self.tokens[s:s + self.seq_len], dtype=np.int64)),)
