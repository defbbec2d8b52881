"""Synthetic-token loader (the reference's ``create_dummy_dataloader``,
``ddp_trainer.py:460-487`` / ``fsdp_trainer.py:508-527``).

Differences: seeded per rank (reproducible; Q13), ``drop_last=True`` (Q18: a ragged
last batch silently shrank the micro-batch), and ``num_samples`` can be kept small
-- the reference materialises 1000 x batch random sequences (262 MB int64 for the
default small config) per rank.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, DistributedSampler, TensorDataset


def create_dummy_dataloader(batch_size: int, seq_len: int, vocab_size: int, distributed: bool = False,
                            rank: int = 0, world_size: int = 1, num_batches: int = 1000, seed: int = 0,
                            num_workers: int = 0) -> DataLoader:
    g = torch.Generator().manual_seed(seed + 7919 * rank)
    n = num_batches * batch_size * (world_size if distributed else 1)
    data = torch.randint(0, vocab_size, (n, seq_len), generator=g)
    ds = TensorDataset(data)
    sampler = DistributedSampler(ds, num_replicas=world_size, rank=rank, shuffle=True, seed=seed) \
        if distributed else None
    return DataLoader(ds, batch_size=batch_size, sampler=sampler, shuffle=sampler is None, drop_last=True,
                      pin_memory=torch.cuda.is_available(), num_workers=num_workers)
