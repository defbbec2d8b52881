"""ctypes front-end of the native token loader (``runtime/csrc/loader.cpp``).

``NativeTokenLoader`` is an iterator of ``LongTensor[batch, seq_len]`` batches that live
in a ring of pinned host slots filled by C++ producer threads; with ``device`` set it
also issues the H2D copy on a side stream and hands out device tensors, returning a
slot to the producers only once its copy has completed (event-tracked).

Order semantics (``file`` mode) match ``DistributedSampler(shuffle, drop_last=True)``
over the reference's non-overlapping windows (``tinystories.py:44-50``): the window
permutation of epoch ``e`` is a seeded Fisher-Yates shuffle and rank ``r`` takes
positions ``r, r+W, ...``.  ``dummy`` mode draws uniform ids from a counter hash of
(seed, rank, step, position) -- the reference's synthetic data
(``ddp_trainer.py:460-487``) without the 262 MB per-rank tensor.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import build as _build

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_build.LIB):
            _build.build(verbose=False)
        L = ctypes.CDLL(_build.LIB)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.dlt_loader_open.restype = vp
        L.dlt_loader_open.argtypes = [ctypes.c_char_p, i32, i64, i64, i64, i64, i32, i32, ctypes.c_uint64, i32, i32,
                                      i32, ctypes.POINTER(i32)]
        L.dlt_loader_set_slot.argtypes = [vp, i32, vp, i32]
        L.dlt_loader_seek.argtypes = [vp, i64]
        L.dlt_loader_next.argtypes = [vp, ctypes.POINTER(i64)]
        L.dlt_loader_release.argtypes = [vp, i32]
        L.dlt_loader_fill.argtypes = [vp, i64, vp]
        for f in ("dlt_loader_steps_per_epoch", "dlt_loader_num_windows", "dlt_loader_produced"):
            getattr(L, f).restype = i64
            getattr(L, f).argtypes = [vp]
        L.dlt_loader_close.argtypes = [vp]
        _LIB = L
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


_ERR = {1: "cannot open / mmap the token file", 2: "invalid arguments", 3: "too few tokens for one batch per rank"}


class NativeTokenLoader:
    def __init__(self, path: Optional[str], seq_len: int, batch_size: int, *, vocab_size: int = 0,
                 token_bytes: int = 2, max_tokens: Optional[int] = None, rank: int = 0, world_size: int = 1,
                 seed: int = 0, shuffle: bool = True, prefetch: int = 4, threads: int = 2,
                 device: Optional[torch.device] = None, start_step: int = 0):
        L = lib()
        self.seq_len, self.batch_size = seq_len, batch_size
        err = ctypes.c_int(0)
        self._h = L.dlt_loader_open(path.encode() if path is not None else None, token_bytes, max_tokens or 0,
                                    vocab_size, seq_len, batch_size, rank, world_size, seed & (2 ** 64 - 1),
                                    int(shuffle), prefetch, threads, ctypes.byref(err))
        if not self._h:
            raise ValueError(f"native loader: {_ERR.get(err.value, err.value)} ({path})")
        self.device = torch.device(device) if device is not None else None
        pin = torch.cuda.is_available()
        self._slots = [torch.empty((batch_size, seq_len), dtype=torch.int64, pin_memory=pin) for _ in range(prefetch)]
        self._events = [None] * prefetch
        self._stream = torch.cuda.Stream(self.device) if (self.device is not None and self.device.type == "cuda") else None
        if start_step:
            L.dlt_loader_seek(self._h, start_step)
        for i, t in enumerate(self._slots):
            L.dlt_loader_set_slot(self._h, i, t.data_ptr(), threads)
        self._held = []  # slots handed out whose copies may still be running

    # dataset geometry ------------------------------------------------------
    @property
    def steps_per_epoch(self) -> int:
        return int(lib().dlt_loader_steps_per_epoch(self._h))

    @property
    def num_windows(self) -> int:
        return int(lib().dlt_loader_num_windows(self._h))

    def batch_at(self, step: int) -> torch.Tensor:
        """Deterministic random access (no ring): the batch the stream yields at ``step``."""
        out = torch.empty((self.batch_size, self.seq_len), dtype=torch.int64)
        lib().dlt_loader_fill(self._h, step, out.data_ptr())
        return out

    def seek(self, step: int) -> None:
        self._drain()
        lib().dlt_loader_seek(self._h, step)

    # iteration -------------------------------------------------------------
    def _drain(self, keep: int = 0):
        L = lib()
        while len(self._held) > keep:
            slot, ev = self._held.pop(0)
            if ev is not None:
                ev.synchronize()
            L.dlt_loader_release(self._h, slot)

    def __iter__(self):
        return self

    def __next__(self) -> torch.Tensor:
        L = lib()
        self._drain(keep=1)  # the previous batch's copy normally finished long ago
        step = ctypes.c_int64(0)
        slot = L.dlt_loader_next(self._h, ctypes.byref(step))
        host = self._slots[slot]
        if self._stream is None:
            out = host.clone() if self.device is None else host.to(self.device)
            self._held.append((slot, None))
            return out
        with torch.cuda.stream(self._stream):
            out = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        torch.cuda.current_stream(self.device).wait_event(ev)
        out.record_stream(torch.cuda.current_stream(self.device))
        self._held.append((slot, ev))
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._drain()
            lib().dlt_loader_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
