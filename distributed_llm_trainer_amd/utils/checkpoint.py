"""Checkpoint save / load in the reference's ``torch.save`` dict format.

Schema (``ddp_trainer.py:408-417``, ``fsdp_trainer.py:452-463``)::

    {"model": state_dict (147 keys for small, fp32, incl. RoPE buffers),
     "optimizer": torch-AdamW-style state dict,
     "global_step": int, "tokens_seen": int,
     "model_config": GPTConfig, "training_config": TrainingConfig,
     ["fsdp_config": FSDPConfig]}

Fixes vs the reference:
* Q8: the reference's own ``load_checkpoint`` fails on torch >= 2.6 because
  ``weights_only=True`` rejects the pickled config objects.  Here the config classes
  are registered as safe globals -- including aliases under the reference's module
  names (``models.config.GPTConfig``, ``__main__.TrainingConfig``,
  ``training.{ddp,fsdp}_trainer.*``) -- so both our checkpoints and the reference's
  load with ``weights_only=True``: nothing in the file is executed.
* Writes are atomic (tmp file + rename), so a crash mid-save never leaves a
  truncated ``final.pt`` behind for ``--resume_from``.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Dict, Optional

import torch

from ..models.config import GPTConfig

_REGISTERED = False


def _alias(cls, module: str, name: Optional[str] = None):
    alias = type(name or cls.__name__, (cls,), {})
    alias.__module__ = module
    alias.__qualname__ = name or cls.__name__
    return alias


class _PlaceholderConfig:
    """Stand-in for reference config classes we do not model field-for-field."""

    def __setstate__(self, state):
        self.__dict__.update(state)


def register_safe_globals() -> None:
    global _REGISTERED
    if _REGISTERED:
        return
    from ..training.configs import FSDPConfig, FSDPTrainingConfig, TrainingConfig
    safe = [GPTConfig, TrainingConfig, FSDPTrainingConfig, FSDPConfig,
            _alias(GPTConfig, "models.config"), _alias(GPTConfig, "src.models.config"),
            _alias(TrainingConfig, "__main__"), _alias(TrainingConfig, "training.ddp_trainer"),
            _alias(TrainingConfig, "src.training.ddp_trainer"),
            _alias(FSDPTrainingConfig, "training.fsdp_trainer", "TrainingConfig"),
            _alias(FSDPTrainingConfig, "src.training.fsdp_trainer", "TrainingConfig"),
            _alias(FSDPConfig, "__main__"), _alias(FSDPConfig, "training.fsdp_trainer"),
            _alias(FSDPConfig, "src.training.fsdp_trainer")]
    try:
        torch.serialization.add_safe_globals(safe)
    except AttributeError:  # very old torch
        pass
    _REGISTERED = True


def save_checkpoint(path: str, payload: Dict[str, Any]) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(payload, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    register_safe_globals()
    return torch.load(path, map_location=map_location, weights_only=True)


def config_to_dict(cfg) -> Dict[str, Any]:
    if dataclasses.is_dataclass(cfg):
        return dataclasses.asdict(cfg)
    return dict(getattr(cfg, "__dict__", {}))


def model_state_dict_cpu(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """fp32 CPU copies (never views of the flat training buffers)."""
    out = {}
    for k, v in model.state_dict().items():
        out[k] = v.detach().to("cpu", copy=True).clone()
    return out
