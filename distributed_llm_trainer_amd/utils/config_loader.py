"""YAML config loading for ``--config configs/*.yaml`` (schema of the reference's
``configs/small_model.yaml`` / ``medium_model.yaml``).

The reference documents ``--config`` but its argparse rejects it and no code parses
the YAML (Q1/Q2).  Precedence here: explicit CLI flag > YAML > dataclass default.
"""
from __future__ import annotations

import argparse
import dataclasses
from typing import Any, Dict, Optional, Sequence, Tuple

import yaml

from ..models.config import GPTConfig

_TRAIN_MAP = {"batch_size": "batch_size", "gradient_accumulation_steps": "gradient_accumulation_steps",
              "learning_rate": "learning_rate", "weight_decay": "weight_decay", "beta1": "beta1", "beta2": "beta2",
              "grad_clip": "grad_clip", "max_steps": "max_steps", "warmup_steps": "warmup_steps",
              "log_interval": "log_interval", "eval_interval": "eval_interval", "save_interval": "save_interval"}


def explicit_args(parser: argparse.ArgumentParser, argv: Optional[Sequence[str]]) -> set:
    """Names of the options the user actually passed on the command line."""
    shadow = argparse.ArgumentParser(add_help=False)
    for a in parser._actions:
        if a.dest == "help" or not a.option_strings:
            continue
        kw = {"dest": a.dest, "default": argparse.SUPPRESS}
        if isinstance(a, (argparse._StoreTrueAction, argparse._StoreFalseAction)):
            kw["action"] = "store_true"
        else:
            kw["nargs"] = a.nargs
        shadow.add_argument(*a.option_strings, **kw)
    ns, _ = shadow.parse_known_args(argv)
    return set(vars(ns).keys())


def _set(obj, key, val):
    if obj is not None and hasattr(obj, key) and val is not None:
        cur = getattr(obj, key)
        if isinstance(cur, bool):
            val = bool(val)
        elif isinstance(cur, int) and not isinstance(cur, bool):
            val = int(float(val))
        elif isinstance(cur, float):
            val = float(val)
        setattr(obj, key, val)


def load_yaml_config(path: str, model_cfg: GPTConfig, train_cfg, fsdp_cfg=None, keep_model_preset: bool = False
                     ) -> Tuple[GPTConfig, Any, Any, Dict[str, Any]]:
    with open(path) as f:
        y = yaml.safe_load(f) or {}
    m = y.get("model", {}) or {}
    if not keep_model_preset:
        fields = {f.name for f in dataclasses.fields(GPTConfig)}
        kw = {k: v for k, v in m.items() if k in fields}
        if kw:
            base = dataclasses.asdict(model_cfg)
            base.update(kw)
            if "hidden_size" in kw and "intermediate_size" not in kw:
                base["intermediate_size"] = None
            model_cfg = GPTConfig(**base)
    else:
        for k in ("dropout", "attention_dropout", "use_flash_attention", "gradient_checkpointing"):
            _set(model_cfg, k, m.get(k))
    t = y.get("training", {}) or {}
    for yk, ak in _TRAIN_MAP.items():
        _set(train_cfg, ak, t.get(yk))
    d = y.get("distributed", {}) or {}
    _set(train_cfg, "mixed_precision", d.get("mixed_precision"))
    if fsdp_cfg is not None:
        _set(fsdp_cfg, "mixed_precision", d.get("mixed_precision"))
        for k, v in (y.get("fsdp", {}) or {}).items():
            _set(fsdp_cfg, k, v)
    c = y.get("checkpoint", {}) or {}
    _set(train_cfg, "checkpoint_dir", c.get("dir"))
    _set(train_cfg, "resume_from", c.get("resume_from"))
    return model_cfg, train_cfg, fsdp_cfg, (y.get("data", {}) or {})
