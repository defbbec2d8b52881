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
* Reverse direction: the config objects are pickled under the reference's class paths
  (``models.config.GPTConfig``, ``__main__.TrainingConfig`` / ``__main__.FSDPConfig``),
  so the reference's own loader reads our files without this package installed
  (``tests/test_checkpoint_data.py::test_checkpoint_readable_by_reference_loader``).
* FSDP SHARDED_STATE_DICT (discussed, not implemented, in the reference): per-rank
  shard files + ``meta.json``; ``consolidate_sharded`` turns one into the full format
  (``python -m distributed_llm_trainer_amd.utils.checkpoint consolidate DIR OUT``).
* Writes are atomic (tmp file + rename), so a crash mid-save never leaves a
  truncated ``final.pt`` behind for ``--resume_from``.
"""
from __future__ import annotations

import dataclasses
import json
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


# Reverse compatibility: the config objects of a checkpoint are
# pickled under the class paths the REFERENCE writes -- ``models.config.GPTConfig``
# (its model package, imported with ``src`` on sys.path) and ``__main__.TrainingConfig``
# / ``__main__.FSDPConfig`` (its trainers run as scripts) -- so the reference's loader
# (``src/eval/infer.py:15-21,53-57``: ``from models.config import GPTConfig`` plus a
# placeholder ``TrainingConfig`` in ``__main__``) reads our files without this package.
_REF_PATHS = {"GPTConfig": ("models.config", "GPTConfig"), "TrainingConfig": ("__main__", "TrainingConfig"),
              "FSDPTrainingConfig": ("__main__", "TrainingConfig"), "FSDPConfig": ("__main__", "FSDPConfig")}
_REF_ALIASES: Dict[Any, Any] = {}


def _ref_alias(cls):
    """Subclass of ``cls`` whose pickled name is the reference's class path."""
    if cls not in _REF_ALIASES:
        module, name = _REF_PATHS[cls.__name__]
        _REF_ALIASES[cls] = type(name, (cls,), {"__module__": module, "__qualname__": name})
    return _REF_ALIASES[cls]


def _to_reference_pickle(payload: Dict[str, Any]):
    """(payload with config objects re-classed to their reference aliases, list of
    (module, name, alias) the pickler must be able to look up)."""
    out, need = dict(payload), []
    for k, v in payload.items():
        name = type(v).__name__
        if k.endswith("_config") and dataclasses.is_dataclass(v) and not isinstance(v, type) and name in _REF_PATHS:
            base = type(v) if type(v) not in _REF_ALIASES.values() else type(v).__mro__[1]
            alias = _ref_alias(base)
            obj = alias.__new__(alias)
            obj.__dict__.update(v.__dict__)
            out[k] = obj
            need.append((alias.__module__, alias.__qualname__, alias))
    return out, need


class _RefModules:
    """Make ``module.name`` resolve to the alias classes while pickling (pickle checks
    that a class is importable under the path it writes), then restore sys.modules and
    every attribute it set.  Process-wide while active: checkpoints are saved from the
    trainer's main thread only."""

    def __init__(self, need):
        self.need = need
        self.saved = []

    def __enter__(self):
        import sys
        import types
        for module, name, alias in self.need:
            parts = module.split(".")
            for i in range(1, len(parts) + 1):
                mn = ".".join(parts[:i])
                if mn not in sys.modules:
                    self.saved.append(("mod", mn, None))
                    sys.modules[mn] = types.ModuleType(mn)
                    if i > 1:
                        # the parent's attribute too: a real parent package imported
                        # earlier must not keep pointing at the stand-in afterwards
                        parent = ".".join(parts[:i - 1])
                        pmod = sys.modules[parent]
                        self.saved.append(("attr", parent, (parts[i - 1], getattr(pmod, parts[i - 1], _MISSING))))
                        setattr(pmod, parts[i - 1], sys.modules[mn])
            mod = sys.modules[module]
            self.saved.append(("attr", module, (name, getattr(mod, name, _MISSING))))
            setattr(mod, name, alias)
        return self

    def __exit__(self, *exc):
        import sys
        for kind, mn, extra in reversed(self.saved):
            if kind == "attr":
                name, old = extra
                mod = sys.modules.get(mn)
                if mod is None:
                    continue
                if old is _MISSING:
                    if hasattr(mod, name):
                        delattr(mod, name)
                else:
                    setattr(mod, name, old)
            else:
                sys.modules.pop(mn, None)
        return False


_MISSING = object()


def save_checkpoint(path: str, payload: Dict[str, Any]) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    payload, need = _to_reference_pickle(payload)
    with _RefModules(need):
        torch.save(payload, tmp)
    os.replace(tmp, path)


def _canonical_config(v):
    """A config object unpickled through one of the reference-path aliases, as an
    instance of this package's own class (dataclass ``==`` compares classes).  The
    reference pickles both trainers' TrainingConfig as ``__main__.TrainingConfig``: the
    field set tells the DDP and FSDP schemas apart."""
    from ..training.configs import FSDPConfig, FSDPTrainingConfig, TrainingConfig
    bases = (GPTConfig, TrainingConfig, FSDPTrainingConfig, FSDPConfig)
    if type(v) in bases or not any(isinstance(v, b) for b in bases):
        return v
    base = next(b for b in bases if isinstance(v, b))
    if base in (TrainingConfig, FSDPTrainingConfig):
        keys = set(v.__dict__)
        base = max((TrainingConfig, FSDPTrainingConfig),
                   key=lambda c: len(keys & {f.name for f in dataclasses.fields(c)}) - len(
                       {f.name for f in dataclasses.fields(c)} - keys))
    obj = base.__new__(base)
    obj.__dict__.update(v.__dict__)
    return obj


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    register_safe_globals()
    ck = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(ck, dict):
        for k in list(ck):
            if k.endswith("_config"):
                ck[k] = _canonical_config(ck[k])
    return ck


SHARDED_FORMAT = "dlt-fsdp-sharded-v1"


def write_json_atomic(path: str, obj: Dict[str, Any]) -> None:
    tmp = f"{path}.tmp.{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1)
    os.replace(tmp, path)


def read_sharded_meta(path: str) -> Dict[str, Any]:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != SHARDED_FORMAT:
        raise ValueError(f"{path}: not a sharded checkpoint ({meta.get('format')!r})")
    return meta


@torch.no_grad()
def consolidate_sharded(path: str, out: Optional[str] = None) -> Dict[str, Any]:
    """Rebuild the reference FULL_STATE_DICT payload (fp32 ``model`` with
    the reference keys incl. RoPE buffers and the tied ``lm_head.weight``; FQN-keyed
    ``optimizer``; counters; config objects) from a SHARDED_STATE_DICT directory written
    by ``FSDPTrainer.save_sharded_checkpoint``.  Runs offline on CPU, one unit at a
    time; writes it to ``out`` if given.  Any world size can then load the result."""
    from ..training.configs import FSDPConfig, FSDPTrainingConfig
    meta = read_sharded_meta(path)
    W = meta["shard_world"]
    # one file per shard index (HYBRID_SHARD replicas hold identical shards)
    by_shard: Dict[int, Dict[str, Any]] = {}
    for fn in sorted(os.listdir(path)):
        if fn.startswith("shard_") and fn.endswith(".pt") and len(by_shard) < W:
            c = torch.load(os.path.join(path, fn), map_location="cpu", weights_only=True, mmap=True)
            by_shard.setdefault(int(c["shard_rank"]), c["units"])
    missing = [i for i in range(W) if i not in by_shard]
    if missing:
        raise FileNotFoundError(f"{path}: missing shard files for shard ranks {missing}")
    shards = [by_shard[i] for i in range(W)]
    params, mom, var = {}, {}, {}
    for uid, lay in meta["units"].items():
        full = {k: torch.cat([shards[i][uid][k] for i in range(W)]) for k in ("param", "exp_avg", "exp_avg_sq")}
        if full["param"].numel() != lay["padded"]:
            raise ValueError(f"unit {uid}: {full['param'].numel()} elements, layout says {lay['padded']}")
        for name, off, n, shape in lay["segs"]:
            params[name] = full["param"][off:off + n].view(shape).clone()
            mom[name] = full["exp_avg"][off:off + n].view(shape).clone()
            var[name] = full["exp_avg_sq"][off:off + n].view(shape).clone()
    buffers = load_checkpoint(os.path.join(path, "extra.pt"))["buffers"]
    model = {}
    for k in meta["state_dict_keys"]:
        if k in params:
            model[k] = params[k]
        elif k == "lm_head.weight":
            model[k] = params["embed_tokens.weight"]
        else:
            model[k] = buffers[k]
    step = torch.tensor(float(meta["optimizer_step"]))
    names = [n for n in meta["param_order"] if n in params]
    group = dict(meta["param_group"])
    if isinstance(group.get("betas"), list):
        group["betas"] = tuple(group["betas"])
    group["params"] = names
    optim = {"state": {n: {"step": step.clone(), "exp_avg": mom[n], "exp_avg_sq": var[n]} for n in names},
             "param_groups": [group]}
    payload = {"model": model, "optimizer": optim, "global_step": meta["global_step"],
               "tokens_seen": meta["tokens_seen"], "model_config": GPTConfig.from_dict(meta["model_config"]),
               "training_config": FSDPTrainingConfig(**meta["training_config"]),
               "fsdp_config": FSDPConfig(**meta["fsdp_config"])}
    if out:
        save_checkpoint(out, payload)
    return payload


_ROPE_BUFFERS = (".rotary_emb.inv_freq", ".rotary_emb.cos_cached", ".rotary_emb.sin_cached")


def normalize_state_dict_keys(sd: Dict[str, Any]) -> Dict[str, Any]:
    """Drop wrapper prefixes (DDP ``module.``, ``torch.compile``'s ``_orig_mod.``,
    FSDP / checkpoint-wrapper module names) that a checkpoint written by another
    trainer may carry."""
    out = {}
    for k, v in sd.items():
        parts = [p for p in k.split(".") if p not in ("module", "_orig_mod", "_fsdp_wrapped_module",
                                                       "_checkpoint_wrapped_module")]
        out[".".join(parts)] = v
    return out


@torch.no_grad()
def load_model_state(model: torch.nn.Module, sd: Dict[str, Any]) -> None:
    """Load a reference-format ``"model"`` state dict, strictly.

    The only keys allowed to be missing are the RoPE buffers (deterministic, rebuilt by
    the model); any other missing key or any unexpected key raises -- a checkpoint of a
    different model (or one whose keys do not match) must not silently leave random
    weights in place while training continues."""
    res = model.load_state_dict(normalize_state_dict_keys(sd), strict=False)
    missing = [k for k in res.missing_keys if not k.endswith(_ROPE_BUFFERS)]
    if missing or res.unexpected_keys:
        raise RuntimeError(f"checkpoint does not match the model: missing {missing[:8]}"
                           f"{'...' if len(missing) > 8 else ''} ({len(missing)}), unexpected "
                           f"{list(res.unexpected_keys)[:8]} ({len(res.unexpected_keys)})")


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


def _main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="checkpoint tools")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("consolidate", help="sharded FSDP checkpoint dir -> reference full checkpoint file")
    c.add_argument("src")
    c.add_argument("out")
    args = ap.parse_args(argv)
    if args.cmd == "consolidate":
        p = consolidate_sharded(args.src, args.out)
        print(f"wrote {args.out}: {len(p['model'])} tensors, step {p['global_step']}")


if __name__ == "__main__":
    _main()
