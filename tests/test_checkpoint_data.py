"""Checkpoint format compatibility and the data loaders."""
import gzip
import os
import pickle

import pytest
import torch

from distributed_llm_trainer_amd.data.dummy import create_dummy_dataloader
from distributed_llm_trainer_amd.data.native import TokenFileDataset, write_token_file
from distributed_llm_trainer_amd.data.openwebtext import create_openwebtext_dataloader
from distributed_llm_trainer_amd.data.text import StreamingTextDataset, TextDataConfig, TokenizedTextDataset
from distributed_llm_trainer_amd.data.tokenizer import ByteTokenizer
from distributed_llm_trainer_amd.models.config import GPTConfig
from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint, save_checkpoint


def test_reference_format_checkpoint_loads_weights_only(tmp_path):
    """A checkpoint pickled the way the reference writes it (models.config.GPTConfig,
    __main__.TrainingConfig) loads with weights_only=True via the registered aliases."""
    from distributed_llm_trainer_amd.utils import checkpoint as ck
    ck.register_safe_globals()
    cfg_alias = ck._alias(GPTConfig, "models.config")
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    tc_alias = ck._alias(TrainingConfig, "__main__")
    import sys
    import types
    cfg = cfg_alias(vocab_size=100, hidden_size=32, num_layers=1, num_heads=2)
    tc = tc_alias()
    path = str(tmp_path / "ref.pt")
    # make the reference module paths resolvable for pickling (what the reference process has)
    fake_pkg, fake_mod = types.ModuleType("models"), types.ModuleType("models.config")
    fake_mod.GPTConfig = cfg_alias
    main = sys.modules["__main__"]
    had = hasattr(main, "TrainingConfig")
    old = getattr(main, "TrainingConfig", None)
    sys.modules["models"], sys.modules["models.config"] = fake_pkg, fake_mod
    main.TrainingConfig = tc_alias
    try:
        torch.save({"model": {"w": torch.ones(2)}, "optimizer": {"state": {}, "param_groups": []},
                    "global_step": 3, "tokens_seen": 9, "model_config": cfg, "training_config": tc}, path)
    finally:
        del sys.modules["models"], sys.modules["models.config"]
        if had:
            main.TrainingConfig = old
        else:
            del main.TrainingConfig
    raw = open(path, "rb").read()
    assert b"models.config" in raw and b"__main__" in raw
    c = load_checkpoint(path)
    assert c["global_step"] == 3 and c["model_config"].hidden_size == 32


_REF_LOADER = r"""
import importlib.abc, sys, types, dataclasses
class _Block(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in ("distributed_llm_trainer_amd", "src"):
            raise ImportError("blocked: " + name)
        return None
sys.meta_path.insert(0, _Block())
import torch
# the reference process: models.config.GPTConfig (a dataclass) and the placeholder
# TrainingConfig / FSDPConfig classes of its __main__ (infer.py:19-21)
@dataclasses.dataclass
class GPTConfig:
    vocab_size: int = 50257
    hidden_size: int = 768
    num_layers: int = 12
    num_heads: int = 12
    intermediate_size: int = None
    max_seq_len: int = 1024
models = types.ModuleType("models"); cfgmod = types.ModuleType("models.config")
GPTConfig.__module__ = "models.config"; cfgmod.GPTConfig = GPTConfig; models.config = cfgmod
sys.modules["models"], sys.modules["models.config"] = models, cfgmod
class TrainingConfig: pass
class FSDPConfig: pass
main = sys.modules["__main__"]; main.TrainingConfig = TrainingConfig; main.FSDPConfig = FSDPConfig
TrainingConfig.__module__ = FSDPConfig.__module__ = "__main__"
torch.serialization.add_safe_globals([GPTConfig, TrainingConfig, FSDPConfig])
ck = torch.load(sys.argv[1], map_location="cpu", weights_only=True)
assert "distributed_llm_trainer_amd" not in sys.modules
mc = ck["model_config"]
assert type(mc) is GPTConfig and mc.hidden_size == int(sys.argv[2]), (type(mc), mc.__dict__)
assert type(ck["training_config"]) is TrainingConfig
if len(sys.argv) > 3:
    assert type(ck["fsdp_config"]) is FSDPConfig and ck["fsdp_config"].sharding_strategy == sys.argv[3]
assert "embed_tokens.weight" in ck["model"]
print("REF-LOAD-OK", ck["global_step"])
"""


def _ref_load(path, hidden, fsdp=None):
    import subprocess
    import sys
    args = [sys.executable, "-c", _REF_LOADER, str(path), str(hidden)] + ([fsdp] if fsdp else [])
    r = subprocess.run(args, capture_output=True, text=True, cwd="/", timeout=300,
                       env={k: v for k, v in __import__("os").environ.items() if k != "PYTHONPATH"})
    assert r.returncode == 0 and "REF-LOAD-OK" in r.stdout, r.stderr[-3000:]


def test_checkpoint_readable_by_reference_loader(tmp_path):
    """Reverse direction: a DDP checkpoint written by this package
    pickles its configs as models.config.GPTConfig / __main__.TrainingConfig, so a
    process WITHOUT this package (import blocked) loads it with weights_only=True given
    only the reference's own classes -- and our side still loads it too."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig(vocab_size=128, hidden_size=64, num_layers=1, num_heads=2, max_seq_len=32,
                    dropout=0.0, attention_dropout=0.0)
    tr = DistributedTrainer(cfg, TrainingConfig(batch_size=2, gradient_accumulation_steps=1, warmup_steps=1))
    path = tmp_path / "final.pt"
    tr.save_checkpoint(str(path))
    raw = open(path, "rb").read()
    assert b"distributed_llm_trainer_amd" not in raw
    _ref_load(path, 64)
    c = load_checkpoint(str(path))
    assert c["model_config"].hidden_size == 64 and isinstance(c["model_config"], GPTConfig)
    import sys
    assert "models.config" not in sys.modules  # the pickling aliases were removed again
    # saving again what was loaded (alias instances) keeps the reference paths
    save_checkpoint(str(tmp_path / "again.pt"), c)
    _ref_load(tmp_path / "again.pt", 64)


def test_checkpoint_save_restores_existing_parent_package(tmp_path, monkeypatch):
    """Saving with a real (unrelated) ``models`` package already imported must leave it
    as it was: no ``models.config`` attribute pointing at the pickling stand-in."""
    import sys
    import types
    real = types.ModuleType("models")
    monkeypatch.setitem(sys.modules, "models", real)
    cfg = GPTConfig(vocab_size=128, hidden_size=64, num_layers=1, num_heads=2, max_seq_len=32)
    save_checkpoint(str(tmp_path / "c.pt"), {"model": {}, "model_config": cfg})
    assert sys.modules["models"] is real and not hasattr(real, "config")
    assert "models.config" not in sys.modules
    assert load_checkpoint(str(tmp_path / "c.pt"))["model_config"].hidden_size == 64


def test_fsdp_checkpoint_readable_by_reference_loader(tmp_path):
    """Same for the FSDP trainer's FULL_STATE_DICT file (adds __main__.FSDPConfig)."""
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    path = tmp_path / "fsdp.pt"
    cfg = GPTConfig(vocab_size=128, hidden_size=48, num_layers=1, num_heads=2, max_seq_len=32)
    save_checkpoint(str(path), {"model": {"embed_tokens.weight": torch.zeros(128, 48)},
                                "optimizer": {"state": {}, "param_groups": []}, "global_step": 5, "tokens_seen": 7,
                                "model_config": cfg, "training_config": FSDPTrainingConfig(),
                                "fsdp_config": FSDPConfig(sharding_strategy="SHARD_GRAD_OP")})
    _ref_load(path, 48, "SHARD_GRAD_OP")
    c = load_checkpoint(str(path))
    assert c["fsdp_config"].sharding_strategy == "SHARD_GRAD_OP"


def test_atomic_save(tmp_path):
    p = str(tmp_path / "a" / "b.pt")
    save_checkpoint(p, {"x": torch.arange(3)})
    assert os.path.exists(p) and not [f for f in os.listdir(tmp_path / "a") if ".tmp." in f]


def _write_corpus(path, n=200):
    lines = [f"Story {i}: the quick brown fox jumps over the lazy dog number {i}." for i in range(n)]
    with open(path, "w") as f:
        f.write("\n".join(lines))
    return lines


def test_map_style_windows(tmp_path):
    p = str(tmp_path / "t.txt")
    _write_corpus(p)
    ds = TokenizedTextDataset(TextDataConfig(path=p, seq_len=64), tokenizer=ByteTokenizer())
    n = len(ds.tokens)
    assert len(ds) == (n - 1) // 64
    (x,) = ds[1]
    assert torch.equal(x, ds.tokens[64:128])


def test_streaming_sharding_and_cache(tmp_path):
    p = str(tmp_path / "t.txt")
    _write_corpus(p)
    tok = ByteTokenizer()
    cfg = TextDataConfig(path=p, seq_len=32, cache_max_tokens=100000)
    shards = [list(StreamingTextDataset(cfg, rank=r, world_size=2, tokenizer=tok)) for r in range(2)]
    assert shards[0] and shards[1]
    assert not torch.equal(shards[0][0], shards[1][0])
    ds = StreamingTextDataset(cfg, rank=0, world_size=1, tokenizer=tok)
    a = list(ds)
    misses = ds.cache.misses
    b = list(ds)
    assert ds.cache.misses == misses and ds.cache.hits >= misses  # second pass: all cache hits (Q9 fixed)
    assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_openwebtext_gz_and_path_fallback(tmp_path):
    p = str(tmp_path / "owt.txt")
    lines = _write_corpus(p)
    with gzip.open(p + ".gz", "wt") as f:
        f.write("\n".join(lines))
    os.remove(p)
    dl = create_openwebtext_dataloader(p, batch_size=2, seq_len=32, tokenizer=ByteTokenizer(), num_workers=0)
    (batch,) = next(iter(dl))
    assert batch.shape == (2, 32)


def test_token_file_dataset(tmp_path):
    p = str(tmp_path / "tok.bin")
    write_token_file(p, list(range(1000)))
    ds = TokenFileDataset(p, 100)
    assert len(ds) == 9
    (x,) = ds[2]
    assert x.tolist() == list(range(200, 300))


def test_dummy_loader_seeded_drop_last():
    a = next(iter(create_dummy_dataloader(4, 16, 100, num_batches=3, seed=1, native=False)))[0]
    b = next(iter(create_dummy_dataloader(4, 16, 100, num_batches=3, seed=1, native=False)))[0]
    assert a.shape == (4, 16)
    dl = create_dummy_dataloader(3, 16, 100, num_batches=2, seed=1, native=False)
    assert all(x[0].shape[0] == 3 for x in dl)


def test_load_model_state_is_strict():
    """Loading a model state dict: wrapper prefixes are stripped, missing RoPE buffers
    are tolerated (deterministic), anything else missing or unexpected raises instead
    of silently leaving random weights in place."""
    from distributed_llm_trainer_amd.models.gpt import GPT
    from distributed_llm_trainer_amd.utils.checkpoint import load_model_state
    cfg = GPTConfig(vocab_size=64, hidden_size=32, num_layers=1, num_heads=2, max_seq_len=16)
    torch.manual_seed(0)
    src = GPT(cfg)
    dst = GPT(cfg)
    sd = {f"module.{k}": v for k, v in src.state_dict().items() if "rotary_emb" not in k}
    load_model_state(dst, sd)
    assert torch.equal(dst.embed_tokens.weight, src.embed_tokens.weight)
    bad = dict(sd)
    bad.pop("module.layers.0.mlp.up_proj.weight")
    with pytest.raises(RuntimeError, match="missing"):
        load_model_state(GPT(cfg), bad)
    extra = dict(sd)
    extra["module.layers.5.mlp.up_proj.weight"] = torch.zeros(1)
    with pytest.raises(RuntimeError, match="unexpected"):
        load_model_state(GPT(cfg), extra)


def test_tokenizer_offline_is_usable():
    """get_tokenizer('gpt2') never hands out a tokenizer that encodes to nothing (this
    image's offline transformers yields vocab_size 0): real GPT-2 BPE if its files are
    available, else the byte tokenizer with a warning; DLT_TOKENIZER_STRICT=1 raises."""
    import warnings
    from distributed_llm_trainer_amd.data.tokenizer import get_tokenizer
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        tok = get_tokenizer("gpt2")
    ids = tok.encode("once upon a time")
    assert len(ids) > 0 and all(0 <= i < 50257 for i in ids)
    if isinstance(tok, ByteTokenizer):
        os.environ["DLT_TOKENIZER_STRICT"] = "1"
        try:
            with pytest.raises(RuntimeError, match="could not load tokenizer"):
                get_tokenizer("gpt2")
        finally:
            del os.environ["DLT_TOKENIZER_STRICT"]
