"""End-to-end CLI runs on CPU: YAML config -> train -> checkpoints -> resume (DDP and FSDP
trainers, single process, native dummy loader)."""
import json
import os

import torch

from distributed_llm_trainer_amd.training import ddp_trainer, fsdp_trainer
from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint

TINY = """
model:
  vocab_size: 256
  hidden_size: 64
  num_layers: 2
  num_heads: 2
  max_seq_len: 32
training:
  batch_size: 2
  gradient_accumulation_steps: 2
  learning_rate: 0.001
  warmup_steps: 2
  save_interval: 5
  log_interval: 1
data:
  dataset: dummy
"""


def _yaml(tmp_path):
    p = tmp_path / "tiny.yaml"
    p.write_text(TINY)
    return str(p)


def test_ddp_cli_train_save_resume(tmp_path, capsys):
    cfg = _yaml(tmp_path)
    ck = str(tmp_path / "ck")
    mj = str(tmp_path / "m.jsonl")
    tr = ddp_trainer.main(["--config", cfg, "--max_steps", "12", "--checkpoint_dir", ck, "--metrics_jsonl", mj])
    out = capsys.readouterr().out
    assert "Step      0 | Loss:" in out and "Steady-state tokens/sec" in out and "MFU" in out
    assert sorted(os.listdir(ck)) == ["final.pt", "step_10.pt", "step_5.pt"]
    recs = [json.loads(l) for l in open(mj)]
    assert recs[-1].get("summary") and recs[0]["step"] == 0
    c = load_checkpoint(os.path.join(ck, "final.pt"))
    assert c["global_step"] == 12 and len(c["optimizer"]["param_groups"]) == 2
    assert c["tokens_seen"] == 12 * 4 * 32
    losses = [r["loss"] for r in recs if "loss" in r]
    assert losses[-1] < losses[0]
    tr2 = ddp_trainer.main(["--config", cfg, "--max_steps", "14", "--checkpoint_dir", str(tmp_path / "ck2"),
                            "--resume_from", os.path.join(ck, "final.pt")])
    assert tr2.global_step == 14 and tr2.tokens_seen == 14 * 4 * 32
    for (n, p1) in tr.model.named_parameters():
        assert p1.shape == dict(tr2.model.named_parameters())[n].shape


def test_fsdp_cli_single_process(tmp_path, capsys):
    cfg = _yaml(tmp_path)
    ck = str(tmp_path / "ckf")
    tr = fsdp_trainer.main(["--config", cfg, "--max_steps", "6", "--checkpoint_dir", ck])
    out = capsys.readouterr().out
    assert "Tokens/s:" in out and "Mem:" in out
    c = load_checkpoint(os.path.join(ck, "final.pt"))
    assert c["global_step"] == 6 and "fsdp_config" in c
    assert all(isinstance(k, str) for k in c["optimizer"]["state"])
    assert torch.isfinite(torch.stack([v.float().norm() for v in c["model"].values()])).all()
