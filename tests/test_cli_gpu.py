"""End-to-end CLI runs on the MI355X (fused HIP engine, native loader, checkpoints):
the reference-compatible DDP and FSDP trainer CLIs, killed mid-way by fault injection
and resumed, land on the uninterrupted run's weights bit for bit (every gradient
reduction is fixed-order, dropout streams and the data stream resume exactly)."""
import math
import os
import subprocess
import sys

import pytest
import torch

from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint

pytestmark = pytest.mark.gpu

TINY = """
model:
  vocab_size: 1000
  hidden_size: 256
  num_layers: 2
  num_heads: 4
  max_seq_len: 256
training:
  batch_size: 2
  gradient_accumulation_steps: 4
  learning_rate: 0.001
  warmup_steps: 2
  save_interval: 4
  log_interval: 1
data:
  dataset: dummy
"""


def _run(module, args, env_extra, tmp_path):
    cfg = tmp_path / "tiny.yaml"
    cfg.write_text(TINY)
    env = dict(os.environ, **env_extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "DLT_FORCE_CPU"):
        env.pop(k, None)
    return subprocess.run([sys.executable, "-m", module, "--config", str(cfg), *args], env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("module", ["distributed_llm_trainer_amd.training.ddp_trainer",
                                    "distributed_llm_trainer_amd.training.fsdp_trainer"])
def test_cli_fault_injection_resume_is_exact_gpu(module, tmp_path):
    """The GEMM choices are pinned across the three processes with a plan file
    (DLT_GEMM_PLAN: written by the first run after its step 2, replayed by the others),
    the production recipe for bitwise-reproducible runs."""
    full, part = str(tmp_path / "full"), str(tmp_path / "part")
    plan = {"DLT_GEMM_PLAN": str(tmp_path / "gemm_plan.json")}
    r = _run(module, ["--max_steps", "10", "--checkpoint_dir", full], plan, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Step      0 | Loss:" in r.stdout
    r = _run(module, ["--max_steps", "10", "--checkpoint_dir", part], {"DLT_FAULT_INJECT": "6", **plan}, tmp_path)
    assert r.returncode == 17 and "injected fault at step 6" in r.stderr, r.stderr[-3000:]
    r = _run(module, ["--max_steps", "10", "--checkpoint_dir", part, "--resume_from", os.path.join(part, "step_4.pt")],
             plan, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.isfile(plan["DLT_GEMM_PLAN"])
    a = load_checkpoint(os.path.join(full, "final.pt"))
    b = load_checkpoint(os.path.join(part, "final.pt"))
    assert a["global_step"] == b["global_step"] == 10
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i, st in a["optimizer"]["state"].items():
        assert torch.equal(st["exp_avg_sq"], b["optimizer"]["state"][i]["exp_avg_sq"]), i


def test_infer_cli_gpu(tmp_path):
    """Train a tiny model through the DDP CLI on the GPU, then generate from its
    final.pt with the reference-compatible infer CLI (KV-cached HIP-graph decode)."""
    ck = str(tmp_path / "ck")
    r = _run("distributed_llm_trainer_amd.training.ddp_trainer", ["--max_steps", "3", "--checkpoint_dir", ck], {},
             tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ)
    env.pop("DLT_FORCE_CPU", None)
    r = subprocess.run([sys.executable, "src/eval/infer.py", "--checkpoint", os.path.join(ck, "final.pt"),
                        "--prompt", "Once upon a time,", "--max_new_tokens", "24", "--seed", "1"],
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Once upon a time," in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("streaming", [False, True])
def test_text_dataset_cli_gpu(tmp_path, streaming):
    """The TinyStories / OpenWebText paths on the GPU: a text corpus (gzip for the
    OpenWebText loader), tokenised offline, streamed or map-style, through the engine."""
    import gzip
    story = "Once upon a time, a little fox found a shiny stone near the river. " * 8
    text = "\n".join(f"{i}: {story}" for i in range(400))
    p = tmp_path / "corpus.txt.gz"
    with gzip.open(p, "wt") as f:
        f.write(text)
    args = ["--max_steps", "4", "--checkpoint_dir", str(tmp_path / "ck"), "--dataset", "openwebtext",
            "--data_path", str(p), "--no_final_save"] + (["--streaming"] if streaming else [])
    r = _run("distributed_llm_trainer_amd.training.ddp_trainer", args, {}, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    losses = [float(ln.split("Loss:")[1].split("|")[0]) for ln in r.stdout.splitlines() if "Loss:" in ln]
    assert len(losses) == 4 and all(math.isfinite(x) for x in losses), r.stdout[-2000:]
