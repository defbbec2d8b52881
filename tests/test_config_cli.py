"""Config presets, YAML loading (--config) and CLI precedence; CLI entry points run."""
import os
import subprocess
import sys

import pytest
import torch

from distributed_llm_trainer_amd.models.config import GPTConfig
from distributed_llm_trainer_amd.training import ddp_trainer, fsdp_trainer
from distributed_llm_trainer_amd.training.common import cosine_lr
from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig, TrainingConfig
from distributed_llm_trainer_amd.utils.config_loader import explicit_args, load_yaml_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_defaults():
    t = TrainingConfig()
    assert (t.batch_size, t.learning_rate, t.gradient_accumulation_steps, t.log_interval, t.checkpoint_dir) == \
        (8, 6e-4, 4, 1, "checkpoints")
    f = FSDPTrainingConfig()
    assert (f.batch_size, f.learning_rate, f.gradient_accumulation_steps, f.log_interval, f.checkpoint_dir) == \
        (4, 3e-4, 8, 10, "checkpoints_fsdp")
    c = FSDPConfig()
    assert c.sharding_strategy == "FULL_SHARD" and c.activation_checkpointing and c.limit_all_gathers
    assert GPTConfig().intermediate_size == 3072 and GPTConfig.gpt2_xl().num_heads == 25


def test_yaml_loading_and_precedence():
    p = ddp_trainer.build_parser()
    argv = ["--config", os.path.join(ROOT, "configs/small_model.yaml"), "--batch_size", "2"]
    given = explicit_args(p, argv)
    assert "batch_size" in given and "max_steps" not in given
    m, t, _, data = load_yaml_config(argv[1], GPTConfig.gpt2_small(), TrainingConfig(), None)
    assert m.use_flash_attention is True and t.log_interval == 10 and t.learning_rate == 6e-4
    assert t.checkpoint_dir == "checkpoints/gpt2-small" and data["dataset"] == "openwebtext"
    m2, t2, f2, _ = load_yaml_config(os.path.join(ROOT, "configs/medium_model.yaml"), GPTConfig(),
                                     FSDPTrainingConfig(), FSDPConfig())
    assert m2.hidden_size == 1024 and m2.num_layers == 24 and m2.gradient_checkpointing
    assert t2.gradient_accumulation_steps == 8 and f2.backward_prefetch == "BACKWARD_PRE"


def test_lr_schedule():
    # warmup then cosine to 0.1*lr; clamped past max_steps (reference DDP is not, Q6)
    assert cosine_lr(0, 6e-4, 3, 10) == 0.0
    assert abs(cosine_lr(3, 6e-4, 3, 10) - 6e-4) < 1e-12
    assert abs(cosine_lr(10, 6e-4, 3, 10) - 6e-5) < 1e-12
    assert abs(cosine_lr(17, 6e-4, 3, 10) - 6e-5) < 1e-12
    assert abs(cosine_lr(17, 6e-4, 3, 10, clamp=False) - 6e-4) < 1e-9  # reference quirk reproduced


def test_reference_lr_order_option():
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    os.environ.pop("RANK", None)
    cfg = GPTConfig(vocab_size=128, hidden_size=32, num_layers=1, num_heads=2, max_seq_len=16)
    tc = TrainingConfig(batch_size=1, gradient_accumulation_steps=1, warmup_steps=3, max_steps=10,
                        lr_schedule_fix=False)
    tr = DistributedTrainer(cfg, tc)
    lrs = [tr.train_step({"input_ids": torch.randint(0, 128, (1, 16))})["lr"] for _ in range(3)]
    # reference semantics (ddp_trainer.py:360-362): the LR set AFTER step k is get_lr(k)
    assert lrs == [0.0, 6e-4 / 3, 2 * 6e-4 / 3]


@pytest.mark.parametrize("entry", ["src/training/ddp_trainer.py", "src/training/fsdp_trainer.py"])
def test_cli_help(entry):
    r = subprocess.run([sys.executable, os.path.join(ROOT, entry), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--model_size" in r.stdout and "--config" in r.stdout


def test_ddp_cli_end_to_end(tmp_path):
    """The plumbing config: CPU, dummy data, tiny step count, checkpoint + resume."""
    env = dict(os.environ, DLT_DUMMY_BATCHES="2")
    env.pop("RANK", None)
    args = [sys.executable, os.path.join(ROOT, "src/training/ddp_trainer.py"), "--model_size", "small",
            "--batch_size", "1", "--max_steps", "2", "--seq_len", "32", "--gradient_accumulation_steps", "1",
            "--checkpoint_dir", str(tmp_path), "--save_interval", "1"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Step      0 | Loss:" in r.stdout and "Tokens/sec:" in r.stdout
    assert (tmp_path / "final.pt").exists() and (tmp_path / "step_1.pt").exists()
    r2 = subprocess.run(args[:-4] + ["--max_steps", "3", "--resume_from", str(tmp_path / "final.pt"),
                                     "--checkpoint_dir", str(tmp_path / "r"), "--no_final_save"],
                        capture_output=True, text=True, timeout=600, env=env)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "Loaded Checkpoint" in r2.stdout and "Step      2 |" in r2.stdout


def test_debug_kernel_library_builds():
    """The DLT_DEBUG (device bounds-check) build of every HIP source compiles for gfx950
    (hipcc cross-compiles here without a GPU)."""
    import shutil
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    from distributed_llm_trainer_amd.ops import build as kb
    path = kb.build(verbose=False, debug=True)
    assert path.endswith("_dlt_kernels_debug.so") and os.path.exists(path)


@pytest.mark.parametrize("given,knob,expect", [("4", None, "16"), (None, None, "16"), ("32", None, "32"),
                                               ("4", "0", "4"), ("4", "8", "8")])
def test_package_import_raises_hw_queues(given, knob, expect):
    """Importing the package raises GPU_MAX_HW_QUEUES before the HIP runtime starts
    (profiles/r2_hw_queues.md); DLT_HW_QUEUES sets the minimum, 0 leaves it alone."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "DLT_HW_QUEUES")}
    if given is not None:
        env["GPU_MAX_HW_QUEUES"] = given
    if knob is not None:
        env["DLT_HW_QUEUES"] = knob
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", "import os, distributed_llm_trainer_amd; "
                        "print(os.environ.get('GPU_MAX_HW_QUEUES'))"], cwd=root, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == expect
