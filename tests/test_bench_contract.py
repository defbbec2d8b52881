"""bench.py's driver contract, rehearsed on CPU (gloo) with a tiny model override.

The driver runs ``python bench.py --gpus N --steps K --warmup W`` for N=1 and
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
127.0.0.1 --master-port P bench.py ...`` for N>1; rank 0 must print exactly ONE JSON
line with the whole-job tokens/s.  This runs both launch forms end to end (real
collectives over 2 ranks), so the N>1 path is exercised before the driver's 8-GPU run.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = "vocab_size=384,hidden_size=64,num_layers=2,num_heads=4"
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="2", DLT_FORCE_CPU="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check(out, n, steps, warmup):
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == warmup
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["vs_baseline"] is None  # custom model: never compared to the headline number
    cfg = out["config"]
    assert cfg["global_batch"] == 2 * 2 * n and cfg["seq_len"] == 32 and cfg["parallelism"] == f"ddp{n}"
    tokens = steps * cfg["global_batch"] * cfg["seq_len"]
    # value is the whole-job aggregate: total tokens over the (max-over-ranks) elapsed time
    assert out["value"] == pytest.approx(tokens / (out["ms_per_step"] * steps / 1000.0), rel=1e-2)


ARGS = ["--steps", "2", "--warmup", "1", "--batch_size", "2", "--grad_accum", "2", "--seq_len", "32",
        "--model_override", TINY]


def test_bench_single_process_contract():
    out = _run([sys.executable, "bench.py", "--gpus", "1"] + ARGS)
    _check(out, 1, 2, 1)


def test_bench_torchrun_two_ranks_contract():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2"] + ARGS
    out = _run(cmd)
    _check(out, 2, 2, 1)


def test_bench_torchrun_eight_ranks_contract():
    """The driver's largest launch (8 ranks, one node) rehearsed over gloo on the CPU:
    bucket all-reduces across 8 ranks, the max-over-ranks timing, one JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8"] + ARGS
    out = _run(cmd)
    _check(out, 8, 2, 1)
