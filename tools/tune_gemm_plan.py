"""Offline exhaustive GEMM tuning -> the shipped plan file.

Runs the headline training steps (GPT-2 small, micro-batch 8 x GA 4 with the default
micro-step fusion, seq 1024, one GPU) with ``DLT_GEMM_TUNE=exhaustive``: every GEMM key
the step issues is timed over EVERY hipBLASLt solution that supports it (not just the
heuristic's first 24), the hand-written-vs-library races and split-K factors run as
usual, and the resulting picks are written with ``ops.gemm.save_plan``.
``configs/gemm_plan_mi355x.json`` is this tool's output; the GEMM planner loads it by
default (``ops/gemm.py``).  Minutes of tuning: run it on the GPU box, not per job.

usage: python tools/tune_gemm_plan.py [--out configs/gemm_plan_mi355x.json] [--model_size small]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="configs/gemm_plan_mi355x.json")
    ap.add_argument("--model_size", default="small")
    ap.add_argument("--batch_size", type=int, default=8)
    ap.add_argument("--grad_accum", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    os.environ["DLT_GEMM_TUNE"] = "exhaustive"
    os.environ["DLT_GEMM_PLAN"] = "none"  # start from nothing: every key is tuned here
    os.environ.setdefault("DLT_GEMM_VERBOSE", "1")  # one line per tuned key (progress)
    import torch
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.ops import gemm
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig.from_preset(a.model_size)
    tc = TrainingConfig(batch_size=a.batch_size, gradient_accumulation_steps=a.grad_accum, max_steps=1000,
                        mixed_precision="bf16")
    tr = DistributedTrainer(cfg, tc)
    g = torch.Generator().manual_seed(0)
    batch = torch.randint(0, cfg.vocab_size, (a.batch_size * a.grad_accum, cfg.max_seq_len), generator=g)
    for s in range(a.steps):  # step 1: sequential chains (tunes every key); step 2: pipelined
        t = time.time()
        tr.train_step({"input_ids": batch.to(tr.device)})
        torch.cuda.synchronize()
        print(f"step {s}: {time.time() - t:.1f} s", flush=True)
    gemm.save_plan(a.out)
    print(gemm.report(), flush=True)
    print(f"wrote {a.out}", flush=True)


if __name__ == "__main__":
    main()
