"""Offline exhaustive GEMM tuning -> the shipped plan file.

Runs training steps of the given configurations (default: the headline, GPT-2 small,
micro-batch 8 x GA 4 with the default micro-step fusion, seq 1024, one GPU; the other
bench-table rows can be added, all tuned into one plan) with ``DLT_GEMM_TUNE=exhaustive``: every GEMM key
the step issues is timed over EVERY hipBLASLt solution that supports it (not just the
heuristic's first 24), the hand-written-vs-library races and split-K factors run as
usual, and the resulting picks are written with ``ops.gemm.save_plan``.
``configs/gemm_plan_mi355x.json`` is this tool's output; the GEMM planner loads it by
default (``ops/gemm.py``).  Minutes of tuning: run it on the GPU box, not per job.

usage: python tools/tune_gemm_plan.py [--out configs/gemm_plan_mi355x.json] [--configs ddp_small,fsdp_small,...]
       python tools/tune_gemm_plan.py --merge --configs ddp_small_fp32   # add keys to the shipped plan

``--merge`` keeps every pin of the shipped plan (replayed, not re-tuned) and tunes only the
keys it lacks; the fp32 pins of the shipped plan came from this (``--precision fp32``
step 95.8k -> 109.8k tok/s, ``profiles/r5_fp32_attention.md``).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


CONFIGS = {  # name -> (mode, preset, micro-batch, grad-accum[, precision]), the tools/bench_table.py rows
    "ddp_small": ("ddp", "small", 8, 4),
    "fsdp_small": ("fsdp", "small", 8, 4),
    "ddp_medium": ("ddp", "medium", 4, 8),
    "fsdp_medium": ("fsdp", "medium", 4, 8),
    "ddp_xl": ("ddp", "xl", 4, 8),
    "fsdp_xl": ("fsdp", "xl", 4, 8),
    "ddp_small_fp32": ("ddp", "small", 8, 4, "fp32"),
    "ddp_small_fp16": ("ddp", "small", 8, 4, "fp16"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="configs/gemm_plan_mi355x.json")
    ap.add_argument("--configs", default="ddp_small",
                    help="comma-separated: " + ",".join(CONFIGS) + " (all tuned in one process, one plan file)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--merge", action="store_true",
                    help="start from the shipped plan (its pins replayed) and add only the keys it lacks")
    a = ap.parse_args()
    os.environ["DLT_GEMM_TUNE"] = "exhaustive"
    if a.merge:
        os.environ.pop("DLT_GEMM_PLAN", None)  # the shipped plan is loaded and pinned
    else:
        os.environ["DLT_GEMM_PLAN"] = "none"  # start from nothing: every key is tuned here
    os.environ.setdefault("DLT_GEMM_VERBOSE", "1")  # one line per tuned key (progress)
    import gc

    import torch
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.ops import gemm
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig, TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    for name in a.configs.split(","):
        mode, size, bs, ga, *prec = CONFIGS[name]
        prec = prec[0] if prec else "bf16"
        cfg = GPTConfig.from_preset(size)
        if mode == "ddp":
            tr = DistributedTrainer(cfg, TrainingConfig(batch_size=bs, gradient_accumulation_steps=ga, max_steps=1000,
                                                        mixed_precision=prec))
        else:
            tr = FSDPTrainer(cfg, FSDPTrainingConfig(batch_size=bs, gradient_accumulation_steps=ga, max_steps=1000),
                             FSDPConfig(mixed_precision=prec))
        g = torch.Generator().manual_seed(0)
        batch = torch.randint(0, cfg.vocab_size, (bs * ga, cfg.max_seq_len), generator=g)
        for s in range(a.steps):  # step 1: sequential chains (tunes every key); step 2: pipelined
            t = time.time()
            tr.train_step({"input_ids": batch.to(tr.device)})
            torch.cuda.synchronize()
            print(f"{name} step {s}: {time.time() - t:.1f} s", flush=True)
        del tr, batch
        gc.collect()
        torch.cuda.empty_cache()
    gemm.save_plan(a.out)
    print(gemm.report(), flush=True)
    print(f"wrote {a.out}", flush=True)


if __name__ == "__main__":
    main()
