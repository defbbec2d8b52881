"""Full-size convergence check on one GPU: GPT-2 small (151.9M), the headline DDP step
(B8 x GA4, S1024, bf16, dropout 0.1, pipelined engine) trained on a small fixed corpus of
synthetic token sequences for N steps.  A correct forward/backward/optimizer memorises
it, so the loss must fall far below ln(V) = 10.8; the eager autocast model is trained on
the same data in the same way for comparison (parity of the loss curve).

usage: python tools/converge.py --steps 150 [--eager] [--precision bf16|fp16|fp32] [--memory_first]

``--precision`` trains the engine in another activation precision on the same data and
init (fp16: dynamic loss scaling; fp32: the fp32 kernels and GEMM-formulated attention),
so the curves of the three can be compared step by step.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--eager", action="store_true", help="reference-style eager autocast model instead of the engine")
    ap.add_argument("--log", type=int, default=10)
    ap.add_argument("--seed", type=int, default=1234, help="trainer seed (model init + dropout streams)")
    ap.add_argument("--precision", default="bf16", choices=("bf16", "fp16", "fp32"))
    ap.add_argument("--memory_first", action="store_true", help="TrainingConfig.memory_first (the <= 8.2 GB mode)")
    a = ap.parse_args()
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig.gpt2_small()
    tc = TrainingConfig(batch_size=8, gradient_accumulation_steps=4, max_steps=a.steps, warmup_steps=20,
                        learning_rate=a.lr, mixed_precision=a.precision, seed=a.seed, memory_first=a.memory_first)
    tr = DistributedTrainer(cfg, tc, use_engine=not a.eager)
    if a.eager:  # the reference path: torch modules under bf16 autocast
        tr.autocast_ctx = torch.autocast(device_type="cuda", dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(7)
    corpus = torch.randint(0, cfg.vocab_size, (64, 1024), generator=g).cuda()  # 2 distinct batches of 32
    out = []
    t0 = time.time()
    for step in range(a.steps):
        batch = corpus[(step % 2) * 32:(step % 2 + 1) * 32]
        loss = tr.train_step({"input_ids": batch}, sync_loss=(step % a.log == 0 or step == a.steps - 1))["loss"]
        if step % a.log == 0 or step == a.steps - 1:
            out.append({"step": step, "loss": float(loss)})
            print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"path": "eager" if a.eager else "engine", "precision": a.precision, "seed": a.seed,
                      "memory_first": a.memory_first, "seconds": round(time.time() - t0, 1),
                      "first": out[0]["loss"], "last": out[-1]["loss"]}), flush=True)


if __name__ == "__main__":
    main()
