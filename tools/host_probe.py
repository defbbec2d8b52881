"""Host-side issue time of the headline training step vs its GPU time.

Runs the bench.py headline config, then times the Python issue loop of K steps (no
synchronisation inside it) and the wall time until the GPU has finished them.  If the
issue time is close to the wall time, the step is at risk of becoming host-bound on a
loaded host (CPU contention shows up as GPU idle gaps)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = GPTConfig.from_preset("small")
    cfg.max_seq_len = 1024
    tc = TrainingConfig(batch_size=8, gradient_accumulation_steps=4, max_steps=100000, mixed_precision="bf16")
    tr = DistributedTrainer(cfg, tc)
    dev = tr.device
    B = 32
    batches = [torch.randint(0, cfg.vocab_size, (B, 1024)).to(dev) for _ in range(4)]
    for i in range(3):
        tr.train_step({"input_ids": batches[i % 4]}, sync_loss=False)
    torch.cuda.synchronize(dev)
    for rep in range(3):
        t0 = time.perf_counter()
        for i in range(K):
            tr.train_step({"input_ids": batches[i % 4]}, sync_loss=False)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        print(f"K={K}: host issue {1e3 * (t1 - t0) / K:.2f} ms/step, wall {1e3 * (t2 - t0) / K:.2f} ms/step",
              flush=True)


if __name__ == "__main__":
    main()
