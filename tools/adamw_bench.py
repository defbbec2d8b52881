"""Standalone timing of the flat AdamW kernel at the GPT-2-small size (151.9 M fp32
params + bf16 shadow), reported as us per call and effective HBM bandwidth (30 B/param)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import hip  # noqa: E402

n = 151_862_784
dev = "cuda"
p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
v.abs_()
sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
sc = torch.tensor([0.0, 1.0], device=dev)
for _ in range(3):
    hip.adamw_flat(p, g, m, v, sh, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1, sc)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(5):
    e0.record()
    for _ in range(10):
        hip.adamw_flat(p, g, m, v, sh, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1, sc)
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
print(f"adamw {best:.1f} us  {30 * n / best / 1e6:.2f} TB/s")
