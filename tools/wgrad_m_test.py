"""wgrad cost per 8192 rows when the reduction is batched over GA micro-steps."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_llm_trainer_amd.ops import gemm
g = gemm.HipGemm()
def bench(fn, it=10):
    for _ in range(2): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e6
tot = {}
for M in (8192, 16384, 32768):
    s = 0
    for name, n, k in [("qkv", 2304, 768), ("o", 768, 768), ("gu", 6144, 768), ("down", 768, 3072)]:
        x = torch.randn(M, k, device="cuda").bfloat16(); dy = torch.randn(M, n, device="cuda").bfloat16()
        dw = torch.zeros(n, k, device="cuda")
        a = bench(lambda: g.wgrad_acc(dw, dy, x))
        s += a * 8192 / M
        print(f"M={M} {name:5s} {a:7.1f} us  ({2*M*n*k/a/1e6:.0f} TF)  per-8192-rows {a*8192/M:6.1f}")
    print(f"M={M}: per-layer wgrad cost per 8192 rows = {s:.1f} us")
