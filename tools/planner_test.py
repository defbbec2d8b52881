"""Planner vs torch on the model's GEMM shapes (random data)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_llm_trainer_amd.ops import gemm
g = gemm.HipGemm()
M = 8192
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e6
for name, n, k in [("qkv", 2304, 768), ("o", 768, 768), ("gu", 6144, 768), ("down", 768, 3072)]:
    x = torch.randn(M, k, device="cuda").bfloat16(); w = torch.randn(n, k, device="cuda").bfloat16()
    dy = torch.randn(M, n, device="cuda").bfloat16(); dw = torch.zeros(n, k, device="cuda")
    a = bench(lambda: g.wgrad_acc(dw, dy, x)); b = bench(lambda: torch.addmm(dw, dy.t(), x, out_dtype=torch.float32, out=dw))
    c = bench(lambda: g.linear(x, w)); d = bench(lambda: torch.matmul(x, w.t()))
    e = bench(lambda: g.linear_dgrad(dy, w)); f = bench(lambda: torch.matmul(dy, w))
    print(f"{name:5s} wgrad planner {a:6.1f} torch {b:6.1f} | fwd planner {c:6.1f} torch {d:6.1f} | dgrad planner {e:6.1f} torch {f:6.1f}")
print(gemm.report())
