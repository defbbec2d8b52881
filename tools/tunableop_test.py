"""Compare hipBLASLt default heuristics vs TunableOp-tuned GEMMs on the model's shapes."""
import os, sys, time
import torch
M = 8192
shapes = [  # (name, M, N, K) for y = x @ W^T  and the dgrad/wgrad variants
    ("qkv", M, 2304, 768), ("o", M, 768, 768), ("gu", M, 6144, 768), ("down", M, 768, 3072), ("lm", M, 50304, 768)]
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/it*1e6
tot = 0
for name, m, n, k in shapes:
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16); w = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(m, n, device="cuda", dtype=torch.bfloat16); dw = torch.zeros(n, k, device="cuda")
    tf = bench(lambda: torch.matmul(x, w.t())); td = bench(lambda: torch.matmul(dy, w))
    tw = bench(lambda: torch.addmm(dw, dy.t(), x, out_dtype=torch.float32, out=dw))
    fl = 2*m*n*k
    tot += tf+td+tw
    print(f"{name:5s} fwd {tf:7.1f}us {fl/tf/1e6:6.0f}TF  dgrad {td:7.1f}us {fl/td/1e6:6.0f}TF  wgrad(fp32 acc) {tw:7.1f}us {fl/tw/1e6:6.0f}TF")
print("total us", tot)
