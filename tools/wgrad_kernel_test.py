"""Hand-written wgrad MFMA kernel vs hipBLASLt (planner) on the model shapes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_llm_trainer_amd.ops import gemm, hip
g = gemm.HipGemm()
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e6
for M in (8192, 32768):
    for name, n, k in [("qkv", 2304, 768), ("o", 768, 768), ("gu", 6144, 768), ("down", 768, 3072), ("lm", 50304, 768)]:
        if name == "lm" and M > 8192: continue
        x = torch.randn(M, k, device="cuda").bfloat16(); dy = torch.randn(M, n, device="cuda").bfloat16()
        dw = torch.zeros(n, k, device="cuda"); dw2 = torch.zeros(n, k, device="cuda")
        hip.wgrad_gemm(dw, dy, x); g.wgrad_acc(dw2, dy, x); torch.cuda.synchronize()
        err = (dw - dw2).abs().max().item() / dw2.abs().max().item()
        res = [f"M={M} {name:5s} rel.err {err:.1e} planner {bench(lambda: g.wgrad_acc(dw2, dy, x)):7.1f}us"]
        for sp in (1, 2, 4, 8, 0):
            t = bench(lambda: hip.wgrad_gemm(dw, dy, x, sp))
            res.append(f"s{sp}:{t:6.1f}({2*M*n*k/t/1e6:.0f}TF)")
        print(" ".join(res), flush=True)
