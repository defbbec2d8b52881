"""Hand-written TN GEMM (ops/csrc/gemm_tn.hip) vs the hipBLASLt planner on the model's
forward / data-gradient shapes: correctness vs fp32 torch and time per tile config."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import gemm, hip  # noqa: E402

g = gemm.HipGemm()


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


M = 8192
shapes = [("qkv fwd", 2304, 768), ("o fwd / o dgrad", 768, 768), ("gu fwd", 6144, 768), ("down fwd", 768, 3072),
          ("qkv dgrad", 768, 2304), ("gu dgrad", 768, 6144), ("down dgrad", 3072, 768), ("square 8192", 8192, 8192)]
for name, n, k in shapes:
    m = 8192
    a = torch.randn(m, k, device="cuda").bfloat16()
    b = torch.randn(n, k, device="cuda").bfloat16()
    ref = a.float() @ b.float().t()
    fl = 2.0 * m * n * k
    t_lib = bench(lambda: g.linear(a, b))
    line = f"{name:16s} M={m} N={n} K={k}: hipBLASLt {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)"
    for cfg in hip.GEMM_TN_TILES:
        c = hip.gemm_tn(a, b, cfg)
        if c is None:
            continue
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        t = bench(lambda: hip.gemm_tn(a, b, cfg, out=c))
        line += f" | cfg{cfg} {t:7.1f} us ({fl / t / 1e6:5.0f} TF, err {err:.1e})"
    print(line, flush=True)
