"""8-phase 256x256 TN GEMM (ops/csrc/gemm_tn8.hip) vs the hipBLASLt planner and the
older 2-barrier TN kernel: correctness vs fp32 torch and time on the model's shapes."""
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
    best = 1e30
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / it * 1e6)
    return best


M = int(os.environ.get("M", "8192"))  # rows of the projection GEMMs (micro-step chain tokens)
shapes = [("qkv fwd", M, 2304, 768), ("gu fwd", M, 6144, 768), ("down fwd", M, 768, 3072),
          ("o fwd", M, 768, 768), ("lm_head fwd*", M, 50176, 768), ("down dgrad", M, 3072, 768),
          ("qkv dgrad*", M, 768, 2304), ("gu dgrad*", M, 768, 6144),
          ("square 4096", 4096, 4096, 4096), ("square 8192", 8192, 8192, 8192)]
only = sys.argv[1:] if len(sys.argv) > 1 else None
for name, m, n, k in shapes:
    torch.manual_seed(0)
    a = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(n, k, device="cuda") * 2 - 1).bfloat16()
    ref = a.float() @ b.float().t()
    fl = 2.0 * m * n * k
    y = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    t_lib = bench(lambda: g._lib_linear(a, b, y))
    line = f"{name:13s} M={m} N={n} K={k}: hipBLASLt {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)"
    for cfg in (1, 5):
        c = hip.gemm_tn(a, b, cfg)
        if c is None:
            continue
        torch.cuda.synchronize()
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        t = bench(lambda: hip.gemm_tn(a, b, cfg, out=c))
        line += f" | cfg{cfg} {t:7.1f} us ({fl / t / 1e6:5.0f} TF, err {err:.1e})"
    print(line, flush=True)
