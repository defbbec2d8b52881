"""Does the weight-gradient GEMM run faster with the reduction dim (tokens) contiguous?
Compares dW[N,K] += dY[M,N]^T X[M,K] in the engine's layout (both operands M-major)
against the same product with pre-transposed operands (dYt[N,M], Xt[K,M]), through the
hipBLASLt planner and torch.matmul.  M = GA x B x S = 32768."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import gemm  # noqa: E402

g = gemm.HipGemm()
M = 32768


def bench(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


for name, n, k in [("qkv", 2304, 768), ("o", 768, 768), ("gu", 6144, 768), ("down", 768, 3072)]:
    x = torch.randn(M, k, device="cuda").bfloat16()
    dy = torch.randn(M, n, device="cuda").bfloat16()
    dw = torch.zeros(n, k, device="cuda")
    xt, dyt = x.t().contiguous(), dy.t().contiguous()
    a = bench(lambda: g.wgrad_acc(dw, dy, x))
    # transposed operands: C[N,K] (row-major) = dyt[N,M] @ xt[K,M]^T ; col-major: C^T[K,N] = xt^T... via planner
    b = bench(lambda: gemm._gemm(1, 0, k, n, M, xt, M, dyt, M, dw, k, 1.0, 1.0))
    c = bench(lambda: torch.matmul(dyt, xt.t()))
    tr = bench(lambda: x.t().contiguous())
    fl = 2.0 * M * n * k
    print(f"{name:5s} engine-layout {a:7.1f} us ({fl / a / 1e6:5.0f} TF) | tokens-contiguous planner {b:7.1f} us "
          f"({fl / b / 1e6:5.0f} TF) torch {c:7.1f} us | transpose of X {tr:6.1f} us")
