"""Time every GEMM role of one GPT-2-small optimizer step through the engine's GEMM
backend (hipBLASLt planner) and report TF/s; plus a large square bf16 GEMM as the
achievable-peak reference.  usage: python tools/gemm_roles.py [M=8192] [GA=4]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import gemm  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
GA = int(sys.argv[2]) if len(sys.argv) > 2 else 4
H, I, V, L = 768, 3072, 50304, 12
g = gemm.HipGemm()
dev = "cuda"


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


def r(*s):
    return torch.randn(*s, device=dev).bfloat16()


rows = []
total_us = 0.0
for name, n, k in [("qkv", 3 * H, H), ("o", H, H), ("gu", 2 * I, H), ("down", H, I), ("lm_head", V, H)]:
    per = 1 if name == "lm_head" else L
    x, w, dy = r(M, k), r(n, k), r(M, n)
    xw, dyw = r(GA * M, k), r(GA * M, n)
    dw = torch.zeros(n, k, device=dev)
    f = bench(lambda: g.linear(x, w))
    d = bench(lambda: g.linear_dgrad(dy, w))
    if name == "lm_head":  # not deferred (tied embedding grad needs it every micro-step)
        wg = bench(lambda: g.wgrad_acc(dw, dy, x))
        wg_step = wg * GA
    else:
        wg = bench(lambda: g.wgrad_acc(dw, dyw, xw))
        wg_step = wg
    fl = 2.0 * M * n * k
    step_us = per * (GA * (f + d) + wg_step)
    total_us += step_us
    rows.append((name, f, fl / f / 1e6, d, fl / d / 1e6, wg, (fl * (1 if name == "lm_head" else GA)) / wg / 1e6,
                 step_us / 1e3))
print(f"M={M} GA={GA}")
print("| role | fwd us | TF/s | dgrad us | TF/s | wgrad us | TF/s | ms/step |")
print("|---|---:|---:|---:|---:|---:|---:|---:|")
for row in rows:
    print("| {} | {:.1f} | {:.0f} | {:.1f} | {:.0f} | {:.1f} | {:.0f} | {:.2f} |".format(*row))
print(f"total GEMM time per optimizer step: {total_us / 1e3:.2f} ms")
a, b = r(8192, 8192), r(8192, 8192)
t = bench(lambda: torch.matmul(a, b), it=10)
print(f"square 8192^3 torch.matmul: {t:.0f} us = {2 * 8192 ** 3 / t / 1e6:.0f} TF/s")
print(gemm.report())
print(g.report_choices())
