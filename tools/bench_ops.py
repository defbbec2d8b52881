"""Isolated timing of the memory-bound HIP ops at the headline shapes (GPT-2 small,
B=8, S=1024 -> M=8192 rows; B=16 env for the fused chain), with the effective HBM
bandwidth of each.

usage: [B=16] python tools/bench_ops.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import hip, rng  # noqa: E402

dev = "cuda"
B = int(os.environ.get("B", "8"))  # sequences per chain (B=16: the fused micro-step chain)
S, H, nh, I, V = 1024, 768, 12, 3072, 50304
M = B * S


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


rows = []


def rec(name, us, nbytes):
    rows.append((name, us, nbytes / us / 1e3))


x = torch.randn(M, H, device=dev)
d = torch.randn(M, H, device=dev).bfloat16()
w = torch.ones(H, device=dev)
key = rng.site_key(1, 2, 3, rng.SITE_RESID)
rec("rmsnorm fwd (add+dropout)", timeit(lambda: hip.add_dropout_rmsnorm_fwd(x, d, w, 1e-6, 0.1, key)),
    M * H * (4 + 2 + 4 + 2))
xo, y, rstd = hip.add_dropout_rmsnorm_fwd(x, d, w, 1e-6, 0.1, key)
dres = torch.randn(M, H, device=dev)
dw = torch.zeros(H, device=dev)
rec("rmsnorm bwd (+dres, ddelta)", timeit(lambda: hip.rmsnorm_bwd(y, xo, rstd, w, dres, dw, 0.1, key)),
    M * H * (2 + 4 + 4 + 4 + 2))
gu = torch.randn(M, 2 * I, device=dev).bfloat16()
rec("swiglu fwd", timeit(lambda: hip.swiglu_fwd(gu)), M * I * (4 + 2))
da = torch.randn(M, I, device=dev).bfloat16()
rec("swiglu bwd", timeit(lambda: hip.swiglu_bwd(gu, da)), M * I * (4 + 2 + 4))
qkv = torch.randn(M, 3 * H, device=dev).bfloat16()
cos, sin = hip.rope_tables(64, S, device=dev)
rec("rope fwd", timeit(lambda: hip.rope_qkv_fwd(qkv, B, S, nh, cos, sin)), M * 3 * H * 4)
q, k, v = hip.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
rec("rope bwd", timeit(lambda: hip.rope_qkv_bwd(q, k, v, cos, sin)), M * 3 * H * 4)
logits = torch.randn(M, V, device=dev).bfloat16()
tg = torch.randint(0, 50257, (M,), device=dev)
nv = torch.tensor([M], device=dev)
rec("cross-entropy fwd+bwd", timeit(lambda: hip.cross_entropy_fwd_bwd(logits, tg, 50257, nv), 10), M * V * 4)
ids = torch.randint(0, 50257, (M,), device=dev)
emb = torch.randn(V, H, device=dev)
rec("embedding fwd", timeit(lambda: hip.embedding_fwd(ids, emb)), M * H * 8)
dout = torch.randn(M, H, device=dev)
demb = torch.zeros(V, H, device=dev)
rec("embedding bwd (sort + segment-sum, uniform ids)", timeit(lambda: hip.embedding_bwd(ids, dout, demb)),
    M * H * 12)
zipf = torch.minimum((torch.rand(M, device=dev) ** 4 * 50257).long(), torch.tensor(50256, device=dev))
rec("embedding bwd (sort + segment-sum, zipf-like ids)", timeit(lambda: hip.embedding_bwd(zipf, dout, demb)),
    M * H * 12)
rec("torch.sort of the ids (part of the above)", timeit(lambda: torch.sort(ids, stable=True)), M * 16)
P = 151_862_784
p_, g_, m_, v_ = (torch.zeros(P, device=dev) for _ in range(4))
sh = torch.zeros(P, device=dev, dtype=torch.bfloat16)
gs = torch.ones(2, device=dev)
rec("adamw (flat, 152M)", timeit(lambda: hip.adamw_flat(p_, g_, m_, v_, sh, 1e-3, 0.9, 0.95, 1e-8, 0.1, 1, gs), 10),
    P * (4 * 4 + 3 * 4 + 2))
out = torch.zeros(2, device=dev)
rec("grad sumsq (152M)", timeit(lambda: hip.sumsq(g_, out), 10), P * 4)
big = torch.empty(M * H * 16, device=dev)
big2 = torch.empty_like(big)
rec("reference: torch copy_ (805 MB)", timeit(lambda: big2.copy_(big), 10), big.numel() * 8)
print("| op | us | GB/s |")
print("|---|---:|---:|")
for n, us, bw in rows:
    print(f"| {n} | {us:.1f} | {bw:.0f} |")
