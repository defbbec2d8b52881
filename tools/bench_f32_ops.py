"""Isolated timing of the fp32-mode kernels (csrc/fp32.hip) at the fp32 bench step's
shapes (16 x 1024 tokens per chain, gpt2_small): achieved bytes/s per kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import hip, hip_f32, rng  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def row(name, us, nbytes):
    print(f"{name:28s} {us:9.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)


def main():
    dev = "cuda"
    B, S, nh, hd, I, V, Vp = 16, 1024, 12, 64, 3072, 50257, 50304
    H, M = nh * hd, B * S
    torch.manual_seed(0)
    resid = torch.randn(M, H, device=dev)
    delta = torch.randn(M, H, device=dev)
    w = torch.ones(H, device=dev)
    key = rng.site_key(1, 0, 0, rng.SITE_RESID)
    row("norm fwd", timeit(lambda: hip.add_dropout_rmsnorm_fwd(resid, delta, w, 1e-5, 0.1, key, out_dtype=torch.float32)), M * H * 16)
    x, y, rstd = hip.add_dropout_rmsnorm_fwd(resid, delta, w, 1e-5, 0.1, key, out_dtype=torch.float32)
    dy, dres, dw = torch.randn(M, H, device=dev), torch.randn(M, H, device=dev), torch.zeros(H, device=dev)
    row("norm bwd (+colsum)", timeit(lambda: hip.rmsnorm_bwd(dy, x, rstd, w, dres, dw, 0.1, key)), M * H * 20)
    gu, da = torch.randn(M, 2 * I, device=dev), torch.randn(M, I, device=dev)
    row("swiglu fwd", timeit(lambda: hip.swiglu_fwd(gu)), M * I * 12)
    row("swiglu bwd", timeit(lambda: hip.swiglu_bwd(gu, da)), M * I * 20)
    qkv = torch.randn(M, 3 * H, device=dev)
    cos, sin = hip.rope_tables(hd, S, device=dev)
    row("rope qk in place", timeit(lambda: hip.rope_qk_inplace(qkv, B, S, nh, cos, sin)), M * 2 * H * 8)
    src = hip_f32._packed_ptrs(qkv, 3, H)
    row("relayout packed->heads x3", timeit(lambda: hip_f32._relayout(src, (S * 3 * H, 3 * H, hd), B, S, nh, hd, qkv.device)),
        M * 3 * H * 8)
    sc = torch.randn(B * nh * S, S, device=dev)
    lse = torch.empty(B * nh * S, device=dev)
    mask = hip.attention_dropout_mask(B, nh, S, 0.1, 7, device=dev)
    L = hip_f32._lib()
    row("attn softmax", timeit(lambda: L.dlt_f32_attn_softmax(hip_f32._p(sc), hip_f32._p(lse), hip_f32._p(mask), B * nh, S,
                                                              0.125, 1 / 0.9, 0, hip_f32._st())), sc.numel() * 8)
    dp = torch.randn_like(sc)
    o, do = torch.randn(M, H, device=dev), torch.randn(M, H, device=dev)
    row("attn dsoftmax", timeit(lambda: L.dlt_f32_attn_dsoftmax(hip_f32._p(sc), hip_f32._p(dp), hip_f32._p(lse),
                                                                hip_f32._p(o), hip_f32._p(do), hip_f32._p(mask), B, nh, S,
                                                                hd, 0.125, 1 / 0.9, 0, hip_f32._st())), sc.numel() * 16)
    q4 = torch.randn(B, nh, S, hd, device=dev)
    row("bmm q.k^T (B*nh x S x S x hd)", timeit(lambda: torch.matmul(q4, q4.transpose(-1, -2))),
        2 * B * nh * S * S * hd / 1e3 * 1e6 / 1e6)  # "TB/s" column = TFLOP/s here
    pm = torch.randn(B, nh, S, S, device=dev)
    row("bmm p.v", timeit(lambda: torch.matmul(pm, q4)), 2 * B * nh * S * S * hd / 1e3)
    lg0 = torch.randn(M, Vp, device=dev)
    lg = lg0.clone()
    tg = torch.randint(0, V, (M,), device=dev)
    nv = (tg != -100).sum()
    t_ce = timeit(lambda: (lg.copy_(lg0), hip.cross_entropy_fwd_bwd(lg, tg, V, nv, 1.0)), 5)
    t_cp = timeit(lambda: lg.copy_(lg0), 5)
    row("cross entropy", t_ce - t_cp, M * Vp * 12)


if __name__ == "__main__":
    main()
