"""Isolated bf16 vs fp16 timing of the memory-bound kernels (CE, norm fwd / bwd, SwiGLU)
at the headline shapes -- where does --precision fp16 lose against bf16?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import hip, rng  # noqa: E402


def timeit(fn, iters=20):
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


def main():
    dev = "cuda"
    M, H, V, Vp, I = 8192, 768, 50257, 50304, 3072
    torch.manual_seed(0)
    for dt in (torch.bfloat16, torch.float16):
        lg0 = (torch.randn(M, Vp, device=dev) * 2).to(dt)
        tg = torch.randint(0, V, (M,), device=dev)
        nv = (tg != -100).sum()
        lg = lg0.clone()
        t_ce = timeit(lambda: (lg.copy_(lg0), hip.cross_entropy_fwd_bwd(lg, tg, V, nv, 1.0)), 10)
        t_cp = timeit(lambda: lg.copy_(lg0), 10)
        resid = torch.randn(2 * M, H, device=dev)
        delta = torch.randn(2 * M, H, device=dev).to(dt)
        w = torch.ones(H, device=dev)
        key = rng.site_key(1, 0, 0, rng.SITE_RESID)
        t_nf = timeit(lambda: hip.add_dropout_rmsnorm_fwd(resid, delta, w, 1e-5, 0.1, key, out_dtype=dt))
        gu = torch.randn(2 * M, 2 * I, device=dev).to(dt)
        t_sw = timeit(lambda: hip.swiglu_fwd(gu))
        da = torch.randn(2 * M, I, device=dev).to(dt)
        t_sb = timeit(lambda: hip.swiglu_bwd(gu, da))
        print(f"{str(dt):15s} CE {t_ce - t_cp:7.1f} us (8192 rows)  norm fwd {t_nf:6.1f} us  swiglu fwd {t_sw:6.1f} us"
              f"  swiglu bwd {t_sb:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
