"""Isolated timing of the bf16 memory-bound kernels at the small (H 768, I 3072) and medium
(H 1024, I 4096) shapes, 16384 rows: achieved bytes/s per kernel, to tell a kernel that
degrades with H from one that only looks slow in the overlapped step trace."""
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
    M = 16384
    torch.manual_seed(0)
    for H, I in ((768, 3072), (1024, 4096), (1280, 5120), (1600, 6400)):
        resid = torch.randn(M, H, device=dev)
        delta = torch.randn(M, H, device=dev).bfloat16()
        w = torch.ones(H, device=dev)
        key = rng.site_key(1, 0, 0, rng.SITE_RESID)
        t_nf = timeit(lambda: hip.add_dropout_rmsnorm_fwd(resid, delta, w, 1e-5, 0.1, key))
        x, y, rstd = hip.add_dropout_rmsnorm_fwd(resid, delta, w, 1e-5, 0.1, key)
        dy = torch.randn(M, H, device=dev).bfloat16()
        dres = torch.randn(M, H, device=dev)
        dw = torch.zeros(H, device=dev)
        t_nb = timeit(lambda: hip.rmsnorm_bwd(dy, x, rstd, w, dres, dw, 0.1, key))
        gu = torch.randn(M, 2 * I, device=dev).bfloat16()
        da = torch.randn(M, I, device=dev).bfloat16()
        t_sb = timeit(lambda: hip.swiglu_bwd(gu, da))
        t_sf = timeit(lambda: hip.swiglu_fwd(gu))
        # bytes: fwd resid f32 + delta bf16 in, x f32 + y bf16 out; bwd dy bf16 + x f32 + dres f32 in,
        # dx f32 + ddelta bf16 out; swiglu bwd gu + da in, dgu out (bf16); fwd gu in, s out
        bnf, bnb = M * H * 12, M * H * 16
        bsb, bsf = M * I * 2 * 5, M * I * 2 * 3
        print(f"H {H:5d} I {I:5d}: norm fwd {t_nf:6.1f} us {bnf / t_nf / 1e6:5.2f} TB/s | norm bwd {t_nb:6.1f} us "
              f"{bnb / t_nb / 1e6:5.2f} TB/s | swiglu bwd {t_sb:6.1f} us {bsb / t_sb / 1e6:5.2f} TB/s | "
              f"swiglu fwd {t_sf:6.1f} us {bsf / t_sf / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
