"""Isolated timing of the forward projection GEMMs at the headline chain shape (M = 16384):
hipBLASLt (the planner's library path) vs the persistent hand kernel (k_gemm_bf16) vs the
one-tile-per-workgroup k_gemm_fw4 (4-wave, 128 x 128 per wave) in its launch variants.  Mean of --iters launches after
warmup, CUDA events.  usage: python tools/bench_gemm_fwd.py [--iters 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from distributed_llm_trainer_amd.ops import gemm, hip  # noqa: E402

SHAPES = {"qkv": (16384, 2304, 768), "o": (16384, 768, 768), "gate/up": (16384, 6144, 768),
          "down": (16384, 768, 3072), "lm_head": (16384, 50304, 768)}


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default=",".join(SHAPES), help="comma list of SHAPES keys")
    ap.add_argument("--impls", default="lib,bf16,fw4", help="comma list of lib / bf16 / fw4 / fw4<variant>")
    ap.add_argument("--dgrad", action="store_true",
                    help="data-gradient shapes dX = dY @ W: the persistent reduction-major kernel (hip.gemm_dgrad), "
                         "hipBLASLt, and k_gemm_fw4 on a transposed weight copy (TN form)")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic: per-workgroup timestamps of k_gemm_fw4 (SCHED 1) on each shape")
    args = ap.parse_args()
    impls = args.impls.split(",")
    if args.dgrad:
        return dgrad(args)
    g = gemm.HipGemm()
    for name in args.shapes.split(","):
        M, N, K = SHAPES[name]
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        row = [f"{name:8s} {M}x{N}x{K}:"]
        for label, fn in (("lib", lambda: g._lib_linear(a, b, y)),
                          ("bf16", (lambda: hip.gemm_bf16(a, b, out=y)) if hip.gemm_bf16_fits(M, N, K) else None),
                          ("fw4", lambda: hip.gemm_fw4(a, b, out=y)),
                          ("fw4p", lambda: hip.gemm_fw4(a, b, out=y, flags=0)),
                          ("fw4nt", lambda: hip.gemm_fw4(a, b, out=y, flags=4)),
                          ("fw4rm", lambda: hip.gemm_fw4(a, b, out=y, flags=150)),
                          ("fw4h", lambda: hip.gemm_fw4(a, b, out=y, flags=148 | 2048)),
                          ("fw4x2", lambda: hip.gemm_fw4(a, b, out=y, flags=4 | 4096)),
                          ("fw4s5x2", lambda: hip.gemm_fw4(a, b, out=y, flags=148 | 4096)),
                          ("fw4hx2", lambda: hip.gemm_fw4(a, b, out=y, flags=148 | 2048 | 4096)),
                          ("fw4px2", lambda: hip.gemm_fw4(a, b, out=y, flags=144 | 4096))):
            if label not in impls:
                continue
            if fn is None:
                row.append(f"{label} -")
                continue
            us = timed(fn, args.iters)
            row.append(f"{label} {us:7.1f} us {flops / us / 1e6:6.0f} TF")
        ref = (a.float() @ b.float().t())
        errs = []
        for label, fn in (("fw4", hip.gemm_fw4),
                          ("fw4x2", lambda a, b, out: hip.gemm_fw4(a, b, out=out, flags=4 | 4096))):
            if label not in impls:
                continue
            y.fill_(float("nan"))
            fn(a, b, out=y)
            errs.append(f"{label} relerr {((y.float() - ref).norm() / ref.norm()).item():.1e}")
        print(" | ".join(row + errs), flush=True)


DGRAD = {"dqkv": (16384, 768, 2304), "do": (16384, 768, 768), "dgu": (16384, 768, 6144),
         "dlm": (8192, 768, 50304), "dlm16": (16384, 768, 50304), "ddown": (16384, 3072, 768)}


def dgrad(args):
    """dX[M, N] = dY[M, K] @ W[K, N]: hand persistent NN kernel vs library vs fw4 on W^T."""
    g = gemm.HipGemm()
    for name, (M, N, K) in DGRAD.items():
        dy = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(K, N, device="cuda").bfloat16()
        wt = w.t().contiguous()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        row = [f"{name:6s} {M}x{N}x{K}:"]
        for label, fn in (("hand", lambda: hip.gemm_dgrad(dy, w, out=y)),
                          ("lib", lambda: g._lib_dgrad(dy, w, y)),
                          ("fw4", lambda: hip.gemm_fw4(dy, wt, out=y, flags=148)),
                          ("fw4b", lambda: hip.gemm_fw4(dy, wt, out=y, flags=4)),
                          ("fw4h", lambda: hip.gemm_fw4(dy, wt, out=y, flags=148 | 2048))):
            us = timed(fn, args.iters)
            row.append(f"{label} {us:7.1f} us {flops / us / 1e6:5.0f} TF")
        ref = dy.float() @ w.float()
        hip.gemm_fw4(dy, wt, out=y, flags=148)
        row.append(f"fw4 relerr {((y.float() - ref).norm() / ref.norm()).item():.1e}")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
