"""Isolated timing of the forward projection GEMMs at the headline chain shape (M = 16384):
hipBLASLt (the planner's library path) vs the persistent hand kernel (k_gemm_bf16) vs the
one-tile-per-workgroup 256 x 128 kernel (k_gemm_fwd).  Mean of --iters launches after
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
    args = ap.parse_args()
    g = gemm.HipGemm()
    for name, (M, N, K) in SHAPES.items():
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        row = [f"{name:8s} {M}x{N}x{K}:"]
        for label, fn in (("lib", lambda: g._lib_linear(a, b, y)),
                          ("bf16", (lambda: hip.gemm_bf16(a, b, out=y)) if hip.gemm_bf16_fits(M, N, K) else None),
                          ("fwd", lambda: hip.gemm_fwd(a, b, out=y))):
            if fn is None:
                row.append(f"{label} -")
                continue
            us = timed(fn, args.iters)
            row.append(f"{label} {us:7.1f} us {flops / us / 1e6:6.0f} TF")
        ref = (a.float() @ b.float().t())
        hip.gemm_fwd(a, b, out=y)
        err = ((y.float() - ref).norm() / ref.norm()).item()
        print(" | ".join(row) + f" | fwd relerr {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
