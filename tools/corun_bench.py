"""Co-run behaviour of the forward projection GEMMs (one MI355X).

In the two-chain training window a GEMM of one chain runs beside the memory-bound
kernels (norms, SwiGLU, RoPE, cross-entropy, AdamW) of the other.  What matters there is
not the GEMM's time alone but how the pair shares the GPU.  For each GEMM backend this
launches the GEMM on stream A and a train of memory-bound copies on stream B at the same
moment and reports: each alone, both together (wall from the common start to the later
end), each stream's own span inside the co-run, and the co-run gain
(alone_gemm + alone_mem) / together (1 = no overlap, 2 = perfect).

usage: python tools/corun_bench.py [--roles gate/up,lm_head] [--copies 8] [--mb 256]
       env DLT_GEMM_FWD_FLAGS / DLT_GEMM_GRID select the hand kernel's launch mode.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from distributed_llm_trainer_amd.ops import gemm, hip  # noqa: E402

SHAPES = {"qkv": (16384, 2304, 768), "o": (16384, 768, 768), "gate/up": (16384, 6144, 768),
          "down": (16384, 768, 3072), "lm_head": (16384, 50304, 768)}


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--roles", default="o,gate/up,down,lm_head")
    ap.add_argument("--copies", type=int, default=8)
    ap.add_argument("--mb", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--backends", default="lib,hand")
    args = ap.parse_args()
    g = gemm.HipGemm()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    n = args.mb * (1 << 20) // 2
    src = torch.randn(n, device="cuda").bfloat16()
    dst = torch.empty_like(src)
    for role in args.roles.split(","):
        M, N, K = SHAPES[role]
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = torch.randn(N, K, device="cuda").bfloat16()
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {"lib": lambda: g._lib_linear(a, b, y), "hand": lambda: hip.gemm_bf16(a, b, out=y),
               "fwd": lambda: hip.gemm_fwd(a, b, out=y)}
        reps = max(1, int(1500 / (2 * M * N * K / 1e12)))  # ~1.5 ms of GEMM per sample
        reps = min(reps, 64)

        def gemm_run():
            for _ in range(reps):
                fns[name]()

        def mem_run():
            for _ in range(args.copies):
                dst.copy_(src)
        for name in args.backends.split(","):
            if name == "hand" and not hip.gemm_bf16_fits(M, N, K):
                continue
            res = []
            for _ in range(args.reps):
                # alone
                torch.cuda.synchronize()
                e = [ev() for _ in range(6)]
                with torch.cuda.stream(sa):
                    e[0].record()
                    gemm_run()
                    e[1].record()
                torch.cuda.synchronize()
                with torch.cuda.stream(sb):
                    e[2].record()
                    mem_run()
                    e[3].record()
                torch.cuda.synchronize()
                t_g, t_m = e[0].elapsed_time(e[1]), e[2].elapsed_time(e[3])
                # together: both streams wait for one start event
                start = ev()
                start.record()
                sa.wait_event(start)
                sb.wait_event(start)
                ea, eb = ev(), ev()
                with torch.cuda.stream(sa):
                    gemm_run()
                    ea.record()
                with torch.cuda.stream(sb):
                    mem_run()
                    eb.record()
                torch.cuda.synchronize()
                ta, tb = start.elapsed_time(ea), start.elapsed_time(eb)
                res.append((t_g, t_m, max(ta, tb), ta, tb))
            res.sort(key=lambda r: r[2])
            t_g, t_m, tt, ta, tb = res[len(res) // 2]
            print(f"{role:8s} {name:5s} x{reps:<3d} gemm alone {t_g:7.3f} ms  mem alone {t_m:7.3f} ms | together "
                  f"{tt:7.3f} ms (gemm {ta:7.3f}, mem {tb:7.3f}) gain {(t_g + t_m) / tt:5.3f}", flush=True)


if __name__ == "__main__":
    main()
