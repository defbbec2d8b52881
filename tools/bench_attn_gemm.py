"""Attention for a head_dim without a flash kernel (default: bf16, head_dim 96, B16 nh8
S1024): fwd + bwd time of the zero-padded flash route, the 16-bit GEMM route, the
fp32-widened route and the PyTorch reference ops, with the head_dim-64 flash kernels at the same FLOPs per token for scale."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import attn_gemm, hip, reference  # noqa: E402


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--nh", type=int, default=8)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--hd", type=int, default=96)
    a = ap.parse_args()
    B, nh, S, hd = a.B, a.nh, a.S, a.hd
    H = nh * hd
    torch.manual_seed(0)
    qkv = (torch.randn(B * S, 3 * H, device="cuda") * 0.5).bfloat16()
    cos, sin = hip.rope_tables(hd, S, device="cuda")
    do = torch.randn(B * S, H, device="cuda").bfloat16()

    def step(mod):
        o, aux = mod.attention_fwd_packed(qkv, B, S, nh, 0.1, 5)
        mod.attention_bwd_packed(qkv, o, do, aux, 0.1, 5, B, S, nh, cos, sin)
    fl = 4 * B * nh * S * S / 2 * hd * 3.5  # causal fwd + bwd (2.5x) FLOPs
    tpad = timeit(lambda: step(attn_gemm))
    attn_gemm.PAD_FLASH = False
    t16 = timeit(lambda: step(attn_gemm))
    use16 = attn_gemm.use16
    attn_gemm.use16 = lambda *x: False
    t32 = timeit(lambda: step(attn_gemm))
    attn_gemm.use16 = use16
    tref = timeit(lambda: step(reference), 3)
    print(f"hd {hd}: zero-padded flash {tpad:8.1f} us ({fl / tpad / 1e6:6.1f} TF/s)  "
          f"16-bit GEMMs {t16:8.1f} us ({fl / t16 / 1e6:6.1f} TF/s)  fp32-widened {t32:8.1f} us  "
          f"reference ops {tref:8.1f} us", flush=True)
    nh64 = H // 64
    q64 = (torch.randn(B * S, 3 * nh64 * 64, device="cuda") * 0.5).bfloat16()
    c64, s64 = hip.rope_tables(64, S, device="cuda")

    def flash():
        o, aux = hip.attention_fwd_packed(q64, B, S, nh64, 0.1, 5)
        hip.attention_bwd_packed(q64, o, do[:, :nh64 * 64].contiguous(), aux, 0.1, 5, B, S, nh64, c64, s64)
    tf = timeit(flash)
    print(f"flash head_dim 64 x {nh64} heads (same H): {tf:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
