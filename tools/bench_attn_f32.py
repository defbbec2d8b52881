"""fp32 attention at the fused-chain shape: the HIP VALU flash kernels (ops/hip_f32.py)
vs the PyTorch reference ops (ops/reference.py: matmul + softmax on the GPU, what the fp32
mode ran before round 5).  Packed QKV, causal, dropout p.  usage:
python tools/bench_attn_f32.py [--B 16] [--nh 12] [--S 1024] [--hd 64] [--p 0.1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from distributed_llm_trainer_amd.ops import hip, hip_f32, reference as ref, rng  # noqa: E402


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--nh", type=int, default=12)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--hd", type=int, default=64)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    B, nh, S, hd, p = a.B, a.nh, a.S, a.hd, a.p
    H = nh * hd
    torch.manual_seed(0)
    qkv = torch.randn(B * S, 3 * H, device="cuda")
    do = torch.randn(B * S, H, device="cuda")
    cos, sin = hip.rope_tables(hd, S, device="cuda")
    key = rng.site_key(1, 2, 3, rng.SITE_ATTN)
    o, aux = hip_f32.attention_fwd_packed(qkv, B, S, nh, p, key)
    t_hf = timed(lambda: hip_f32.attention_fwd_packed(qkv, B, S, nh, p, key, mask=aux[1]))
    t_hb = timed(lambda: hip_f32.attention_bwd_packed(qkv, o, do, aux, p, key, B, S, nh, cos, sin))
    o2, lse2 = ref.attention_fwd_packed(qkv, B, S, nh, p, key)
    t_rf = timed(lambda: ref.attention_fwd_packed(qkv, B, S, nh, p, key))
    t_rb = timed(lambda: ref.attention_bwd_packed(qkv, o2, do, lse2, p, key, B, S, nh, cos, sin))
    print(f"B{B} nh{nh} S{S} hd{hd} p{p}: HIP fp32 fwd {t_hf:.2f} ms bwd {t_hb:.2f} ms | "
          f"PyTorch ops fwd {t_rf:.2f} ms bwd {t_rb:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
