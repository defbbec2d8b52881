"""Micro-benchmark of the attention kernels at the headline shape (B8 nh12 S1024 hd64)."""
import argparse
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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--nh", type=int, default=12)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--packed", action="store_true", help="attention on the packed [B*S, 3H] QKV (engine default)")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16"))
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    torch.manual_seed(0)
    q, k, v = (torch.randn(a.B, a.nh, a.S, 64, device="cuda").to(dt) for _ in range(3))
    key = rng.site_key(1, 2, 3, rng.SITE_ATTN)
    if a.packed:
        qkv = torch.randn(a.B * a.S, 3 * a.nh * 64, device="cuda").to(dt)
        cos, sin = hip.rope_tables(64, a.S, device="cuda")
        o, aux = hip.attention_fwd_packed(qkv, a.B, a.S, a.nh, a.p, key)
        do = torch.randn_like(o)
        t_f = timeit(lambda: hip.attention_fwd_packed(qkv, a.B, a.S, a.nh, a.p, key), a.iters)
        t_b = timeit(lambda: hip.attention_bwd_packed(qkv, o, do, aux, a.p, key, a.B, a.S, a.nh, cos, sin), a.iters)
        if a.p > 0:  # the forward kernel alone (keep bits already generated) -> bits kernel time
            m = aux[1]
            if m is not None:
                t_k = timeit(lambda: hip.attention_fwd_packed(qkv, a.B, a.S, a.nh, a.p, key, mask=m), a.iters)
                print(f"fwd kernel {t_k:.1f} us, keep-bit kernel {t_f - t_k:.1f} us")
    else:
        o, aux = hip.attention_fwd(q, k, v, a.p, key)
        do = torch.randn_like(o)
        t_f = timeit(lambda: hip.attention_fwd(q, k, v, a.p, key), a.iters)
        t_b = timeit(lambda: hip.attention_bwd(q, k, v, o, do, aux, a.p, key), a.iters)
    fl = 4 * a.B * a.nh * a.S * a.S / 2 * 64
    print(f"fwd {t_f:.1f} us ({fl / t_f / 1e6:.1f} TF/s)  bwd {t_b:.1f} us ({2.5 * fl / t_b / 1e6:.1f} TF/s)")


if __name__ == "__main__":
    main()
