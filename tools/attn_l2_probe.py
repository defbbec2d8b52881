"""Is the attention forward / backward waiting on its K/V (Q/dO) tile loads?  Times the
kernels at B16 nh12 S1024 (packed QKV, dropout 0.1) normally and with every (batch,
head) reading head 0's rows (in_bs = in_hs = 0: a one-head working set, L2-resident;
results are garbage, only the time matters)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.ops import hip, rng  # noqa: E402
from distributed_llm_trainer_amd.ops.hip import _off, _p, _stream, lib  # noqa: E402


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


B, nh, S, hd, p = 16, 12, 1024, 64, 0.1
H = nh * hd
M = B * S
key = rng.site_key(1, 2, 3, rng.SITE_ATTN)
qkv = torch.randn(M, 3 * H, device="cuda").bfloat16()
cos, sin = hip.rope_tables(64, S, device="cuda")
o, aux = hip.attention_fwd_packed(qkv, B, S, nh, p, key)
lse, mask = aux
do = torch.randn_like(o)
thr = rng.keep_threshold(p)
ds = 1.0 / (1.0 - p)
delta = torch.empty(B, nh, S, dtype=torch.float32, device="cuda")
dqkv = torch.empty(M, 3 * H, dtype=torch.bfloat16, device="cuda")
st = S * 3 * H
for name, bs, hs in (("normal", st, hd), ("one head (L2)", 0, 0)):
    def fwd():
        lib().dlt_attn_fwd_ex(_p(qkv), _off(qkv, H), _off(qkv, 2 * H), _p(o), _p(lse), _p(mask), B, nh, S, hd,
                              1.0 / math.sqrt(hd), key & 0xFFFFFFFF, thr, ds, 0, bs, hs, 3 * H, 0, _stream())

    def bwd():
        lib().dlt_attn_bwd_ex(_p(qkv), _off(qkv, H), _off(qkv, 2 * H), _p(o), _p(do), _p(lse), _p(mask), _p(delta),
                              _p(dqkv), _off(dqkv, H), _off(dqkv, 2 * H), B, nh, S, hd, 1.0 / math.sqrt(hd), ds,
                              bs, hs, 3 * H, st, hd, 3 * H, _p(cos), _p(sin), 0, _stream())
    print(f"{name:14s} fwd {timeit(fwd):6.1f} us  bwd (dQ + dK/dV) {timeit(bwd):6.1f} us", flush=True)
