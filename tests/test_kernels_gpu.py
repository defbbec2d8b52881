"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference of the same op
(ops/reference.py), on the MI355X.  Dropout is ON where the op has it: the counter-hash
masks are bit-identical between kernel and reference (ops/rng.py)."""
import math

import pytest
import torch

from distributed_llm_trainer_amd.ops import hip, reference as ref, rng

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=0.0, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    bad = (err > lim).sum().item()
    assert bad == 0, f"{what}: {bad} elements out of tolerance, max err {err.max().item():.3e}"


def test_library_loads():
    L = hip.lib()
    assert L is not None


@pytest.mark.parametrize("H", [768, 1024, 1600])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_add_dropout_rmsnorm_fwd(H, p):
    torch.manual_seed(0)
    M = 515
    r = torch.randn(M, H, device=DEV)
    d = torch.randn(M, H, device=DEV).bfloat16()
    w = torch.rand(H, device=DEV) + 0.5
    key = rng.site_key(7, 3, 1, rng.SITE_RESID)
    x, y, rs = hip.add_dropout_rmsnorm_fwd(r, d, w, 1e-6, p, key)
    x2, y2, rs2 = ref.add_dropout_rmsnorm_fwd(r, d, w, 1e-6, p, key)
    _close(x, x2, 1e-5, 1e-5, "x")
    _close(rs, rs2, 1e-5, 1e-4, "rstd")
    _close(y, y2.float(), 2e-2, 1e-2, "y")


@pytest.mark.parametrize("H", [768, 1600])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_rmsnorm_bwd(H, p):
    torch.manual_seed(1)
    M = 1031
    x = torch.randn(M, H, device=DEV)
    rstd = torch.rsqrt(x.pow(2).mean(-1) + 1e-6)
    w = torch.rand(H, device=DEV) + 0.5
    dy = torch.randn(M, H, device=DEV).bfloat16()
    dres = torch.randn(M, H, device=DEV)
    key = rng.site_key(9, 0, 2, rng.SITE_MLP)
    sc = torch.tensor(0.25, device=DEV)
    dw1 = torch.zeros(H, device=DEV)
    dw2 = torch.zeros(H, device=DEV)
    dx, dd = hip.rmsnorm_bwd(dy, x, rstd, w, dres, dw1, p, key, dy_scale=sc)
    dx2, dd2 = ref.rmsnorm_bwd(dy, x, rstd, w, dres, dw2, p, key, dy_scale=sc)
    _close(dx, dx2, 1e-4, 1e-4, "dx")
    _close(dd, dd2.float(), 2e-2, 1e-2, "ddelta")
    _close(dw1, dw2, 1e-2, 1e-4, "dw")


def test_embedding():
    torch.manual_seed(2)
    V, H, M = 1000, 768, 4096
    W = torch.randn(V, H, device=DEV)
    ids = torch.randint(0, V, (M,), device=DEV)
    _close(hip.embedding_fwd(ids, W), ref.embedding_fwd(ids, W), 0.0, 0.0, "emb fwd fp32")
    Wb = W.bfloat16()
    _close(hip.embedding_fwd(ids, Wb), ref.embedding_fwd(ids, Wb), 0.0, 0.0, "emb fwd bf16")
    dout = torch.randn(M, H, device=DEV)
    g1 = torch.zeros(V, H, device=DEV)
    g2 = torch.zeros(V, H, device=DEV)
    hip.embedding_bwd(ids, dout, g1)
    ref.embedding_bwd(ids, dout, g2)
    _close(g1, g2, 1e-4, 1e-5, "emb bwd")


@pytest.mark.parametrize("M,dist", [(4099, "zipf"), (3000, "one_token"), (517, "two_runs"), (16, "uniform")])
def test_embedding_bwd_deterministic(M, dist):
    """Sorted segment-sum scatter-add: runs inside one 16-position chunk, runs cut by
    chunk edges and runs spanning many chunks (a single token id everywhere); the result
    matches the fp64 sum and two calls are bitwise identical (no float atomics)."""
    torch.manual_seed(12)
    V, H = 2000, 768
    if dist == "zipf":  # heavy head like real text: a few ids take most positions
        ids = torch.minimum((torch.rand(M, device=DEV) ** 4 * V).long(), torch.tensor(V - 1, device=DEV))
    elif dist == "one_token":
        ids = torch.full((M,), 7, device=DEV, dtype=torch.long)
    elif dist == "two_runs":
        ids = torch.where(torch.arange(M, device=DEV) % 3 == 0, 5, V - 1)
    else:
        ids = torch.randint(0, V, (M,), device=DEV)
    dout = torch.randn(M, H, device=DEV)
    base = torch.randn(V, H, device=DEV)
    g1, g2 = base.clone(), base.clone()
    hip.embedding_bwd(ids, dout, g1)
    hip.embedding_bwd(ids, dout, g2)
    assert torch.equal(g1, g2), "embedding_bwd is not deterministic"
    exp = base.double().index_add_(0, ids, dout.double())
    _close(g1, exp, 1e-4, 1e-5, "emb bwd vs fp64")


def test_rmsnorm_bwd_dw_deterministic():
    torch.manual_seed(13)
    M, H = 16384, 768
    x = torch.randn(M, H, device=DEV)
    rstd = torch.rsqrt(x.pow(2).mean(-1) + 1e-6)
    w = torch.rand(H, device=DEV) + 0.5
    dy = torch.randn(M, H, device=DEV).bfloat16()
    outs = []
    for _ in range(2):
        dw = torch.ones(H, device=DEV)
        hip.rmsnorm_bwd(dy, x, rstd, w, None, dw, 0.0, 0)
        outs.append(dw)
    assert torch.equal(outs[0], outs[1]), "rmsnorm dw reduction is not deterministic"
    exp = 1.0 + (dy.double() * (x.double() * rstd.double()[:, None])).sum(0)
    _close(outs[0], exp, 1e-2, 1e-4, "dw vs fp64")


def test_rope():
    torch.manual_seed(3)
    B, S, nh, hd = 2, 300, 12, 64
    qkv = torch.randn(B * S, 3 * nh * hd, device=DEV).bfloat16()
    cos, sin = hip.rope_tables(hd, 1024, device=DEV)
    q, k, v = hip.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    q2, k2, v2 = ref.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    for a, b, n in ((q, q2, "q"), (k, k2, "k"), (v, v2, "v")):
        _close(a, b, 2e-2, 1e-2, n)
    dq, dk, dv = (torch.randn(B, nh, S, hd, device=DEV).bfloat16() for _ in range(3))
    _close(hip.rope_qkv_bwd(dq, dk, dv, cos, sin), ref.rope_qkv_bwd(dq, dk, dv, cos, sin), 2e-2, 1e-2, "dqkv")
    dqf = dq.float()
    _close(hip.rope_qkv_bwd(dqf, dk, dv, cos, sin), ref.rope_qkv_bwd(dq, dk, dv, cos, sin), 2e-2, 1e-2, "dqkv f32")


def test_swiglu():
    torch.manual_seed(4)
    M, I = 777, 3072
    gu = (torch.randn(M, 2 * I, device=DEV) * 2).bfloat16()
    _close(hip.swiglu_fwd(gu), ref.swiglu_fwd(gu), 3e-2, 1e-2, "swiglu fwd")
    da = torch.randn(M, I, device=DEV).bfloat16()
    _close(hip.swiglu_bwd(gu, da), ref.swiglu_bwd(gu, da), 3e-2, 1e-2, "swiglu bwd")
    # the optional s output (engine s ring) carries exactly the forward kernel's bits
    s_out = torch.empty(M, I, device=DEV, dtype=torch.bfloat16)
    dgu = hip.swiglu_bwd(gu, da, s_out=s_out)
    assert torch.equal(s_out, hip.swiglu_fwd(gu))
    assert torch.equal(dgu, hip.swiglu_bwd(gu, da))


def test_cross_entropy():
    torch.manual_seed(5)
    M, V, Vp = 1024, 50257, 50304
    logits = (torch.randn(M, Vp, device=DEV) * 3).bfloat16()
    tg = torch.randint(0, V, (M,), device=DEV)
    tg[::7] = -100
    nv = (tg != -100).sum()
    l1 = logits.clone()
    l2 = logits.clone()
    loss1 = hip.cross_entropy_fwd_bwd(l1, tg, V, nv)
    loss2 = ref.cross_entropy_fwd_bwd(l2, tg, V, nv)
    _close(loss1, loss2, 2e-3, 1e-4, "ce loss")
    _close(l1, l2, 1e-6, 2e-2, "ce grad")
    assert l1[:, V:].abs().max().item() == 0.0


def test_adamw_and_norm():
    torch.manual_seed(6)
    n = 100003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.randn(n, device=DEV) * 0.1
    v = torch.rand(n, device=DEV) * 0.01
    sh = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    ss = torch.zeros(1, device=DEV)
    hip.sumsq(g, ss)
    _close(ss, g.pow(2).sum().reshape(1), 1e-1, 1e-5, "sumsq")
    big = torch.randn(50_000_003, device=DEV)  # 4096 blocks' worth: the capped grid
    sums = []
    for _ in range(4):  # bitwise reproducible: replicas must compute the same clip coefficient
        t = torch.zeros(1, device=DEV)
        hip.sumsq(big, t)
        sums.append(t.item())
    assert len(set(sums)) == 1, sums
    assert abs(sums[0] - big.double().pow(2).sum().item()) < 1e-4 * sums[0]
    scale = torch.zeros(2, device=DEV)
    hip.clip_coef(ss, scale, 0.5, 1.0, 0.5)
    norm = g.norm() * 0.5
    _close(scale[0], norm, 1e-3, 1e-5, "norm")
    _close(scale[1], torch.clamp(1.0 / (norm + 1e-6), max=1.0) * 0.5, 1e-6, 1e-5, "coef")
    hip.adamw_flat(p, g, m, v, sh, 1e-3, 0.9, 0.95, 1e-8, 0.1, 5, scale)
    ref.adamw_step(p2, g, m2, v2, None, 1e-3, 0.9, 0.95, 1e-8, 0.1, 5, scale[1])
    _close(p, p2, 1e-6, 1e-5, "param")
    _close(m, m2, 1e-6, 1e-5, "m")
    _close(v, v2, 1e-7, 1e-5, "v")
    _close(sh, p.bfloat16(), 0.0, 0.0, "shadow")


def _attn_inputs(B, nh, S, seed, hd=64):
    torch.manual_seed(seed)
    q = torch.randn(B, nh, S, hd, device=DEV).bfloat16()
    k = torch.randn(B, nh, S, hd, device=DEV).bfloat16()
    v = torch.randn(B, nh, S, hd, device=DEV).bfloat16()
    return q, k, v


# head_dim 128 (template D = 128 of attention.hip) on a subset of the sequence lengths
_ATTN_FWD_CASES = [(S, 64) for S in (64, 128, 200, 1024, 2100)] + [(S, 128) for S in (64, 200, 1024)]


@pytest.mark.parametrize("S,hd", _ATTN_FWD_CASES)
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fwd(S, hd, p):
    B, nh = 2, 3
    q, k, v = _attn_inputs(B, nh, S, 10 + S, hd)
    key = rng.site_key(1, 2, 3, rng.SITE_ATTN)
    o, aux = hip.attention_fwd(q, k, v, p, key)
    lse = aux[0]
    o2, lse2 = ref.attention_fwd(q, k, v, p, key)
    _close(lse, lse2, 2e-3, 1e-4, "lse")
    if p > 0:
        keep = rng.attn_keep_mask(B * nh, S, S, key, p, device=DEV)
        W = (S + 31) // 32
        bits = aux[1][0].view(B * nh, W, S).transpose(1, 2)  # word-major [bh][word][query]
        kk = torch.arange(S, device=DEV)
        got = ((bits[:, :, kk // 32].long() >> (kk % 32)) & 1).bool()
        causal = torch.tril(torch.ones(S, S, dtype=torch.bool, device=DEV))
        assert torch.equal(got & causal, keep & causal), "stored dropout bitmask differs from the hash"
        bitsT = aux[1][1].view(B * nh, W, S).transpose(1, 2)  # [bh][key][query word]
        qq = torch.arange(S, device=DEV)
        gotT = ((bitsT[:, :, qq // 32].long() >> (qq % 32)) & 1).bool()  # [bh][key][query]
        assert torch.equal(gotT.transpose(1, 2) & causal, keep & causal), "transposed bitmask differs"
    _close(o, o2.float(), 2e-2, 2e-2, "o")


def test_attention_fwd_identity_asymmetric():
    """A = I-style check with asymmetric V: catches transposed C/D or operand maps."""
    B, nh, S = 1, 1, 128
    q = torch.zeros(B, nh, S, 64, device=DEV)
    k = torch.zeros(B, nh, S, 64, device=DEV)
    q[..., 0] = 40.0   # huge scores on the diagonal only via position-dependent k
    for j in range(S):
        k[0, 0, j, 0] = 1.0 if j % 2 == 0 else -1.0
    v = torch.arange(S * 64, device=DEV, dtype=torch.float32).view(1, 1, S, 64) / (S * 64)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    o, _ = hip.attention_fwd(q, k, v, 0.0, 0)
    o2, _ = ref.attention_fwd(q, k, v, 0.0, 0)
    _close(o, o2.float(), 1e-2, 1e-2, "o(asym)")


@pytest.mark.parametrize("S", [64, 192, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("hd", [64, 128])
def test_attention_bwd(S, p, hd):
    B, nh = 2, 3
    q, k, v = _attn_inputs(B, nh, S, 20 + S, hd)
    key = rng.site_key(4, 5, 6, rng.SITE_ATTN)
    o, lse = ref.attention_fwd(q, k, v, p, key)
    do = torch.randn_like(o.float()).bfloat16()
    dq, dk, dv = hip.attention_bwd(q, k, v, o, do, lse, p, key)  # regenerates the bitmask
    _, aux = hip.attention_fwd(q, k, v, p, key)
    dq3, dk3, dv3 = hip.attention_bwd(q, k, v, o, do, (lse, aux[1]), p, key)
    assert torch.equal(dq, dq3) and torch.equal(dk, dk3) and torch.equal(dv, dv3)
    dq2, dk2, dv2 = ref.attention_bwd(q, k, v, o, do, lse, p, key)
    for a, b, n in ((dq, dq2, "dq"), (dk, dk2, "dk"), (dv, dv2, "dv")):
        scale = b.float().abs().max().item()
        _close(a, b.float(), 2e-2 * max(1.0, scale), 2e-2, n)


def test_rope_qk_inplace():
    torch.manual_seed(31)
    B, S, nh, hd = 2, 300, 12, 64
    qkv = torch.randn(B * S, 3 * nh * hd, device=DEV).bfloat16()
    cos, sin = hip.rope_tables(hd, 1024, device=DEV)
    got = hip.rope_qk_inplace(qkv.clone(), B, S, nh, cos, sin)
    want = ref.rope_qk_inplace(qkv.float().clone(), B, S, nh, cos, sin)
    _close(got, want, 2e-2, 1e-2, "rope in place")
    H = nh * hd
    assert torch.equal(got[:, 2 * H:], qkv[:, 2 * H:]), "v block must be untouched"


@pytest.mark.parametrize("S", [64, 200, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("hd", [64, 128])
def test_attention_packed_fwd_bwd(S, p, hd):
    """Attention straight on the packed QKV (strided q/k/v) with the inverse RoPE in the
    backward epilogue == the split path (RoPE copy kernel, head-major attention, repack)."""
    torch.manual_seed(32 + S)
    B, nh = 2, 3
    H = nh * hd
    raw = torch.randn(B * S, 3 * H, device=DEV).bfloat16()
    cos, sin = hip.rope_tables(hd, 1024, device=DEV)
    key = rng.site_key(7, 8, 9, rng.SITE_ATTN)
    q, k, v = hip.rope_qkv_fwd(raw, B, S, nh, cos, sin)
    o1, aux1 = hip.attention_fwd(q, k, v, p, key)
    packed = hip.rope_qk_inplace(raw.clone(), B, S, nh, cos, sin)
    o2, aux2 = hip.attention_fwd_packed(packed, B, S, nh, p, key)
    assert torch.equal(o1, o2) and torch.equal(aux1[0], aux2[0])
    do = torch.randn(B * S, H, device=DEV).bfloat16()
    dq, dk, dv = hip.attention_bwd(q, k, v, o1, do, aux1, p, key)
    assert torch.equal(dv.transpose(1, 2).reshape(B * S, H),
                       hip.attention_bwd_packed(packed, o2, do, aux2, p, key, B, S, nh, cos, sin)[:, 2 * H:])
    want = ref.rope_qkv_bwd(dq.float(), dk.float(), dv.float(), cos, sin)
    got = hip.attention_bwd_packed(packed, o2, do, aux2, p, key, B, S, nh, cos, sin)
    scale = want.abs().max().item()
    _close(got, want, 1e-2 * max(1.0, scale), 1e-2, "dqkv packed")
    # against the fp32 reference of the whole chain
    want2 = ref.attention_bwd_packed(packed.float(), o2.float(), do.float(), aux2[0], p, key, B, S, nh, cos, sin)
    _close(got, want2, 2e-2 * max(1.0, scale), 2e-2, "dqkv packed vs fp32 ref")


@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (8192, 768, 3072), (1000, 300, 200), (256, 50304, 768)])
def test_gemm_planner(M, N, K):
    from distributed_llm_trainer_amd.ops import gemm
    assert gemm.available()
    g = gemm.HipGemm()
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    y = g.linear(x, w)
    _close(y, (x.float() @ w.float().t()), 0.05 * K ** 0.5, 2e-2, "linear")
    dx = g.linear_dgrad(dy, w)
    _close(dx, dy.float() @ w.float(), 0.05 * N ** 0.5, 2e-2, "dgrad")
    dw = torch.randn(N, K, device=DEV)
    ref = dw + dy.float().t() @ x.float()
    g.wgrad_acc(dw, dy, x)
    _close(dw, ref, 1e-2 * M ** 0.5, 1e-3, "wgrad acc")
    g.wgrad_acc(dw, dy, x)  # second call uses the cached (tuned) plan, accumulates again
    _close(dw, ref + dy.float().t() @ x.float(), 2e-2 * M ** 0.5, 1e-3, "wgrad acc 2")


@pytest.mark.parametrize("M,N,K", [(32768, 768, 768), (4096, 2304, 768), (2048, 300, 200)])
def test_wgrad_splitk(M, N, K):
    """Split-K weight gradient (strided-batched hipBLASLt slices + fixed-order sum kernel)
    against the fp32 reference, for every split count, and the auto-picked path; the sum
    is deterministic (two identical calls give bit-identical accumulators)."""
    from distributed_llm_trainer_amd.ops import gemm
    g = gemm.HipGemm()
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    base = torch.randn(N, K, device=DEV)
    ref = base + dy.float().t() @ x.float()
    cands = [s for s in gemm.HipGemm.SPLITK_CANDIDATES if M % (s * 8) == 0]
    assert cands, "every tested shape must exercise split-K"
    for s in cands:  # every factor the tuner can pick
        dw = base.clone()
        g._wgrad_split(dw, dy, x, s)
        _close(dw, ref, 1e-2 * M ** 0.5, 1e-3, f"split-K x{s}")
        dw2 = base.clone()
        g._wgrad_split(dw2, dy, x, s)
        assert torch.equal(dw, dw2), "split-K accumulate is not deterministic"
    dw = base.clone()
    g.wgrad_acc(dw, dy, x)
    _close(dw, ref, 1e-2 * M ** 0.5, 1e-3, "wgrad auto")
    assert (M, N, K) in g._splitk


def test_gemm_planner_accumulate_without_backup():
    """An accumulating GEMM whose autotune cannot back up C must not be timed in place
    (timing with beta = 0 would overwrite the accumulator and the real call would then
    return 2*A*B): the planner keeps the heuristic pick and dw == base + dy^T x."""
    from distributed_llm_trainer_amd.ops import gemm
    g = gemm.HipGemm()
    L = gemm.lib()
    M, N, K = 1536, 640, 320  # a key no other test uses (plans are cached per process)
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    base = torch.randn(N, K, device=DEV)
    ref = base + dy.float().t() @ x.float()
    assert L.dlt_gemm_test_fail_backup(1) == 0
    try:
        dw = base.clone()
        g._wgrad_plain(dw, dy, x)
        torch.cuda.synchronize()
    finally:
        L.dlt_gemm_test_fail_backup(0)
    _close(dw, ref, 1e-2 * M ** 0.5, 1e-3, "wgrad acc without backup")
    line = [ln for ln in gemm.report().splitlines() if f"m={K} n={N} k={M} acc=1" in ln]
    assert line and "chosen=0" in line[0], line


def test_gemm_plan_pin_roundtrip(tmp_path):
    """Plan machinery: the exported table names hipBLASLt solution indices; a pinned
    solution is used (no timing) for a key first seen afterwards, and a pin the library
    does not support for the problem is ignored."""
    from distributed_llm_trainer_amd.ops import gemm
    g = gemm.HipGemm()
    x = torch.randn(512, 384, device=DEV).bfloat16()
    w = torch.randn(640, 384, device=DEV).bfloat16()
    g.linear(x, w)
    plan = gemm.export_plan()
    assert plan["hipblaslt_version"] == gemm.lib().dlt_gemm_lib_version()
    line = [ln for ln in plan["hipblaslt"] if ln.split()[2:5] == ["640", "512", "384"]]
    assert line, plan["hipblaslt"]
    sol = int(line[0].split()[-1])
    assert sol >= 0
    path = tmp_path / "plan.json"
    gemm.save_plan(str(path))
    # pin that solution for a fresh forward key of the same (N, K) (m=N, n=M, k=K in BLAS terms)
    M, N, K = 768, 640, 384
    L = gemm.lib()
    assert L.dlt_gemm_pin(1, 0, N, M, K, K, K, N, 1, 1, 1, 0, 1, 0, 0, 0, sol) == 0
    x2 = torch.randn(M, K, device=DEV).bfloat16()
    w2 = torch.randn(N, K, device=DEV).bfloat16()
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    g._lib_linear(x2, w2, y)
    _close(y, x2.float() @ w2.float().t(), 0.05 * K ** 0.5, 2e-2, "pinned linear")
    rep = [ln for ln in gemm.report().splitlines() if f"m={N} n={M} k={K} acc=0" in ln]
    assert rep and f"sol={sol} " in rep[0] and "chosen=-1" in rep[0], rep
    # a pin naming a solution of another GEMM type (an fp32-output NT weight-gradient
    # kernel) is rejected for this bf16 TN problem and the key is tuned normally
    dw = torch.zeros(N, K, device=DEV)
    g._wgrad_plain(dw, torch.randn(256, N, device=DEV).bfloat16(), torch.randn(256, K, device=DEV).bfloat16())
    wl = [ln for ln in gemm.export_plan()["hipblaslt"] if ln.split()[:2] == ["0", "1"] and ln.split()[4] == "256"]
    assert wl
    wsol = int(wl[0].split()[-1])
    misses = L.dlt_gemm_pin_misses()
    assert L.dlt_gemm_pin(1, 0, N, 896, K, K, K, N, 1, 1, 1, 0, 1, 0, 0, 0, wsol) == 0
    x3 = torch.randn(896, K, device=DEV).bfloat16()
    y3 = torch.empty(896, N, device=DEV, dtype=torch.bfloat16)
    g._lib_linear(x3, w2, y3)
    _close(y3, x3.float() @ w2.float().t(), 0.05 * K ** 0.5, 2e-2, "bogus-pin linear")
    assert L.dlt_gemm_pin_misses() == misses + 1
    gemm.load_plan(str(path))  # loading a saved plan re-pins without error


@pytest.mark.parametrize("T,Nr,Nc", [(1024, 256, 192), (2048, 768, 384), (4096, 2304, 768), (1024, 384, 192),
                                     (2048, 50304, 768), (2048, 1024, 1024), (2048, 384, 128), (1024, 1024, 4096)])
def test_gemm_wgrad_kernel(T, Nr, Nc):
    """Hand-written weight-gradient GEMM (in-place and split-K + fixed-order sum) vs
    the fp32 torch reference; split-K results are bitwise repeatable.  Nr % 256 == 128
    (384; the 50304-row lm_head gradient) runs a last half row tile.  Nc % 192 != 0
    (1024, 128, 4096: the medium model's hidden sizes) runs the 256 x 128 column tile."""
    torch.manual_seed(0)
    dy = torch.randn(T, Nr, device=DEV).bfloat16()
    x = torch.randn(T, Nc, device=DEV).bfloat16()
    base = torch.randn(Nr, Nc, device=DEV)
    ref = base + dy.float().t() @ x.float()
    outs = {}
    for splits in (1, 3, 0):
        dw = base.clone()
        assert hip.gemm_wgrad(dw, dy, x, splits)
        _close(dw, ref, 1e-3 * T ** 0.5, 1e-4, f"wgrad splits={splits}")
        outs[splits] = dw
    dw = base.clone()
    assert hip.gemm_wgrad(dw, dy, x, 0)
    assert torch.equal(dw, outs[0]), "split-K wgrad not deterministic"
    assert not hip.gemm_wgrad(base, dy[:, :64], x), "untileable shape must be refused"


@pytest.mark.parametrize("T,Nr,Nc,shares", [(32768, 6144, 768, 0), (4096, 2304, 768, 0), (2048, 384, 192, 5),
                                            (8192, 50304, 768, 0), (1024, 256, 192, 3), (4096, 768, 3072, 7),
                                            (4096, 1024, 1024, 0), (2048, 384, 128, 5)])
def test_gemm_wgrad_stream_k(T, Nr, Nc, shares):
    """Stream-K weight gradient (k_gemm_wgrad_sk + the fixed-order fixup): accumulates
    into dw like the split-K kernel, matches the fp32 reference on the whole output
    (shares crossing row tiles, whole tiles written straight into dw, the half row tile
    of Nr % 256 == 128), and is bitwise repeatable."""
    torch.manual_seed(1)
    dy = torch.randn(T, Nr, device=DEV).bfloat16()
    x = torch.randn(T, Nc, device=DEV).bfloat16()
    base = torch.randn(Nr, Nc, device=DEV)
    ref = base + dy.float().t() @ x.float()
    dw = base.clone()
    assert hip.gemm_wgrad_sk(dw, dy, x, shares)
    _close(dw, ref, 1e-3 * T ** 0.5, 1e-4, f"wgrad stream-K {T}x{Nr}x{Nc}")
    dw2 = base.clone()
    assert hip.gemm_wgrad_sk(dw2, dy, x, shares)
    assert torch.equal(dw, dw2), "stream-K wgrad not deterministic"
    assert not hip.gemm_wgrad_sk(base, dy[:, :64], x), "untileable shape must be refused"


@pytest.mark.parametrize("T,Nr,Nc", [(2048, 768, 384), (4096, 2304, 768), (2048, 384, 192), (2048, 1024, 1024)])
def test_gemm_wgrad_kernels_fp16(T, Nr, Nc):
    """The weight-gradient kernels instantiated for IEEE-half operands
    (v_mfma_f32_16x16x32_f16; --mixed_precision fp16): split-K, in-place and stream-K
    forms vs the fp32 reference, and the planner's hand-written route for fp16 operands
    into an fp32 accumulator."""
    from distributed_llm_trainer_amd.ops import gemm
    torch.manual_seed(6)
    dy = torch.randn(T, Nr, device=DEV).half()
    x = torch.randn(T, Nc, device=DEV).half()
    base = torch.randn(Nr, Nc, device=DEV)
    ref = base + dy.float().t() @ x.float()
    for splits in (1, 3):
        dw = base.clone()
        assert hip.gemm_wgrad(dw, dy, x, splits)
        _close(dw, ref, 1e-3 * T ** 0.5, 1e-4, f"fp16 wgrad splits={splits}")
    dw = base.clone()
    assert hip.gemm_wgrad_sk(dw, dy, x, 0)
    _close(dw, ref, 1e-3 * T ** 0.5, 1e-4, "fp16 wgrad stream-K")
    with pytest.raises(ValueError):
        hip.gemm_wgrad(base.clone(), dy, x.bfloat16(), 1)  # mixed operand formats
    g = gemm.HipGemm()
    # fp16 operands take the hand route into an fp32 accumulator AND into a 16-bit output
    # (FSDP's fp16 reduce buffers; the partial sum kernel dispatches on the format)
    assert g._wgrad_hand_ok(dy, x) and g._wgrad_hand_ok(dy, x, to16=True)
    for s in (-1, -3, g.STREAMK):
        dw = base.clone()
        g._run_wgrad(dw, dy, x, s, False)
        _close(dw, ref, 1e-3 * T ** 0.5, 1e-4, f"fp16 planner route {s}")
    for s in (-1, -3):
        out = torch.empty(Nr, Nc, device=DEV, dtype=torch.float16)
        g._run_wgrad(out, dy, x, s, True)
        _close(out.float(), ref - base, 2e-3 * T ** 0.5, 2e-3, f"fp16 16-bit-output route {s}")


def test_planner_stream_k_route():
    """The planner's stream-K pick (splitk value STREAMK) runs the stream-K kernel for an
    fp32 accumulator and falls back to the split kernel for a bf16 output."""
    from distributed_llm_trainer_amd.ops import gemm
    g = gemm.HipGemm()
    T, N, K = 4096, 2304, 768
    dy = torch.randn(T, N, device=DEV).bfloat16()
    x = torch.randn(T, K, device=DEV).bfloat16()
    want = dy.float().t() @ x.float()
    dw = torch.zeros(N, K, device=DEV)
    g._run_wgrad(dw, dy, x, g.STREAMK, False)
    _close(dw, want, 1e-3 * T ** 0.5, 1e-4, "planner stream-K fp32")
    dwb = torch.zeros(N, K, device=DEV, dtype=torch.bfloat16)
    g._run_wgrad(dwb, dy, x, g.STREAMK, True)
    _close(dwb.float(), want, 2e-2 * T ** 0.5, 1e-2, "planner stream-K bf16 fallback")


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_fwd_growing_max_rescales(p):
    """Scores rise steeply along the keys, so the running row max grows by far more
    than the 2^8 rescale threshold in many tiles: exercises the deferred-rescale path
    (random data almost never takes it)."""
    B, nh, S = 1, 2, 512
    q = torch.zeros(B, nh, S, 64, device=DEV)
    k = torch.zeros(B, nh, S, 64, device=DEV)
    q[..., 0] = 8.0
    k[..., 0] = torch.arange(S, device=DEV, dtype=torch.float32) * 0.05  # score slope 0.05 per key
    k[..., 1] = torch.randn(S, device=DEV)
    q[..., 1] = torch.randn(S, device=DEV)
    v = torch.randn(B, nh, S, 64, device=DEV)
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    key = rng.site_key(7, 8, 9, rng.SITE_ATTN)
    o, aux = hip.attention_fwd(q, k, v, p, key)
    o2, lse2 = ref.attention_fwd(q, k, v, p, key)
    _close(aux[0], lse2, 2e-3, 1e-3, "lse(growing)")
    _close(o, o2.float(), 2e-2, 2e-2, "o(growing)")


def _relerr(got, want):
    """max |got - want| / max |want| (per tensor)."""
    return ((got.float() - want.float()).abs().max() / want.float().abs().max()).item()


# the model's forward-projection shapes at the fused-chain size (M = 16384 rows), a
# medium-size projection, and small multi-round / partial-round grids
@pytest.mark.parametrize("M,N,K,dtype", [(16384, 2304, 768, torch.bfloat16), (16384, 768, 768, torch.bfloat16),
                                         (16384, 768, 3072, torch.bfloat16), (16384, 6144, 768, torch.bfloat16),
                                         (4096, 3072, 1024, torch.bfloat16), (512, 384, 256, torch.bfloat16),
                                         (2560, 1152, 384, torch.bfloat16), (16384, 2304, 768, torch.float16),
                                         (2560, 1152, 384, torch.float16), (4096, 1024, 1024, torch.bfloat16),
                                         (2048, 4096, 1024, torch.bfloat16), (2560, 1280, 384, torch.float16)])
def test_gemm_bf16(M, N, K, dtype):
    """Persistent hand-written MFMA GEMM C = A B^T (csrc/gemm_bf16.hip) vs fp32 torch:
    every element within 16-bit output rounding (relative to the tensor's max); bf16 and
    IEEE-half operands (the --precision fp16 instantiation)."""
    torch.manual_seed(M + N + K)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(dtype)
    b = (torch.rand(N, K, device=DEV) * 2 - 1).to(dtype)
    c = hip.gemm_bf16(a, b)
    assert c is not None and c.dtype == dtype
    want = a.float() @ b.float().t()
    assert _relerr(c, want) < 8e-3
    _close(c, want, 8e-3 * want.abs().max().item(), 8e-3, "gemm_bf16")
    assert hip.gemm_bf16(a[:, :K - 64].contiguous(), b[:, :K - 64].contiguous()) is None  # K % 128


# K = 128 (two stages: no steady-state loop iteration), 192 (three) and 768 / 3072 (the
# projections); ragged last column tile (N % 256 = 128); tile-row counts that are and are
# not multiples of 8
@pytest.mark.parametrize("M,N,K", [(16384, 2304, 768), (16384, 768, 3072), (4096, 6144, 768), (2048, 50304, 768),
                                   (768, 1280, 512), (256, 256, 128), (1280, 640, 192), (2048, 384, 256)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_fw4(M, N, K, dtype):
    """4-wave 256 x 256 MFMA GEMM C = A B^T (csrc/gemm_fw4.hip, AGPR accumulators, both
    schedules) vs fp32 torch, bf16 and fp16 operands: every element within 16-bit output
    rounding, every tile written exactly once (a poisoned output is fully overwritten),
    plain / write-through / nt stores, XCD-band / half-band / row-major tile orders, one
    or two tiles per workgroup -- all bitwise equal."""
    torch.manual_seed(M + N + K)
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(dtype)
    b = (torch.rand(N, K, device=DEV) * 2 - 1).to(dtype)
    want = a.float() @ b.float().t()
    first = None
    tiles = (M // 256) * ((N + 255) // 256)
    two = (4096, 4100, 4240, 4244, 6148) if tiles % 16 == 0 else ()  # two tiles per workgroup
    for flags in (1, 0, 4, 2, 2048, 144, 145, 148, 146) + two:
        c = torch.full((M, N), float("nan"), device=DEV, dtype=dtype)
        assert hip.gemm_fw4(a, b, out=c, flags=flags) is not None
        assert not torch.isnan(c).any(), f"unwritten output (flags {flags})"
        assert _relerr(c, want) < 8e-3
        _close(c, want, 8e-3 * want.abs().max().item(), 8e-3, f"gemm_fw4 flags {flags}")
        if first is None:
            first = c
        assert torch.equal(c, first), f"schedules / store flavours must agree bitwise (flags {flags})"
    if tiles % 16:
        assert hip.gemm_fw4(a, b, flags=4096) is None  # two tiles per workgroup need tiles % 16 == 0
    assert hip.gemm_fw4(a, b, flags=16) is None and hip.gemm_fw4(a, b, flags=128) is None  # retired schedules
    assert hip.gemm_fw4(a[:, :K - 32].contiguous(), b[:, :K - 32].contiguous()) is None  # K % 64
    assert hip.gemm_fw4(a, b[:N - 8].contiguous()) is None  # N % 128


@pytest.mark.parametrize("M,I,K", [(16384, 3072, 768), (512, 256, 128), (1024, 384, 192)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_fw4_swiglu(M, I, K, dtype):
    """k_gemm_fw4 with the SwiGLU epilogue (csrc/gemm_fw4.hip flags 1024): gu bitwise equal to
    the plain k_gemm_fw4 GEMM of the same schedule, s bitwise equal to swiglu_fwd(gu)."""
    torch.manual_seed(M + I + K)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).to(dtype)
    w = (torch.rand(2 * I, K, device=DEV) * 2 - 1).to(dtype)
    for flags in (0, 4, 1, 144, 150, 2048):
        gu, s = hip.gemm_fw4_swiglu(x, w, flags=flags)
        plain = hip.gemm_fw4(x, w, flags=flags)
        assert torch.equal(gu, plain), f"gu differs from the plain GEMM (flags {flags})"
        assert torch.equal(s, hip.swiglu_fwd(gu)), f"s differs from swiglu_fwd (flags {flags})"
    assert hip.gemm_fw4_swiglu(x, w[:2 * I - 128].contiguous()) is None or I % 128 == 64


@pytest.fixture(params=[0, 4096], ids=["stage-in-loop", "epilogue-first"])
def gemm_late_flag(request, monkeypatch):
    """Runs a test with and without flags bit 4096 (epilogue-first staging of the next
    tile: the LATE instances of the RoPE / SwiGLU-backward GEMMs)."""
    monkeypatch.setattr(hip, "_GB_FLAGS", (hip._GB_FLAGS & ~4096) | request.param)
    return request.param


@pytest.mark.parametrize("B,S,nh,K", [(16, 1024, 12, 768), (4, 256, 25, 1600 // 128 * 128), (2, 512, 16, 1024)])
def test_gemm_qkv_rope(B, S, nh, K, gemm_late_flag):
    """QKV GEMM with NeoX RoPE on q/k in the epilogue == fp32 GEMM -> bf16 -> RoPE (the
    unfused GEMM + rope_qk_inplace math), at GPT-2 small (nh 12), an xl-like head count
    (nh 25, packed stride 3*25*64 = 4800) and medium (nh 16); both staging schedules
    (the persistent grid walks 3 tiles per workgroup at the first shape)."""
    torch.manual_seed(nh)
    M, H = B * S, nh * 64
    x = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(3 * H, K, device=DEV) * 2 - 1) / K ** 0.5).bfloat16()
    cos, sin = hip.rope_tables(64, 1024 if S <= 1024 else S, device=DEV)
    got = hip.gemm_qkv_rope(x, w, S, cos, sin)
    if (3 * H) % 192:
        assert got is None
        return
    y = (x.float() @ w.float().t()).bfloat16()
    q, k, v = ref.rope_qkv_fwd(y, B, S, nh, cos, sin)  # [B, nh, S, 64]
    want = torch.cat([t.transpose(1, 2).reshape(M, H) for t in (q, k, v)], dim=1)
    assert _relerr(got, want) < 1e-2
    _close(got, want.float(), 1e-2 * want.float().abs().max().item(), 1e-2, "qkv+rope")


@pytest.mark.parametrize("M,I,K", [(16384, 3072, 768), (4096, 4096, 1024), (2048, 6400, 1536)])
def test_gemm_gu_swiglu(M, I, K):
    """gate/up GEMM with SwiGLU in the epilogue: gu == fp32 GEMM (bf16 rounding) and
    s == silu(g) * u of the bf16-rounded g, u (the swiglu_fwd math)."""
    torch.manual_seed(I)
    x = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) / K ** 0.5).bfloat16()
    r = hip.gemm_gu_swiglu(x, w)
    if I % 96:
        assert r is None
        return
    gu, s = r
    want = x.float() @ w.float().t()
    assert _relerr(gu, want) < 8e-3
    gb = want.bfloat16().float()
    g, u = gb[:, :I], gb[:, I:]
    ws = g * torch.sigmoid(g) * u
    assert _relerr(s, ws) < 1e-2
    _close(s, ws, 1e-2 * ws.abs().max().item(), 1e-2, "swiglu s")


@pytest.mark.parametrize("M,Nout,Nred", [(512, 768, 2304), (512, 768, 768), (256, 768, 6144), (512, 3072, 768),
                                          (256, 768, 50304), (256, 1600, 4800), (512, 192, 128), (512, 1024, 1024),
                                          (256, 1024, 4096), (256, 4096, 1024), (512, 128, 256)])
def test_gemm_dgrad_vs_fp32(M, Nout, Nred):
    """Data gradient dX = dY @ W (W[Nred, Nout] read as stored) on the hand-written
    reduction-major-B kernel against the fp32 product -- every dgrad role of the step
    (q/k/v 2304, o 768, gate/up 6144, down 768 -> 3072, lm_head 50304), the 256 x 128
    column tile (Nout 1024 / 4096 / 128: the medium model) plus shapes that do not tile
    (None, nothing launched)."""
    torch.manual_seed(Nred)
    dy = (torch.rand(M, Nred, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(Nred, Nout, device=DEV) * 2 - 1) / Nred ** 0.5).bfloat16()
    r = hip.gemm_dgrad(dy, w)
    if Nout % 192 and Nout % 128:
        assert r is None
        return
    want = dy.float() @ w.float()
    assert torch.isfinite(r.float()).all()
    assert _relerr(r, want) < 8e-3, _relerr(r, want)


@pytest.mark.parametrize("M,Nout,Nred", [(512, 768, 2304), (1024, 3072, 768), (512, 768, 50304)])
def test_gemm_dgrad_fp16_vs_fp32(M, Nout, Nred):
    """The data-gradient kernel instantiated for IEEE half (k_gemm_bf16<192, 0, true, 1>,
    v_mfma_f32_16x16x32_f16, fp16 output) against the fp32 product, and the planner's
    dgrad route for fp16 operands (hand-written when the shape is pinned or raced so)."""
    from distributed_llm_trainer_amd.ops import gemm
    torch.manual_seed(Nred + 1)
    dy = (torch.rand(M, Nred, device=DEV) * 2 - 1).half()
    w = ((torch.rand(Nred, Nout, device=DEV) * 2 - 1) / Nred ** 0.5).half()
    r = hip.gemm_dgrad(dy, w)
    assert r.dtype == torch.float16
    want = dy.float() @ w.float()
    assert torch.isfinite(r.float()).all()
    assert _relerr(r, want) < 2e-3, _relerr(r, want)
    g = gemm.HipGemm()
    assert g._hand16_ok(dy, w, r) and not g._hand16_ok(dy, w.bfloat16(), r)
    r2 = g.linear_dgrad(dy, w)
    assert _relerr(r2, want) < 2e-3
    with pytest.raises(ValueError):
        hip.gemm_dgrad(dy.float(), w.float())


@pytest.mark.parametrize("M,dtype", [(512, torch.bfloat16), (16384, torch.bfloat16), (512, torch.float16),
                                     (16384, torch.float16)])
def test_gemm_down_swiglu_bwd_vs_fp32(M, dtype, gemm_late_flag):
    """Down-projection dgrad with the SwiGLU backward in the epilogue == the fp32 product
    rounded to the activation format (what the unfused dgrad writes) through
    k_swiglu_bwd's math, and == hip.swiglu_bwd on the library dgrad within 16-bit
    rounding; bf16 and IEEE half.  M 16384: 4 tiles per persistent workgroup (the
    epilogue-first staging's cross-tile path)."""
    torch.manual_seed(7)
    H, I = 768, 3072
    dd = (torch.rand(M, H, device=DEV) * 2 - 1).to(dtype)
    wd = ((torch.rand(H, I, device=DEV) * 2 - 1) / H ** 0.5).to(dtype)
    gu = (torch.randn(M, 2 * I, device=DEV) * 2).to(dtype)
    dgu = hip.gemm_down_swiglu_bwd(dd, wd, gu)
    assert dgu.dtype == dtype
    ds = (dd.float() @ wd.float()).to(dtype).float()
    g, u = gu.float()[:, :I], gu.float()[:, I:]
    sg = torch.sigmoid(g)
    want = torch.cat([ds * u * sg * (1 + g * (1 - sg)), ds * g * sg], dim=1)
    assert torch.isfinite(dgu.float()).all()
    assert _relerr(dgu, want) < 1.5e-2, _relerr(dgu, want)
    ref_k = hip.swiglu_bwd(gu, (dd.float() @ wd.float()).to(dtype))
    assert _relerr(dgu, ref_k.float()) < 1.5e-2
    # s_out: s = silu(g) * u with the forward kernel's exact bits (the engine's s ring),
    # the dgu output unchanged by it
    s = torch.full((M, I), float("nan"), dtype=dtype, device=DEV)
    dgu2 = hip.gemm_down_swiglu_bwd(dd, wd, gu, s_out=s)
    assert torch.equal(dgu2, dgu)
    assert torch.equal(s, hip.swiglu_fwd(gu))


def test_planner_dgrad_races_match_library():
    """HipGemm.linear_dgrad / linear_dgrad_swiglu (whatever the race picks) == the
    library dgrad (+ swiglu_bwd); the choices are recorded under kinds dgrad / dswiglu."""
    from distributed_llm_trainer_amd.ops import gemm
    torch.manual_seed(5)
    g = gemm.HipGemm()
    M, H, I = 4096, 768, 3072
    dy = (torch.rand(M, 3 * H, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(3 * H, H, device=DEV) * 2 - 1) / H ** 0.5).bfloat16()
    dx = g.linear_dgrad(dy, w)
    dx2 = torch.empty_like(dx)
    g._lib_dgrad(dy, w, dx2)
    assert _relerr(dx, dx2.float()) < 1e-2
    dd = (torch.rand(M, H, device=DEV) * 2 - 1).bfloat16()
    wd = ((torch.rand(H, I, device=DEV) * 2 - 1) / H ** 0.5).bfloat16()
    gu = (torch.randn(M, 2 * I, device=DEV) * 2).bfloat16()
    dgu = g.linear_dgrad_swiglu(dd, wd, gu, hip)
    ds = torch.empty(M, I, dtype=torch.bfloat16, device=DEV)
    g._lib_dgrad(dd, wd, ds)
    assert _relerr(dgu, hip.swiglu_bwd(gu, ds).float()) < 1.5e-2
    kinds = {k[0] for k in g._choice if len(k) == 4}
    assert {"dgrad", "dswiglu"} <= kinds


def test_planner_fused_races_match_unfused():
    """HipGemm.linear_rope / linear_swiglu (whatever the race picks) == the unfused
    library GEMM + kernel, and the choices are recorded process-wide."""
    from distributed_llm_trainer_amd.ops import gemm
    torch.manual_seed(4)
    g = gemm.HipGemm()
    B, S, nh, K, I = 4, 1024, 12, 768, 3072  # M = 4096: no shipped pin (the 8192-row shapes are pinned)
    M = B * S
    x = (torch.rand(M, K, device=DEV) * 2 - 1).bfloat16()
    wqkv = ((torch.rand(3 * nh * 64, K, device=DEV) * 2 - 1) / K ** 0.5).bfloat16()
    wgu = ((torch.rand(2 * I, K, device=DEV) * 2 - 1) / K ** 0.5).bfloat16()
    cos, sin = hip.rope_tables(64, S, device=DEV)
    qkv = g.linear_rope(x, wqkv, B, S, nh, cos, sin, hip)
    y = torch.empty_like(qkv)
    g._lib_linear(x, wqkv, y)
    hip.rope_qk_inplace(y, B, S, nh, cos, sin)
    assert _relerr(qkv, y) < 1e-2
    gu, s = g.linear_swiglu(x, wgu, hip)
    gu2 = torch.empty_like(gu)
    g._lib_linear(x, wgu, gu2)
    s2 = hip.swiglu_fwd(gu2)
    assert _relerr(gu, gu2) < 1e-2 and _relerr(s, s2) < 2e-2
    assert ("rope", M, 3 * nh * 64, K) in g._choice and ("swiglu", M, 2 * I, K) in g._choice
    plan = gemm.export_plan()
    assert f"rope:{M}x{3 * nh * 64}x{K}" in plan["fused"]


@pytest.mark.parametrize("choice", [-1, -3, 1, 2])
def test_planner_wgrad_choices_fp32_and_bf16(choice):
    """Every weight-gradient route of HipGemm -- hand-written kernel in place (-1) or with
    split-K partials (-3), hipBLASLt plain (1) or split-K (2) -- into an fp32 accumulator
    (wgrad_acc) and straight into a bf16 buffer (wgrad_set, the FSDP reduce-dtype path)
    against the fp32 reference."""
    from distributed_llm_trainer_amd.ops import gemm
    torch.manual_seed(5)
    g = gemm.HipGemm()
    T, N, K = 2048, 768, 384
    dy = torch.randn(T, N, device=DEV).bfloat16()
    x = torch.randn(T, K, device=DEV).bfloat16()
    keys = [(T, N, K), (T, N, K, "bf16")]  # fp32-accumulate and bf16-output races
    saved = {k: g._splitk.get(k, "absent") for k in keys}
    for k in keys:
        g._splitk[k] = choice
    try:
        base = torch.randn(N, K, device=DEV)
        ref = dy.float().t() @ x.float()
        dw = base.clone()
        g.wgrad_acc(dw, dy, x)
        _close(dw, base + ref, 1e-3 * T ** 0.5, 1e-4, f"wgrad_acc {choice}")
        db = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
        g.wgrad_set(db, dy, x)
        assert _relerr(db, ref) < 1e-2, f"wgrad_set {choice}"
    finally:
        for k in keys:
            if saved[k] == "absent":
                g._splitk.pop(k, None)
            else:
                g._splitk[k] = saved[k]


def test_scale_bf16():
    x = torch.randn(64, 768, device=DEV).bfloat16()
    s = torch.tensor(0.25, device=DEV)
    _close(hip.scale_bf16(x, s), ref.scale_bf16(x, s), 1e-6, 0.0, "scale_bf16")


def test_rmsnorm_bf16_weight_in_place():
    """bf16 norm weights (the gathered FSDP unit) are read in place and give the same
    result as the same values in fp32."""
    torch.manual_seed(40)
    M, H = 300, 768
    r = torch.randn(M, H, device=DEV)
    d = torch.randn(M, H, device=DEV).bfloat16()
    wb = (torch.rand(H, device=DEV) + 0.5).bfloat16()
    wf = wb.float()
    x1, y1, s1 = hip.add_dropout_rmsnorm_fwd(r, d, wf, 1e-6, 0.1, 123)
    x2, y2, s2 = hip.add_dropout_rmsnorm_fwd(r, d, wb, 1e-6, 0.1, 123)
    assert torch.equal(y1, y2) and torch.equal(x1, x2)
    dy = torch.randn(M, H, device=DEV).bfloat16()
    dw1, dw2 = torch.zeros(H, device=DEV), torch.zeros(H, device=DEV)
    g1 = hip.rmsnorm_bwd(dy, x1, s1, wf, None, dw1, 0.1, 77)
    g2 = hip.rmsnorm_bwd(dy, x1, s1, wb, None, dw2, 0.1, 77)
    assert torch.equal(g1[0], g2[0]) and torch.equal(g1[1], g2[1])
    _close(dw1, dw2, 1e-4, 1e-5, "dw")


def test_add_bf16_into_f32():
    torch.manual_seed(41)
    n = 7 * 1024 * 8 + 8
    dst = torch.randn(n, device=DEV)
    src = torch.randn(n, device=DEV).bfloat16()
    want = dst + src.float()
    assert hip.add_bf16_into_f32(dst, src)
    assert torch.equal(dst, want)
    assert not hip.add_bf16_into_f32(dst[:13], src[:13])  # outside the vector path: caller falls back


@pytest.mark.parametrize("B,S,nh", [(2, 1024, 25), (16, 1024, 12)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_packed_real_shapes(B, S, nh, p):
    """The packed attention kernels at the model's own shapes -- xl (nh 25: packed row
    stride 3*25*64 = 4800) and the GPT-2-small fused chain (B16 x nh 12) -- against the
    fp32 reference of the whole chain, with per-tensor relative-error bounds."""
    torch.manual_seed(B * nh + S)
    H = nh * 64
    raw = torch.randn(B * S, 3 * H, device=DEV).bfloat16()
    cos, sin = hip.rope_tables(64, S, device=DEV)
    key = rng.site_key(3, 1, 4, rng.SITE_ATTN)
    packed = hip.rope_qk_inplace(raw.clone(), B, S, nh, cos, sin)
    o, aux = hip.attention_fwd_packed(packed, B, S, nh, p, key)
    o_ref, lse_ref = ref.attention_fwd_packed(packed.float(), B, S, nh, p, key)
    assert _relerr(o, o_ref) < 1.5e-2
    _close(aux[0], lse_ref, 2e-3, 1e-3, "lse")
    do = torch.randn(B * S, H, device=DEV).bfloat16()
    got = hip.attention_bwd_packed(packed, o, do, aux, p, key, B, S, nh, cos, sin)
    want = ref.attention_bwd_packed(packed.float(), o.float(), do.float(), lse_ref, p, key, B, S, nh, cos, sin)
    for blk, name in ((slice(0, H), "dq"), (slice(H, 2 * H), "dk"), (slice(2 * H, 3 * H), "dv")):
        assert _relerr(got[:, blk], want[:, blk]) < 2e-2, name


# ------------------------------------------------------------------ fp16 (HK = 1)
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fp16_attention_packed_vs_fp32(p):
    """--mixed_precision fp16: the packed attention kernels instantiated for IEEE half
    (v_mfma_f32_32x32x16_f16, fp16 P / dS operands) against the fp32 reference of the
    whole chain (RoPE in place, causal attention with dropout, inverse RoPE in the
    backward epilogue), per-tensor relative error."""
    torch.manual_seed(61)
    B, S, nh = 2, 512, 4
    H = nh * 64
    raw = torch.randn(B * S, 3 * H, device=DEV).half()
    cos, sin = hip.rope_tables(64, S, device=DEV)
    key = rng.site_key(5, 2, 1, rng.SITE_ATTN)
    packed = hip.rope_qk_inplace(raw.clone(), B, S, nh, cos, sin)
    want_packed = ref.rope_qk_inplace(raw.float().clone(), B, S, nh, cos, sin)
    assert packed.dtype == torch.float16 and _relerr(packed, want_packed) < 2e-3
    o, aux = hip.attention_fwd_packed(packed, B, S, nh, p, key)
    assert o.dtype == torch.float16
    o_ref, lse_ref = ref.attention_fwd_packed(packed.float(), B, S, nh, p, key)
    assert _relerr(o, o_ref) < 4e-3, _relerr(o, o_ref)
    _close(aux[0], lse_ref, 2e-3, 1e-3, "lse fp16")
    do = torch.randn(B * S, H, device=DEV).half()
    got = hip.attention_bwd_packed(packed, o, do, aux, p, key, B, S, nh, cos, sin)
    assert got.dtype == torch.float16
    want = ref.attention_bwd_packed(packed.float(), o.float(), do.float(), lse_ref, p, key, B, S, nh, cos, sin)
    for blk, name in ((slice(0, H), "dq"), (slice(H, 2 * H), "dk"), (slice(2 * H, 3 * H), "dv")):
        e = _relerr(got[:, blk], want[:, blk])
        assert e < 6e-3, (name, e)


def test_fp16_norm_swiglu_ce_scale_vs_fp32():
    """The elementwise / norm / loss kernels in fp16 against fp32 references: residual +
    dropout + RMSNorm forward and backward (fp16 delta, y, dy, ddelta), SwiGLU forward /
    backward, cross-entropy with the loss-scaled in-place gradient, scale."""
    torch.manual_seed(62)
    M, H, I, V = 512, 768, 3072, 1000
    key = rng.site_key(1, 2, 3, rng.SITE_RESID)
    r = torch.randn(M, H, device=DEV)
    d = torch.randn(M, H, device=DEV).half()
    w = torch.rand(H, device=DEV) + 0.5
    x, y, rstd = hip.add_dropout_rmsnorm_fwd(r, d, w, 1e-6, 0.1, key, out_dtype=torch.float16)
    xr, yr, rstdr = ref.add_dropout_rmsnorm_fwd(r, d.float(), w, 1e-6, 0.1, key, out_dtype=torch.float32)
    assert y.dtype == torch.float16 and _relerr(y, yr) < 1e-3
    _close(x, xr, 1e-5, 1e-5, "x fp16 path")
    dy = torch.randn(M, H, device=DEV).half()
    dres = torch.randn(M, H, device=DEV)
    dw1, dw2 = torch.zeros(H, device=DEV), torch.zeros(H, device=DEV)
    dx, dd = hip.rmsnorm_bwd(dy, x, rstd, w, dres, dw1, 0.1, key, dy_mul=0.5)
    dxr, ddr = ref.rmsnorm_bwd(dy.float(), xr, rstdr, w, dres, dw2, 0.1, key, dy_mul=0.5)
    assert dd.dtype == torch.float16
    assert _relerr(dx, dxr) < 1e-4 and _relerr(dd, ddr) < 1e-3 and _relerr(dw1, dw2) < 1e-4
    gu = (torch.randn(M, 2 * I, device=DEV) * 2).half()
    s = hip.swiglu_fwd(gu)
    g, u = gu.float()[:, :I], gu.float()[:, I:]
    assert s.dtype == torch.float16 and _relerr(s, g * torch.sigmoid(g) * u) < 1e-3
    da = torch.randn(M, I, device=DEV).half()
    dgu = hip.swiglu_bwd(gu, da)
    dgu_r = ref.swiglu_bwd(gu.float(), da.float())
    assert _relerr(dgu, dgu_r) < 1e-3
    Vp = 1024
    logits = torch.randn(M, Vp, device=DEV).half()
    tgt = torch.randint(0, V, (M,), device=DEV)
    tgt[::7] = -100
    nv = (tgt != -100).sum()
    lg_ref = logits.float().clone()
    loss_r = ref.cross_entropy_fwd_bwd(lg_ref, tgt, V, nv, grad_scale=4096.0)
    lg = logits.clone()
    loss = hip.cross_entropy_fwd_bwd(lg, tgt, V, nv, grad_scale=4096.0)
    _close(loss, loss_r, 2e-3, 1e-3, "ce loss fp16")
    assert _relerr(lg, lg_ref) < 2e-3  # the gradient is representable (no fp16 underflow)
    sc = torch.full((), 0.25, device=DEV)
    z = hip.scale_bf16(d, sc, mul=2.0)
    assert z.dtype == torch.float16 and torch.equal(z, (d.float() * 0.5).half())


@pytest.mark.parametrize("cap", [8, 64, 192])
def test_gemm_persistent_multi_tile_matches(cap):
    """The persistent hand GEMMs with a capped grid (the ffbb window runs them on 192
    workgroups): every workgroup walks several tiles and prefetches the next tile's
    K-tiles, so the forward (K-major B) and the data-gradient (reduction-major B) forms
    must give bit-identical outputs to the one-tile-per-workgroup launches, and match
    the fp32 product."""
    torch.manual_seed(cap)
    M = 4096
    x = (torch.rand(M, 768, device=DEV) * 2 - 1).bfloat16()
    w = ((torch.rand(2304, 768, device=DEV) * 2 - 1) / 768 ** 0.5).bfloat16()
    dy = (torch.rand(M, 2304, device=DEV) * 2 - 1).bfloat16()
    prev = hip.gemm_grid_cap(0)
    try:
        y_full = hip.gemm_bf16(x, w)
        dx_full = hip.gemm_dgrad(dy, w)
        hip.gemm_grid_cap(cap)
        y_cap = hip.gemm_bf16(x, w)
        dx_cap = hip.gemm_dgrad(dy, w)
    finally:
        hip.gemm_grid_cap(prev)
    torch.cuda.synchronize()
    assert _relerr(dx_full, dy.float() @ w.float()) < 8e-3
    assert torch.equal(y_cap, y_full), (y_cap.float() - y_full.float()).abs().max().item()
    assert torch.equal(dx_cap, dx_full), (dx_cap.float() - dx_full.float()).abs().max().item()
