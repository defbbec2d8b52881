"""fp32-activation HIP kernels (csrc/fp32.hip, the engine's --mixed_precision fp32 mode)
against the fp32 PyTorch reference ops (ops/reference.py) with the same dropout bits,
and an fp32 training step that runs them (no ATen fallback for the model's ops)."""
import pytest
import torch

from distributed_llm_trainer_amd.ops import hip, reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp(min=1e-30)).item()


@pytest.mark.parametrize("H,p", [(768, 0.0), (768, 0.1), (1600, 0.1), (100, 0.1)])
def test_f32_norm_fwd_bwd(H, p):
    torch.manual_seed(H)
    M = 300
    r = torch.randn(M, H, device=DEV)
    d = torch.randn(M, H, device=DEV)
    w = torch.rand(H, device=DEV) + 0.5
    x, y, rs = hip.add_dropout_rmsnorm_fwd(r, d, w, 1e-6, p, 1234, out_dtype=torch.float32)
    xr, yr, rsr = ref.add_dropout_rmsnorm_fwd(r, d, w, 1e-6, p, 1234, out_dtype=torch.float32)
    assert y.dtype == torch.float32
    assert torch.allclose(x, xr, atol=1e-6, rtol=1e-6) and _rel(y, yr) < 1e-5 and _rel(rs, rsr) < 1e-5
    dy = torch.randn(M, H, device=DEV)
    dres = torch.randn(M, H, device=DEV)
    sc = torch.tensor(0.5, device=DEV)
    dw, dwr = torch.zeros(H, device=DEV), torch.zeros(H, device=DEV)
    dx, dd = hip.rmsnorm_bwd(dy, x, rs, w, dres, dw, p, 77, dy_scale=sc, dy_mul=2.0)
    dxr, ddr = ref.rmsnorm_bwd(dy, xr, rsr, w, dres, dwr, p, 77, dy_scale=sc, dy_mul=2.0)
    assert dd.dtype == torch.float32
    assert _rel(dx, dxr) < 1e-5 and _rel(dd, ddr) < 1e-5 and _rel(dw, dwr) < 1e-5
    # deterministic weight gradient (fixed-order column partials)
    dw2 = torch.zeros(H, device=DEV)
    hip.rmsnorm_bwd(dy, x, rs, w, dres, dw2, p, 77, dy_scale=sc, dy_mul=2.0)
    assert torch.equal(dw, dw2)


@pytest.mark.parametrize("hd", [64, 128])
def test_f32_rope_layouts(hd):
    torch.manual_seed(hd)
    B, S, nh = 2, 96, 3
    qkv = torch.randn(B * S, 3 * nh * hd, device=DEV)
    cos, sin = hip.rope_tables(hd, 128, device=DEV)
    q, k, v = hip.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    qr, kr, vr = ref.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    assert _rel(q, qr) < 1e-6 and _rel(k, kr) < 1e-6 and torch.equal(v, vr)
    back = hip.rope_qkv_bwd(q, k, v, cos, sin)
    assert _rel(back, ref.rope_qkv_bwd(qr, kr, vr, cos, sin)) < 1e-6
    assert _rel(back, qkv) < 1e-5  # the inverse rotation undoes the forward
    packed = qkv.clone()
    hip.rope_qk_inplace(packed, B, S, nh, cos, sin)
    assert _rel(packed, ref.rope_qk_inplace(qkv.clone(), B, S, nh, cos, sin)) < 1e-6


def test_f32_swiglu_ce_scale():
    torch.manual_seed(3)
    gu = torch.randn(257, 2 * 384, device=DEV)
    s = hip.swiglu_fwd(gu)
    assert s.dtype == torch.float32 and _rel(s, ref.swiglu_fwd(gu)) < 1e-5
    da = torch.randn(257, 384, device=DEV)
    s2 = torch.empty_like(s)
    dgu = hip.swiglu_bwd(gu, da, s_out=s2)
    assert _rel(dgu, ref.swiglu_bwd(gu, da)) < 1e-5 and torch.equal(s2, s)
    V, Vp = 1000, 1024
    lg = torch.randn(300, Vp, device=DEV) * 3
    tg = torch.randint(0, V, (300,), device=DEV)
    tg[::7] = -100
    nv = (tg != -100).sum()
    lg2 = lg.clone()
    loss = hip.cross_entropy_fwd_bwd(lg, tg, V, nv, 2.0)
    lr = ref.cross_entropy_fwd_bwd(lg2, tg, V, nv, 2.0)
    assert _rel(loss, lr) < 1e-5 and _rel(lg, lg2) < 1e-5
    assert float(lg[:, V:].abs().max()) == 0.0
    x = torch.randn(1000, device=DEV)
    assert torch.allclose(hip.scale_bf16(x, torch.tensor(0.25, device=DEV), mul=2.0), x * 0.5)


@pytest.mark.parametrize("impl", ["flash", "gemm"])
@pytest.mark.parametrize("hd,S,p", [(64, 256, 0.0), (64, 200, 0.1), (128, 160, 0.1), (64, 1100, 0.1)])
def test_f32_attention_packed_vs_reference(hd, S, p, impl, monkeypatch):
    """fp32 attention fwd + bwd (packed QKV, inverse RoPE of the gradient) against the fp32
    reference with the same dropout keep bits; ragged S (not a tile multiple), both the
    flash kernels and the GEMM formulation (S 1100: 5 keys per softmax thread)."""
    from distributed_llm_trainer_amd.ops import hip_f32
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", impl)
    torch.manual_seed(hd + S)
    B, nh = 2, 3
    H = nh * hd
    qkv = torch.randn(B * S, 3 * H, device=DEV) * 0.5
    cos, sin = hip.rope_tables(hd, S, device=DEV)
    o, aux = hip.attention_fwd_packed(qkv, B, S, nh, p, 4242)
    orf, lser = ref.attention_fwd_packed(qkv, B, S, nh, p, 4242)
    assert o.dtype == torch.float32
    assert _rel(o, orf) < 2e-5, _rel(o, orf)
    assert _rel(aux[0], lser) < 2e-5
    do = torch.randn(B * S, H, device=DEV)
    g = hip.attention_bwd_packed(qkv, o, do, aux, p, 4242, B, S, nh, cos, sin)
    gr = ref.attention_bwd_packed(qkv, orf, do, lser, p, 4242, B, S, nh, cos, sin)
    assert _rel(g, gr) < 5e-5, _rel(g, gr)


@pytest.mark.parametrize("impl,hd", [("flash", 64), ("gemm", 64), ("gemm", 96), ("gemm-planner", 64)])
def test_f32_attention_head_major(impl, hd, monkeypatch):
    """Head-major fp32 attention vs the reference: flash kernels, the GEMM formulation
    (torch.matmul products; "gemm-planner": the autotuned planner's batched GEMMs)."""
    from distributed_llm_trainer_amd.ops import hip_f32
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", impl.split("-")[0])
    monkeypatch.setattr(hip_f32, "BMM_PLANNER", impl.endswith("planner"))
    torch.manual_seed(9)
    B, nh, S = 2, 2, 130
    q, k, v = (torch.randn(B, nh, S, hd, device=DEV) for _ in range(3))
    o, aux = hip.attention_fwd(q, k, v, 0.1, 99)
    orf, lser = ref.attention_fwd(q, k, v, 0.1, 99)
    assert _rel(o, orf) < 2e-5
    do = torch.randn(B * S, nh * hd, device=DEV)
    got = hip.attention_bwd(q, k, v, o, do, aux, 0.1, 99)
    want = ref.attention_bwd(q, k, v, orf, do, lser, 0.1, 99)
    for a, b in zip(got, want):
        assert _rel(a, b) < 5e-5


def test_fp32_training_runs_hip_kernels():
    """--mixed_precision fp32 builds the engine on the HIP op namespace (fp32 kernels, not
    the PyTorch reference ops) and trains: step-0 loss equal to the fp32 autograd model."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig(vocab_size=1000, hidden_size=256, num_layers=2, num_heads=4, max_seq_len=256, dropout=0.1,
                    attention_dropout=0.1)
    torch.manual_seed(5)
    tr = DistributedTrainer(cfg, TrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1,
                                                learning_rate=3e-3, mixed_precision="fp32"))
    assert tr.dtype == torch.float32 and tr.model.engine.ops.backend == "hip"
    data = torch.randint(0, 1000, (4, 256), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    losses = [tr.train_step({"input_ids": data})["loss"] for _ in range(5)]
    assert all(l == l for l in losses) and losses[-1] < losses[0], losses


@pytest.mark.parametrize("dt,hd,pad", [(torch.bfloat16, 48, True), (torch.float16, 80, True), (torch.bfloat16, 40, True),
                                       (torch.bfloat16, 48, False), (torch.float16, 80, False),
                                       (torch.bfloat16, 40, False), (torch.bfloat16, 160, True), (torch.float32, 32, True),
                                       (torch.float32, 32, False), (torch.bfloat16, 36, True), (torch.float32, 96, True)])
def test_attn_gemm_odd_head_dims_vs_reference(dt, hd, pad, monkeypatch):
    """ops/attn_gemm.py (head_dims without a flash kernel) against the PyTorch reference
    attention (fp32 arithmetic on the same inputs, same keep bits), forward + backward +
    inverse RoPE, on every route: heads zero-padded onto the flash kernels (pad, head_dim
    < 128: 16-bit MFMA and fp32 VALU flash kernels), 16-bit GEMMs with fp32 scores
    (head_dim % 16 == 0: 48, 80, 160), the fp32 formulation on widened inputs (40 without
    padding; fp32 32 without padding); 36: the widened fp32 RoPE."""
    from distributed_llm_trainer_amd.ops import attn_gemm
    monkeypatch.setattr(attn_gemm, "PAD_FLASH", pad)
    torch.manual_seed(hd)
    B, nh, S, p = 2, 3, 200, 0.1
    H = nh * hd
    qkv = (torch.randn(B * S, 3 * H, device=DEV) * 0.5).to(dt)
    cos, sin = hip.rope_tables(hd, S, device=DEV)
    assert attn_gemm.fits(B, nh, S, hd)
    assert (attn_gemm.pad_dim(dt, hd) is not None) == (pad and hd < 128)
    assert attn_gemm.use16(dt, B, nh, S, hd) == (dt != torch.float32 and hd % 16 == 0)
    o, aux = attn_gemm.attention_fwd_packed(qkv, B, S, nh, p, 77)
    orf, lser = ref.attention_fwd_packed(qkv, B, S, nh, p, 77)
    if hd % 16:  # the ops namespace's RoPE for this head_dim (widened onto the fp32 kernel)
        qr = qkv.clone()
        attn_gemm.rope_qk_inplace(qr, B, S, nh, cos, sin)
        want = ref.rope_qk_inplace(qkv.clone(), B, S, nh, cos, sin)
        assert _rel(qr, want) < (1e-6 if dt == torch.float32 else 8e-3)
    assert o.dtype == dt
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _rel(o, orf) < tol, _rel(o, orf)
    assert _rel(aux[0], lser) < 2e-5
    do = torch.randn(B * S, H, device=DEV).to(dt)
    g = attn_gemm.attention_bwd_packed(qkv, o, do, aux, p, 77, B, S, nh, cos, sin)
    gr = ref.attention_bwd_packed(qkv, orf, do, lser, p, 77, B, S, nh, cos, sin)
    assert g.dtype == dt and g.shape == qkv.shape
    assert _rel(g, gr) < (5e-5 if dt == torch.float32 else 2e-2), _rel(g, gr)


@pytest.mark.parametrize("dt,hd,S", [(torch.bfloat16, 40, 5000), (torch.float32, 40, 5000), (torch.bfloat16, 160, 4200)])
def test_attn_long_rows_native_route(dt, hd, S, monkeypatch):
    """Rows past the register-resident softmax (> 4096 keys) on head dims without a flash
    kernel stay native: head_dim 40 (bf16 / fp32) zero-padded onto the flash kernels, head
    dim 160 on the GEMM route with the long-row softmax kernel; the reference-op functions
    are made to raise, so a silent fallback would fail the test."""
    from distributed_llm_trainer_amd.ops import attn_gemm, reference
    for name in ("attention_fwd_packed", "attention_bwd_packed", "attention_fwd", "attention_bwd", "rope_qkv_bwd",
                 "rope_qk_inplace"):
        monkeypatch.setattr(reference, name, lambda *a, **k: (_ for _ in ()).throw(AssertionError("reference op")))
    torch.manual_seed(S)
    B, nh, p = 1, 2, 0.1
    H = nh * hd
    assert (attn_gemm.pad_dim(dt, hd) is not None) == (hd < 128)
    qkv = (torch.randn(B * S, 3 * H, device=DEV) * 0.5).to(dt)
    cos, sin = hip.rope_tables(hd, S, device=DEV)
    o, aux = attn_gemm.attention_fwd_packed(qkv, B, S, nh, p, 5)
    do = torch.randn(B * S, H, device=DEV).to(dt)
    g = attn_gemm.attention_bwd_packed(qkv, o, do, aux, p, 5, B, S, nh, cos, sin)
    monkeypatch.undo()
    orf, lser = ref.attention_fwd_packed(qkv, B, S, nh, p, 5)
    gr = ref.attention_bwd_packed(qkv, orf, do, lser, p, 5, B, S, nh, cos, sin)
    tol = (2e-5, 5e-5) if dt == torch.float32 else (1e-2, 2e-2)
    assert _rel(o, orf) < tol[0], _rel(o, orf)
    assert _rel(aux[0], lser) < 2e-5
    assert _rel(g, gr) < tol[1], _rel(g, gr)


@pytest.mark.parametrize("dt,pad", [(torch.bfloat16, False), (torch.float16, False), (torch.bfloat16, True)])
def test_attn_gemm_16bit_head_major(dt, pad, monkeypatch):
    """The head-major attn_gemm entry points at head_dim 96: 16-bit GEMM route, and the
    zero-padded flash route."""
    from distributed_llm_trainer_amd.ops import attn_gemm
    monkeypatch.setattr(attn_gemm, "PAD_FLASH", pad)
    torch.manual_seed(3)
    B, nh, S, hd = 2, 2, 130, 96
    q, k, v = ((torch.randn(B, nh, S, hd, device=DEV) * 0.5).to(dt) for _ in range(3))
    assert attn_gemm.use16(dt, B, nh, S, hd)
    o, aux = attn_gemm.attention_fwd(q, k, v, 0.1, 99)
    orf, lser = ref.attention_fwd(q, k, v, 0.1, 99)
    assert o.dtype == dt and _rel(o, orf) < 1e-2
    do = torch.randn(B * S, nh * hd, device=DEV).to(dt)
    got = attn_gemm.attention_bwd(q, k, v, o, do, aux, 0.1, 99)
    want = ref.attention_bwd(q, k, v, orf, do, lser, 0.1, 99)
    for a, b in zip(got, want):
        assert a.dtype == dt and _rel(a, b) < 2e-2, _rel(a, b)
