"""Micro-step pipelining (``GPTEngine.train_window``): the forward of micro-step k+1
interleaved block by block with the backward of micro-step k must give exactly the
gradients, losses and dropout masks of the sequential schedule.  Also covers the
packed-QKV attention path of the CPU reference ops against the split q/k/v path."""
import copy
import os

import pytest
import torch

from distributed_llm_trainer_amd.models import GPT, GPTConfig
from distributed_llm_trainer_amd.models.engine import shift_targets
from distributed_llm_trainer_amd.ops import reference as ref


def tiny(**kw):
    d = dict(vocab_size=256, hidden_size=64, num_layers=3, num_heads=4, max_seq_len=32, dropout=0.1,
             attention_dropout=0.1)
    d.update(kw)
    return GPTConfig(**d)


@pytest.mark.parametrize("GA,recompute,chunks", [(2, False, 0), (3, False, 0), (4, True, 0), (2, False, 2),
                                                  (3, True, 1), (2, False, 3)])
def test_train_window_matches_sequential(GA, recompute, chunks):
    """chunks > 0: the chunked lm_head (GPTEngine.head_chunks) -- run in the window's
    forwards ("early head") vs from the kept logits in the sequential backward."""
    torch.manual_seed(11)
    m1 = GPT(tiny())
    m2 = copy.deepcopy(m1)
    e1 = m1.enable_engine(seed=5)
    e2 = m2.enable_engine(seed=5)
    e1.head_chunks = e2.head_chunks = chunks
    m1.gradient_checkpointing = m2.gradient_checkpointing = recompute
    m1.train()
    m2.train()
    data = torch.randint(0, 256, (GA, 2, 32))
    seq = []
    for j in range(GA):
        e1.set_accumulation(j, GA, defer=True)
        _, loss = m1(data[j], labels=data[j])
        (loss / GA).backward()
        seq.append(loss.detach())
    dloss = torch.full((), 1.0 / GA)
    win = e2.train_window([data[j] for j in range(GA)], [shift_targets(data[j]) for j in range(GA)], dloss,
                          recompute=recompute)
    assert e1.micro_counter == e2.micro_counter == GA
    for a, b in zip(seq, win):
        assert torch.equal(a, b)
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p1.grad, p2.grad, atol=1e-7, rtol=1e-6), n


def test_train_window_single_micro_step_is_plain_step():
    torch.manual_seed(12)
    m1 = GPT(tiny(dropout=0.0, attention_dropout=0.0))
    m2 = copy.deepcopy(m1)
    e1 = m1.enable_engine(seed=1)
    e2 = m2.enable_engine(seed=1)
    ids = torch.randint(0, 256, (2, 32))
    e1.set_accumulation(0, 1)
    _, loss = m1(ids, labels=ids)
    loss.backward()
    (l2,) = e2.train_window([ids], [shift_targets(ids)], torch.ones(()))
    assert torch.equal(loss.detach(), l2)
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p1.grad, p2.grad, atol=1e-7, rtol=1e-6), n


def test_trainer_pipelined_step_matches_sequential():
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    torch.manual_seed(13)
    data = torch.randint(0, 256, (8, 32))
    res = []
    for pipe in (False, True):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            pipeline_micro_steps=pipe)
        tr = DistributedTrainer(tiny(), tc)
        losses = [tr.train_step({"input_ids": data})["loss"] for _ in range(3)]
        res.append((losses, tr.flat_params().clone()))
    assert res[0][0] == res[1][0]
    assert torch.allclose(res[0][1], res[1][1], atol=1e-7, rtol=1e-6)


@pytest.mark.parametrize("recompute", [False, True])
def test_trainer_memory_lean_matches_deferred(recompute):
    """Per-role deferral: --memory_lean (defer_roles 'qkv,o': gate/up, down and lm_head
    weight gradients in each pipelined chain's own backward), single roles, and no
    deferral at all (defer_wgrad=False, no slot buffers) train like the default deferred
    schedule (same sums in another order: allclose, not bitwise)."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import LEAN_DEFER_ROLES, DistributedTrainer
    torch.manual_seed(14)
    data = torch.randint(0, 256, (8, 32))
    res = []
    variants = [(True, "all"), (True, LEAN_DEFER_ROLES), (True, "qkv,o"), (True, "gu,head"), (True, "down"),
                (False, "all")]
    for defer, roles in variants:
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            defer_wgrad=defer, defer_roles=roles)
        cfg = tiny()
        cfg.gradient_checkpointing = recompute
        tr = DistributedTrainer(cfg, tc)
        losses = [tr.train_step({"input_ids": data})["loss"] for _ in range(3)]
        res.append((losses, tr.flat_params().clone()))
        slots = {name for (_, name) in tr.model.engine._slots}
        if not defer:
            assert not slots  # nothing deferred, no slot buffers
        elif roles == LEAN_DEFER_ROLES:
            assert not slots, slots  # --memory_lean defers nothing
        elif roles == "qkv,o":
            assert slots == {"n1", "dqkv", "o", "da"}, slots
    for losses, flat in res[1:]:
        for a, b in zip(res[0][0], losses):
            assert abs(a - b) < 1e-5
        assert torch.allclose(res[0][1], flat, atol=1e-6, rtol=1e-5)


def test_defer_roles_parse():
    from distributed_llm_trainer_amd.training.ddp_trainer import parse_defer_roles
    assert parse_defer_roles("all") == {"qkv", "o", "gu", "down", "head"}
    assert parse_defer_roles(" qkv , o") == {"qkv", "o"}
    with pytest.raises(ValueError):
        parse_defer_roles("qkv,mlp")


def test_packed_qkv_reference_matches_split():
    torch.manual_seed(14)
    B, S, nh, hd = 2, 24, 3, 16
    qkv = torch.randn(B * S, 3 * nh * hd, dtype=torch.float64).float()
    cos, sin = ref.rope_tables(hd, 32)
    q, k, v = ref.rope_qkv_fwd(qkv, B, S, nh, cos, sin)
    o1, l1 = ref.attention_fwd(q, k, v, 0.1, 77)
    packed = ref.rope_qk_inplace(qkv.clone(), B, S, nh, cos, sin)
    o2, l2 = ref.attention_fwd_packed(packed, B, S, nh, 0.1, 77)
    assert torch.allclose(o1, o2, atol=1e-6) and torch.allclose(l1, l2, atol=1e-6)
    do = torch.randn_like(o1)
    dq, dk, dv = ref.attention_bwd(q, k, v, o1, do, l1, 0.1, 77)
    d1 = ref.rope_qkv_bwd(dq, dk, dv, cos, sin)
    d2 = ref.attention_bwd_packed(packed, o2, do, l2, 0.1, 77, B, S, nh, cos, sin)
    assert torch.allclose(d1, d2, atol=1e-6)


def test_engine_packed_matches_split_path(monkeypatch):
    torch.manual_seed(15)
    base = GPT(tiny())
    grads = []
    for packed in ("1", "0"):
        monkeypatch.setenv("DLT_PACKED_QKV", packed)
        m = copy.deepcopy(base)
        e = m.enable_engine(seed=2)
        assert e.packed_qkv == (packed == "1")
        ids = torch.randint(0, 256, (2, 32), generator=torch.Generator().manual_seed(3))
        _, loss = m(ids, labels=ids)
        loss.backward()
        grads.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*grads):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("sync_every", [True, False])
@pytest.mark.parametrize("strategy", ["FULL_SHARD", "SHARD_GRAD_OP"])
def test_fsdp_trainer_pipelined_matches_sequential(strategy, sync_every):
    """The FSDP runtime under the pipelined window (reference-counted unit residency,
    per-micro-step or deferred reduce) == its sequential schedule."""
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    torch.manual_seed(16)
    data = torch.randint(0, 256, (8, 32))
    res = []
    for pipe in (False, True):
        tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                                pipeline_micro_steps=pipe)
        fc = FSDPConfig(sharding_strategy=strategy, sync_every_micro_step=sync_every)
        tr = FSDPTrainer(tiny(), tc, fc)
        losses = [tr.train_step({"input_ids": data})["loss"] for _ in range(3)]
        res.append((losses, tr.runtime.state_dict_full()))
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert torch.allclose(res[0][1][k], res[1][1][k], atol=1e-7, rtol=1e-6), k


@pytest.mark.parametrize("F,pipe,chunks", [(2, True, None), (2, False, None), (4, True, None), (2, True, "2"),
                                           (4, True, "1")])
def test_micro_step_fusion_matches_unfused(F, pipe, chunks, monkeypatch):
    """micro_step_fusion=F executes F micro-steps as one chain of F*batch rows: the
    trainer step equals the unfused GA average (dropout off: fused chains draw other
    dropout streams by design).  Ragged ignore_index counts: the next test.  chunks:
    the chunked lm_head (DLT_HEAD_CHUNKS; per-segment chunks when fewer are asked)."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    if chunks is not None:
        monkeypatch.setenv("DLT_HEAD_CHUNKS", chunks)
    torch.manual_seed(14)
    data = torch.randint(0, 256, (8, 32))
    res = []
    for fuse in (1, F):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            pipeline_micro_steps=pipe, micro_step_fusion=fuse)
        tr = DistributedTrainer(tiny(dropout=0.0, attention_dropout=0.0), tc)
        assert tr.fusion_factor(4, 2, 32) == fuse
        losses = [tr.train_step({"input_ids": data})["loss"] for _ in range(3)]
        res.append((losses, tr.flat_params().clone()))
    for a, b in zip(res[0][0], res[1][0]):
        assert abs(a - b) < 1e-5 * max(1.0, abs(a)), (a, b)
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6, rtol=1e-5)


def test_fused_loss_segments_normalise_per_micro_step():
    """Engine-level check with ignore_index: a fused forward over two micro-steps whose
    valid-target counts differ gives mean(loss_0, loss_1) and the gradient of
    (loss_0 + loss_1) / 2 -- not the pooled token mean."""
    torch.manual_seed(15)
    m1 = GPT(tiny(dropout=0.0, attention_dropout=0.0))
    m2 = copy.deepcopy(m1)
    e1 = m1.enable_engine(seed=3)
    e2 = m2.enable_engine(seed=3)
    ids = torch.randint(0, 256, (4, 32))
    tg = shift_targets(ids)
    tg[:40] = -100  # micro-step 0 (rows 0-63) keeps 23 targets, micro-step 1 keeps 31
    # unfused reference: two micro-steps of 2 sequences
    e1.set_accumulation(0, 2, defer=False)
    losses = []
    for j in range(2):
        loss, _, st = e1.forward(ids[2 * j:2 * j + 2], tg[64 * j:64 * (j + 1)], train=True, need_backward=True)
        e1.backward(st, torch.full((), 0.5))
        losses.append(loss)
    e2.set_loss_segments(2)
    e2.set_accumulation(0, 1, defer=False)
    loss2, _, st2 = e2.forward(ids, tg, train=True, need_backward=True)
    e2.backward(st2, torch.ones(()))
    assert torch.allclose(loss2, (losses[0] + losses[1]) / 2, atol=1e-6)
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.allclose(p1.grad, p2.grad, atol=1e-6, rtol=1e-5), n


def test_window_auto_choice(monkeypatch):
    """Under gradient collectives the window schedule is chosen by timing: the first four
    pipelined windows run fb, ffbb, fb, ffbb; at the next entry the faster schedule's best
    whole-step time wins and is kept (stubbed GPU events; the max over ranks is the
    identity on one rank)."""
    import types
    for k in ("DLT_WINDOW_SCHED", "DLT_BWD_OVERLAP", "DLT_QUEUE_PROBE", "DLT_WINDOW_AUTO"):
        monkeypatch.delenv(k, raising=False)
    e = GPT(tiny()).enable_engine(seed=1)
    e.provider.hooks = types.SimpleNamespace(collectives=True)

    def run(step_ms):
        stamps = iter([sum(step_ms[:i]) for i in range(len(step_ms) + 1)] + [1e9] * 8)

        class Ev:
            def __init__(self, enable_timing=False):
                self.t = None

            def record(self, stream=None):
                self.t = next(stamps)

            def synchronize(self):
                pass

            def elapsed_time(self, other):
                return other.t - self.t
        monkeypatch.setattr(torch.cuda, "Event", Ev)
        monkeypatch.setattr(torch.cuda, "current_stream", lambda dev=None: None)
        dev = types.SimpleNamespace(type="cuda")
        e.window_auto = None
        seq = []
        for _ in range(7):
            _, s = e.window_schedule(2, True, cuda=True)
            if e._auto_enter(dev):
                _, s = e.window_schedule(2, True, cuda=True)
            seq.append(s)
        return seq
    # first windows of each kind carry one-time costs: the best of two decides
    assert run([45.0, 44.0, 41.6, 41.2, 40.0, 40.0]) == ["fb", "ffbb", "fb", "ffbb", "ffbb", "ffbb", "ffbb"]
    assert e.window_auto["decided"] == "ffbb" and e.window_auto["ms"] == {"fb": 41.6, "ffbb": 41.2}
    assert run([45.0, 47.0, 41.6, 46.0, 40.0, 40.0]) == ["fb", "ffbb", "fb", "ffbb", "fb", "fb", "fb"]
    monkeypatch.setenv("DLT_WINDOW_AUTO", "0")
    e.window_auto = None
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")
    assert e.window_auto is None


def test_window_schedule_choice(monkeypatch):
    """Two-chain window schedule: ffbb only with overlapped backwards, two chains, every
    weight gradient deferred, a GPT-2-small-sized model, and with gradient collectives in
    flight only on verified stream placement; fb otherwise (profiles/r3_window_ffbb.md,
    r5_stream_queues.md)."""
    import types
    monkeypatch.delenv("DLT_WINDOW_SCHED", raising=False)
    monkeypatch.delenv("DLT_BWD_OVERLAP", raising=False)
    torch.manual_seed(0)
    m = GPT(tiny())
    e = m.enable_engine(seed=1)
    assert getattr(e.provider, "overlap_backward_ok", False)
    assert e.window_schedule(2, True, cuda=True) == (True, "ffbb")
    assert e.window_schedule(4, True, cuda=True) == (True, "fb")          # more than two chains
    assert e.window_schedule(2, False, cuda=True) == (True, "fb")         # per-micro-step weight grads
    assert e.window_schedule(2, True, cuda=False) == (False, "fb")        # no streams on the CPU
    e.defer_roles = frozenset(("qkv", "o"))                               # memory-lean
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")
    e.defer_roles = frozenset(e.ROLES)
    # DDP buckets in flight: fb, and ffbb only with the opt-in placement probe verifying
    # the side streams' hardware queues (Engine._place_streams; stubbed here, no GPU)
    monkeypatch.setenv("DLT_QUEUE_PROBE", "1")
    placement = {"verified": False}

    def fake_place(dev):
        e.queue_placement = dict(placement)
    monkeypatch.setattr(e, "_place_streams", fake_place)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)  # no GPU here: only the index is read
    e.provider.hooks = types.SimpleNamespace(collectives=True)
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")
    placement["verified"] = True
    assert e.window_schedule(2, True, cuda=True) == (True, "ffbb")
    monkeypatch.delenv("DLT_QUEUE_PROBE")
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")             # default: first timed trial
    placement["verified"] = False
    e.provider.hooks = types.SimpleNamespace(collectives=False)
    monkeypatch.setenv("DLT_BWD_OVERLAP", "0")
    assert e.window_schedule(2, True, cuda=True) == (False, "fb")
    monkeypatch.delenv("DLT_BWD_OVERLAP")
    monkeypatch.setenv("DLT_WINDOW_SCHED", "fb")
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")
    monkeypatch.delenv("DLT_WINDOW_SCHED")
    # a provider that reports its own collectives (FSDPRuntime.collectives) keeps fb too
    e.provider.hooks = None
    e.provider.collectives = True
    assert e.window_schedule(2, True, cuda=True) == (True, "fb")


def test_wgrad_set_and_acc_contracts():
    """wgrad_acc accumulates into fp32 and refuses bf16; wgrad_set overwrites a bf16
    buffer (both GEMM backends: the FSDP bf16 send-buffer mode must not depend on which
    one the engine uses)."""
    from distributed_llm_trainer_amd.models.engine import _TorchGemm, _wgrad
    g = _TorchGemm()
    torch.manual_seed(0)
    dy, x = torch.randn(64, 24), torch.randn(64, 16)
    ref_ = dy.t() @ x
    acc = torch.ones(24, 16)
    g.wgrad_acc(acc, dy, x)
    assert torch.allclose(acc, 1 + ref_, atol=1e-4)
    db = torch.full((24, 16), float("nan"), dtype=torch.bfloat16)
    _wgrad(g, db, dy.bfloat16(), x.bfloat16())
    assert torch.isfinite(db.float()).all()
    assert (db.float() - ref_).norm() / ref_.norm() < 2e-2
    with pytest.raises(ValueError):
        g.wgrad_acc(db, dy.bfloat16(), x.bfloat16())


def test_lazy_optimizer_step_matches_end_of_step_update(tmp_path):
    """The recorded optimizer step (TrainingConfig.lazy_optimizer: each unit's AdamW +
    gradient zeroing launched by the next forward's pre_forward hook) trains bitwise like
    the reference's end-of-step update: same losses, weights, AdamW moments; state_dict,
    checkpoints and generation flush a pending step first."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    torch.manual_seed(15)
    data = [torch.randint(0, 256, (8, 32)) for _ in range(4)]
    res = []
    for mode in ("off", "inline"):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            lazy_optimizer=mode)
        tr = DistributedTrainer(tiny(), tc)
        losses = [tr.train_step({"input_ids": d})["loss"] for d in data]
        if mode == "inline":
            assert tr.store.pending is not None and not tr.store.pending.complete
            sd = tr.model.state_dict()  # the state_dict pre-hook flushes the pending step
            assert tr.store.pending is None
            assert float(tr.store.grad.abs().max()) == 0.0  # gradients zeroed by the unit updates
        else:
            sd = tr.model.state_dict()
        res.append((losses, tr.flat_params().clone(), tr.optimizer.exp_avg.clone(), tr.optimizer.exp_avg_sq.clone(),
                    {k: v.clone() for k, v in sd.items()}))
    (l0, f0, m0, v0, s0), (l1, f1, m1, v1, s1) = res
    assert l0 == l1
    assert torch.equal(f0, f1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert all(torch.equal(s0[k], s1[k]) for k in s0)
    # a checkpoint taken with a step pending holds the updated weights
    tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                        lazy_optimizer="inline", checkpoint_dir=str(tmp_path))
    tr = DistributedTrainer(tiny(), tc)
    for d in data:
        tr.train_step({"input_ids": d})
    tr.save_checkpoint(str(tmp_path / "c.pt"))
    from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint
    c = load_checkpoint(str(tmp_path / "c.pt"))
    assert torch.equal(c["model"]["norm.weight"], s0["norm.weight"])
    assert torch.equal(c["model"]["layers.1.mlp.down_proj.weight"], s0["layers.1.mlp.down_proj.weight"])


def test_lazy_optimizer_never_replays_onto_loaded_weights():
    """Weights loaded (model.load_state_dict, utils.checkpoint.load_model_state) or written
    into the master and re-derived (refresh_shadow) while a lazy optimizer step is pending
    are final: the next forward must not apply the stale update on top of them.  The
    optimizer's state_dict reports the moments of its step count (the pending step is
    applied first)."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    from distributed_llm_trainer_amd.utils.checkpoint import load_model_state
    torch.manual_seed(16)
    data = [torch.randint(0, 256, (8, 32)) for _ in range(3)]

    def trained(mode):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            lazy_optimizer=mode)
        tr = DistributedTrainer(tiny(), tc)
        for d in data[:2]:
            tr.train_step({"input_ids": d})
        return tr

    ref_tr = trained("off")
    ref_sd = {k: v.clone() for k, v in ref_tr.model.state_dict().items()}
    ref_m = ref_tr.optimizer.exp_avg.clone()
    # optimizer state_dict with a step pending: the moments of step_count
    tr = trained("inline")
    assert tr.store.pending is not None and not tr.store.pending.complete
    osd = tr.optimizer.state_dict()
    assert all(int(s["step"]) == ref_tr.optimizer.step_count for s in osd["state"].values())
    assert torch.equal(tr.optimizer.exp_avg, ref_m)
    # load_state_dict with a step pending, for both load entry points
    other = {k: torch.randn_like(v) if v.dtype.is_floating_point else v for k, v in ref_sd.items()}
    if "lm_head.weight" in other:  # tied: one tensor
        other["lm_head.weight"] = other["embed_tokens.weight"]
    for load in (lambda m, sd: m.load_state_dict(sd), load_model_state):
        tr = trained("inline")
        assert tr.store.pending is not None and not tr.store.pending.complete
        load(tr.model, other)
        tr.store.refresh_shadow()
        tr.train_step({"input_ids": data[2]})  # its forward runs every unit's pre_forward hook
        sd = tr.model.state_dict()  # flushes the step this train_step recorded: compare before
        # the new step is applied: re-load and take the parameters straight from the store
        tr2 = trained("inline")
        load(tr2.model, other)
        tr2.store.refresh_shadow()
        tr2.train_step({"input_ids": data[2]})
        for k in ("norm.weight", "layers.1.mlp.down_proj.weight", "embed_tokens.weight"):
            seg = tr2.store.layout.by_name[k]
            got = tr2.store.flat[seg.offset:seg.offset + seg.numel].view(seg.shape)
            assert torch.equal(got, other[k].to(got.dtype)), k  # loaded weights untouched by the old step
        assert set(sd) == set(other)
    # external edit of the master + refresh_shadow: the edit is final, the pending step is dropped
    tr = trained("inline")
    edited = torch.randn_like(tr.store.flat)
    tr.store.flat.copy_(edited)
    tr.store.refresh_shadow()
    assert tr.store.pending is None and float(tr.store.grad.abs().max()) == 0.0
    tr.train_step({"input_ids": data[2]})
    assert torch.equal(tr.store.flat, edited)


def test_f32_attention_impl_choice(monkeypatch):
    """fp32 attention picks the GEMM formulation while its two [B*nh, S, S] score buffers fit
    and S <= 4096, else the flash kernels; a forced "gemm" beyond the limits is an error."""
    from distributed_llm_trainer_amd.ops import hip_f32
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", "auto")
    assert hip_f32._use_gemm(16, 12, 1024, 64)
    assert not hip_f32._use_gemm(1, 12, 8192, 64)  # rows longer than the softmax kernel takes
    assert not hip_f32._use_gemm(256, 32, 2048, 128)  # 2 x 128 GiB of scores
    assert not hip_f32._use_gemm(2, 2, 64, 512)
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", "flash")
    assert not hip_f32._use_gemm(16, 12, 1024, 64)
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", "gemm")
    with pytest.raises(ValueError):
        hip_f32._use_gemm(1, 12, 8192, 64)
    monkeypatch.setattr(hip_f32, "ATTN_IMPL", "bogus")
    with pytest.raises(ValueError):
        hip_f32._use_gemm(1, 1, 64, 64)


def test_attn_gemm_routes(monkeypatch):
    """Head dims without a flash kernel: heads under 128 pad to 64 / 128 (16-bit: any
    head_dim; fp32: even ones), head_dim >= 128 and DLT_ATTN_PAD=0 do not pad; the GEMM
    formulation takes rows of any length and raises (no silent fallback) past its score
    buffer budget."""
    from distributed_llm_trainer_amd.ops import attn_gemm
    monkeypatch.setattr(attn_gemm, "PAD_FLASH", True)
    assert attn_gemm.pad_dim(torch.bfloat16, 32) == 64 and attn_gemm.pad_dim(torch.float16, 48) == 64
    assert attn_gemm.pad_dim(torch.bfloat16, 96) == 128 and attn_gemm.pad_dim(torch.bfloat16, 80) == 128
    assert attn_gemm.pad_dim(torch.bfloat16, 160) is None and attn_gemm.pad_dim(torch.float32, 96) == 128
    assert attn_gemm.pad_dim(torch.bfloat16, 36) == 64 and attn_gemm.pad_dim(torch.float32, 40) == 64
    assert attn_gemm.pad_dim(torch.float32, 35) is None
    monkeypatch.setattr(attn_gemm, "PAD_FLASH", False)
    assert attn_gemm.pad_dim(torch.bfloat16, 96) is None
    assert attn_gemm.fits(16, 12, 1024, 96) and attn_gemm.fits(1, 1, 8192, 96) and attn_gemm.fits(1, 1, 64, 258)
    monkeypatch.setattr(attn_gemm, "GEMM_ROUTE_BYTES", 1 << 20)
    assert not attn_gemm.fits(1, 1, 8192, 160)
    with pytest.raises(NotImplementedError, match="DLT_ATTN_GEMM_GB"):
        attn_gemm._need_fit(1, 1, 8192, 160)
    import inspect
    assert "reference." not in inspect.getsource(attn_gemm).split('"""', 2)[2]  # no reference-op route

def test_memory_first_matches_memory_lean():
    """TrainingConfig.memory_first (lean + unfused micro-steps + the SwiGLU output rewritten
    by the backward instead of kept): same losses and weights as --memory_lean, bitwise on
    the CPU ops (s is recomputed from the kept gu with the forward's arithmetic)."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import LEAN_DEFER_ROLES, DistributedTrainer
    torch.manual_seed(17)
    data = [torch.randint(0, 256, (8, 32)) for _ in range(3)]
    res = []
    for first in (False, True):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            defer_roles=LEAN_DEFER_ROLES, micro_step_fusion=1, memory_first=first)
        tr = DistributedTrainer(tiny(), tc)
        assert tr.model.engine.s_refill == first
        # memory-first takes a micro-step's head rows in one chunk, lean in two: same chunking
        # here, so the only difference left is the SwiGLU output's refill
        assert tr.model.engine.head_chunks == (1 if first else 2)
        tr.model.engine.head_chunks = 1
        losses = [tr.train_step({"input_ids": d})["loss"] for d in data]
        res.append((losses, tr.flat_params().clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_partial_layer_deferral_matches_inline():
    """GPTEngine.defer_layers (DLT_DEFER_LAYERS): only layers below it defer their roles'
    weight gradients to the window.  --memory_first --defer_roles o with the o weight
    gradient deferred for layer 0 only: same losses, and weights within summation-order
    noise of deferring it for every layer and of deferring nothing."""
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    torch.manual_seed(23)
    data = [torch.randint(0, 256, (8, 32)) for _ in range(3)]
    res = {}
    for name, roles, layers in (("none", "none", 0), ("all", "o", 0), ("part", "o", 1)):
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=2, max_steps=10,
                            defer_roles=roles, memory_first=True)
        tr = DistributedTrainer(tiny(), tc)
        tr.model.engine.defer_layers = layers
        losses = [tr.train_step({"input_ids": d})["loss"] for d in data]
        res[name] = (losses, tr.flat_params().clone())
    for name in ("all", "part"):
        assert res[name][0][0] == res["none"][0][0]
        torch.testing.assert_close(res[name][1], res["none"][1], rtol=1e-5, atol=1e-6)
