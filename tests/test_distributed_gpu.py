"""Multi-rank DDP / FSDP on the GPU: two ranks share the one MI355X of the test box
(gloo carries the collectives -- RCCL itself needs one GPU per rank), running the fused
HIP engine with micro-step pipelining, side-stream gradient buckets and FSDP unit
residency exactly as on a multi-GPU node.  Each run is compared with one process that
consumes every rank's micro-batches (GA = 2 x world):

* ranks hold bit-identical parameters after every step (the all-reduce / gather worked),
* the global gradient norm of every step matches the single process (gradients were
  averaged over the right set, once),
* the parameter updates point the same way (cosine of the deltas).

bf16 GEMMs over a different micro-batch split change the fp32 accumulation order, so
the comparisons are relative, not bitwise (the CPU versions in
``test_distributed_cpu.py`` are bitwise-tight)."""
import os

import pytest
import torch

from tests.dist_utils import run_multiprocess

pytestmark = pytest.mark.gpu

TINY = dict(vocab_size=1000, hidden_size=256, num_layers=3, num_heads=4, max_seq_len=256, dropout=0.0,
            attention_dropout=0.0)
GPU_ENV = {"DLT_FORCE_CPU": None, "DLT_SHARE_GPU": "1"}
STEPS = 3


def _cpu_dry_run():
    """DLT_FORCE_CPU=1 with GPU_ENV emptied runs the same logic on the CPU."""
    return os.environ.get("DLT_FORCE_CPU") == "1"


def _data(step, rank):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randint(0, TINY["vocab_size"], (4, TINY["max_seq_len"]), generator=g)


def _ddp(rank, world, single):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=2 * (world if single else 1), warmup_steps=1,
                        max_steps=100, learning_rate=1e-3, bucket_cap_mb=1.0)
    tr = DistributedTrainer(GPTConfig(**TINY), tc)
    assert tr.use_engine and (tr.device.type == "cuda" or _cpu_dry_run())
    init = tr.flat_params().detach().float().cpu().clone()
    norms = []
    for s in range(STEPS):
        batch = torch.cat([_data(s, r) for r in range(world)]) if single else _data(s, rank)
        tr.train_step({"input_ids": batch})
        norms.append(float(tr._last_norm))
    nb = len(tr.ddp.buckets) if tr.ddp is not None else 0
    return init, tr.flat_params().detach().float().cpu().clone(), norms, nb


def _fsdp(rank, world, single, strategy):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2 * (world if single else 1),
                            warmup_steps=1, max_steps=100, learning_rate=1e-3)
    fc = FSDPConfig(sharding_strategy=strategy)
    tr = FSDPTrainer(GPTConfig(**TINY), tc, fc)
    assert tr.device.type == "cuda" or _cpu_dry_run()

    def full():
        sd = tr._full_state()
        return torch.cat([v.detach().float().cpu().flatten() for k, v in sorted(sd.items()) if "rotary" not in k])

    init = full()
    norms = []
    for s in range(STEPS):
        batch = torch.cat([_data(s, r) for r in range(world)]) if single else _data(s, rank)
        tr.train_step({"input_ids": batch})
        norms.append(float(tr._last_norm))
    return init, full(), norms, 0


def _check(outs, ref):
    (i0, p0, n0, _), (i1, p1, n1, _) = outs
    ri, rp, rn, _ = ref
    assert torch.equal(i0, i1) and torch.equal(i0, ri), "initialisation differs"
    assert torch.equal(p0, p1), f"ranks diverged: {(p0 - p1).abs().max()}"
    for a, b in zip(n0, rn):
        assert abs(a - b) <= 2e-3 * abs(b), (n0, rn)
    assert n0 == n1
    d, dr = p0 - i0, rp - ri
    cos = torch.nn.functional.cosine_similarity(d, dr, dim=0).item()
    assert cos > 0.99, cos


def test_ddp_two_ranks_on_gpu_match_single_process():
    outs = run_multiprocess(_ddp, world=2, args=(False,), env=GPU_ENV, timeout=240)
    assert outs[0][3] > 2  # several gradient buckets were all-reduced from the side stream
    _check(outs, _ddp(0, 2, True))


@pytest.mark.parametrize("strategy", ["FULL_SHARD", "SHARD_GRAD_OP"])
def test_fsdp_two_ranks_on_gpu_match_single_process(strategy):
    outs = run_multiprocess(_fsdp, world=2, args=(False, strategy), env=GPU_ENV, timeout=240)
    _check(outs, _fsdp(0, 2, True, strategy))


# shapes every hand-written kernel tiles (M % 256, N % 192, K % 128: hidden 384, 3H 1152,
# 2I 3072, vocab 1152, 512-token micro-steps), so the shipped hand GEMM / wgrad / dgrad
# kernels feed the RCCL buckets in the forced-collectives rehearsal
HANDCFG = dict(vocab_size=1152, hidden_size=384, num_layers=2, num_heads=6, intermediate_size=1536,
               max_seq_len=256, dropout=0.0, attention_dropout=0.0)


def _forced(rank, world, mode):
    """One rank over RCCL; DLT_FORCE_COLLECTIVES=1 issues every bucket all-reduce /
    unit all-gather / reduce-scatter anyway (the multi-GPU code path on one GPU)."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    import torch.distributed as dist
    if mode == "ddp_hand":
        from distributed_llm_trainer_amd.training.configs import TrainingConfig
        from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
        from distributed_llm_trainer_amd.ops import gemm
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                            learning_rate=1e-3, bucket_cap_mb=2.0)
        tr = DistributedTrainer(GPTConfig(**HANDCFG), tc)
        assert tr.device.type == "cuda" and dist.get_backend() == "nccl"
        for s in range(STEPS):
            g = torch.Generator().manual_seed(77 + s)
            tr.train_step({"input_ids": torch.randint(0, HANDCFG["vocab_size"], (4, 256), generator=g)})
        rep = gemm.race_report()
        return {"flat": tr.flat_params().detach().float().cpu().clone()}, (tr.ddp.launched, rep)
    if mode == "ddp_auto":
        # enough steps for the timed fb / ffbb choice (first step unpipelined, four trial
        # windows, the decision at the next window's entry)
        from distributed_llm_trainer_amd.training.configs import TrainingConfig
        from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                            learning_rate=1e-3, bucket_cap_mb=2.0)
        tr = DistributedTrainer(GPTConfig(**HANDCFG), tc)
        assert tr.device.type == "cuda" and dist.get_backend() == "nccl"
        for s in range(7):
            g = torch.Generator().manual_seed(77 + s)
            tr.train_step({"input_ids": torch.randint(0, HANDCFG["vocab_size"], (4, 256), generator=g)})
        eng = tr.model.engine
        auto = dict(eng.window_auto) if eng.window_auto is not None else None
        return {"flat": tr.flat_params().detach().float().cpu().clone()}, (eng.last_window, auto)
    if mode == "fsdp_hand":
        from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
        from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
        from distributed_llm_trainer_amd.ops import gemm
        tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                                learning_rate=1e-3)
        tr = FSDPTrainer(GPTConfig(**HANDCFG), tc, FSDPConfig(sharding_strategy="FULL_SHARD"))
        assert tr.device.type == "cuda" and dist.get_backend() == "nccl"
        for s in range(STEPS):
            g = torch.Generator().manual_seed(77 + s)
            tr.train_step({"input_ids": torch.randint(0, HANDCFG["vocab_size"], (4, 256), generator=g)})
        rep = gemm.race_report()
        sd = {k: v.detach().float().cpu().clone() for k, v in tr._full_state().items() if "rotary" not in k}
        return sd, (1 if tr.runtime.force else 0, rep)
    if mode.startswith("ddp"):
        from distributed_llm_trainer_amd.training.configs import TrainingConfig
        from distributed_llm_trainer_amd.training.ddp_trainer import LEAN_DEFER_ROLES, DistributedTrainer
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=1, max_steps=100,
                            learning_rate=1e-3, bucket_cap_mb=1.0,
                            defer_roles=LEAN_DEFER_ROLES if mode == "ddp_lean" else "all",
                            reduce_dtype="bf16" if mode == "ddp_bf16" else "fp32")
        tr = DistributedTrainer(GPTConfig(**TINY), tc)
    else:
        from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
        from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
        tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=1, max_steps=100,
                                learning_rate=1e-3)
        tr = FSDPTrainer(GPTConfig(**TINY), tc, FSDPConfig(sharding_strategy="FULL_SHARD", reduce_dtype="fp32"))
    assert tr.device.type == "cuda" and dist.get_backend() == "nccl"
    for s in range(STEPS):
        tr.train_step({"input_ids": torch.cat([_data(s, 0), _data(s, 1)])})
    launched = tr.ddp.launched if mode.startswith("ddp") else -1
    sd = tr._full_state() if mode == "fsdp" else {"flat": tr.flat_params()}
    return {k: v.detach().float().cpu().clone() for k, v in sd.items() if "rotary" not in k}, launched


@pytest.mark.parametrize("mode", ["ddp_hand", "fsdp_hand"])
def test_rccl_forced_collectives_with_hand_kernels(tmp_path, mode):
    """The forced-collectives rehearsal with the SHIPPED kernel choices: every GEMM role
    races hand-written vs library as in production (first run, plan written), the second
    run replays that plan with DLT_FORCE_COLLECTIVES=1, so the hand wgrad / stream-K /
    dgrad kernels feed the RCCL bucket all-reduces (DDP) or the unit all-gathers and
    reduce-scatters (FSDP).  A 1-rank sum is the identity: parameters equal bit for bit."""
    plan = str(tmp_path / "plan.json")
    env = {"DLT_FORCE_CPU": None, "DLT_BACKEND": "nccl", "DLT_GEMM_PLAN": plan}
    a, (_, rep) = run_multiprocess(_forced, world=1, args=(mode,), env=env, timeout=300)[0]
    assert os.path.exists(plan)
    b, (launched, rep_b) = run_multiprocess(_forced, world=1, args=(mode,),
                                            env={**env, "DLT_FORCE_COLLECTIVES": "1"}, timeout=300)[0]
    assert launched > (2 if mode == "ddp_hand" else 0)
    assert rep == rep_b
    # the hand-written kernels are among the choices (shapes tile by construction)
    assert any("hand-written" in v or "fused gemm_bf16" in v for v in rep.values()), rep
    for k in a:
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())


def test_rccl_forced_collectives_timed_window_choice(tmp_path):
    """Under forced RCCL collectives the window schedule is chosen by timing (four trial
    windows fb / ffbb, then the faster one): the decision is taken and recorded, and the
    parameters equal bit for bit those of the run without a communicator (ffbb throughout:
    every schedule runs the same kernels in the same accumulation order; the second run
    replays the first one's GEMM plan, so both use the same kernel per shape)."""
    env = {"DLT_FORCE_CPU": None, "DLT_BACKEND": "nccl", "DLT_GEMM_PLAN": str(tmp_path / "plan.json")}
    a, (win_a, auto_a) = run_multiprocess(_forced, world=1, args=("ddp_auto",), env=env, timeout=300)[0]
    b, (win_b, auto_b) = run_multiprocess(_forced, world=1, args=("ddp_auto",),
                                          env={**env, "DLT_FORCE_COLLECTIVES": "1"}, timeout=300)[0]
    assert auto_a is None and win_a == "ffbb"
    assert auto_b is not None and auto_b["decided"] in ("fb", "ffbb") and win_b == auto_b["decided"], auto_b
    assert set(auto_b["ms"]) == {"fb", "ffbb"}
    for k in a:
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())


@pytest.mark.parametrize("mode", ["ddp", "ddp_lean", "fsdp"])
def test_rccl_forced_collectives_one_rank(mode):
    """RCCL kernels launched from the weight-gradient / pipeline streams, with the
    bucket and unit schedules of a multi-GPU run: a 1-rank sum is the identity, so the
    parameters must equal the run without collectives bit for bit.  ddp_lean: per-role
    deferral (bucket hooks issued after both the side-stream and the per-chain wgrads)."""
    # timing-free GEMM choices, so the two processes run the same kernels
    env = {"DLT_FORCE_CPU": None, "DLT_BACKEND": "nccl", "DLT_GEMM_TUNE": "0", "DLT_WGRAD_SPLITK": "0",
           "DLT_GEMM_TN": "0", "DLT_GEMM_FUSED": "0", "DLT_WGRAD_HAND": "0"}
    a, _ = run_multiprocess(_forced, world=1, args=(mode,), env=env, timeout=240)[0]
    b, launched = run_multiprocess(_forced, world=1, args=(mode,), env={**env, "DLT_FORCE_COLLECTIVES": "1"},
                                   timeout=240)[0]
    if mode.startswith("ddp"):
        assert launched > 2
    for k in a:
        assert torch.equal(a[k], b[k]), (k, (a[k] - b[k]).abs().max().item())


def test_rccl_forced_bf16_wire_matches_fp32_wire():
    """DDP with reduce_dtype bf16 (the gradient buckets cast to bf16 for the RCCL
    all-reduce, summed, cast back into the fp32 accumulators) on one forced RCCL rank: every
    bucket goes through the bf16 transport (so the parameters differ from the fp32 wire's
    in the last bits) and the trained parameters stay within bf16 gradient rounding of the
    fp32-wire run."""
    env = {"DLT_FORCE_CPU": None, "DLT_BACKEND": "nccl", "DLT_GEMM_TUNE": "0", "DLT_WGRAD_SPLITK": "0",
           "DLT_GEMM_TN": "0", "DLT_GEMM_FUSED": "0", "DLT_WGRAD_HAND": "0", "DLT_FORCE_COLLECTIVES": "1"}
    a, la = run_multiprocess(_forced, world=1, args=("ddp",), env=env, timeout=240)[0]
    b, lb = run_multiprocess(_forced, world=1, args=("ddp_bf16",), env=env, timeout=240)[0]
    assert la == lb and la > 2
    fa, fb = a["flat"], b["flat"]
    assert not torch.equal(fa, fb)  # the bf16 transport ran
    # AdamW normalises the update, so a bf16-rounded gradient moves each weight by at most
    # ~lr per step either way; the parameters agree to well under one step's update
    rel = ((fa - fb).norm() / fa.norm()).item()
    assert rel < 1e-3, rel
    assert (fa - fb).abs().max().item() < 3 * 1e-3 * STEPS
