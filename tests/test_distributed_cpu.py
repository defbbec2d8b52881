"""Multi-process (gloo, CPU) correctness of the DDP and FSDP runtimes.

These are the reference's missing tests: collectives are exercised for
real with 2 ranks; results are compared against single-process runs on the same data.
"""
import os

import pytest
import torch

from tests.dist_utils import run_multiprocess

TINY = dict(vocab_size=384, hidden_size=64, num_layers=2, num_heads=4, max_seq_len=32, dropout=0.0,
            attention_dropout=0.0)


def _data(step, rank, n=8, seq=32, vocab=384):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randint(0, vocab, (n, seq), generator=g)


def _ddp_worker(rank, world, steps, bucket_mb, fusion=1, GA=2):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig(**TINY)
    tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=GA, warmup_steps=1, max_steps=100,
                        learning_rate=1e-2, bucket_cap_mb=bucket_mb, micro_step_fusion=fusion)
    tr = DistributedTrainer(cfg, tc)
    losses = []
    for s in range(steps):
        losses.append(tr.train_step({"input_ids": _data(s, rank, n=2 * GA)})["loss"])
    return tr.flat_params().clone(), losses, len(tr.ddp.buckets)


def _single_worker_equiv(steps, world, GA=2):
    """One process, GA = world*GA, consuming every rank's micro-batches in order."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    cfg = GPTConfig(**TINY)
    tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=GA * world, warmup_steps=1, max_steps=100,
                        learning_rate=1e-2, micro_step_fusion=1)
    tr = DistributedTrainer(cfg, tc)
    for s in range(steps):
        batch = torch.cat([_data(s, r, n=2 * GA) for r in range(world)], dim=0)
        tr.train_step({"input_ids": batch})
    return tr.flat_params().clone()


@pytest.mark.parametrize("bucket_mb", [0.05, 64.0])
def test_ddp_matches_single_process(bucket_mb):
    outs = run_multiprocess(_ddp_worker, world=2, args=(3, bucket_mb))
    (p0, l0, nb0), (p1, l1, nb1) = outs
    assert torch.equal(p0, p1), "ranks diverged"
    ref = _single_worker_equiv(3, 2)
    assert torch.allclose(p0, ref, atol=2e-5, rtol=1e-4), (p0 - ref).abs().max()
    if bucket_mb < 1:
        assert nb0 > 2  # several buckets exercised


@pytest.mark.parametrize("fusion,GA", [(2, 4), (2, 2)])
def test_ddp_micro_step_fusion_matches_single_process(fusion, GA):
    """DDP with fused micro-step chains (2 pipelined chains of 2 micro-steps, or one
    chain): replicas stay bit-identical and equal the unfused single-process GA run."""
    outs = run_multiprocess(_ddp_worker, world=2, args=(3, 0.05, fusion, GA))
    (p0, _, _), (p1, _, _) = outs
    assert torch.equal(p0, p1), "ranks diverged"
    ref = _single_worker_equiv(3, 2, GA=GA)
    assert torch.allclose(p0, ref, atol=2e-5, rtol=1e-4), (p0 - ref).abs().max()


def _fsdp_worker(rank, world, strategy, steps, ac, offload, fusion=1):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                            learning_rate=1e-2, micro_step_fusion=fusion)
    fc = FSDPConfig(sharding_strategy=strategy, activation_checkpointing=ac, cpu_offload=offload,
                    reduce_dtype="fp32")
    tr = FSDPTrainer(cfg, tc, fc)
    for s in range(steps):
        tr.train_step({"input_ids": _data(s, rank, n=4)})
    sd = tr._full_state()
    return {k: v for k, v in sd.items() if "rotary" not in k}


def _fsdp_single(steps, world, ac=False):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2 * world, warmup_steps=1, max_steps=100,
                            learning_rate=1e-2, micro_step_fusion=1)
    fc = FSDPConfig(sharding_strategy="FULL_SHARD", activation_checkpointing=ac, reduce_dtype="fp32")
    tr = FSDPTrainer(cfg, tc, fc)
    for s in range(steps):
        batch = torch.cat([_data(s, r, n=4) for r in range(world)], dim=0)
        tr.train_step({"input_ids": batch})
    return {k: v for k, v in tr._full_state().items() if "rotary" not in k}


@pytest.mark.parametrize("strategy,ac,offload", [("FULL_SHARD", True, False), ("SHARD_GRAD_OP", False, False),
                                                 ("NO_SHARD", False, False), ("FULL_SHARD", False, True),
                                                 ("HYBRID_SHARD", True, False)])
def test_fsdp_matches_single_process(strategy, ac, offload):
    outs = run_multiprocess(_fsdp_worker, world=2, args=(strategy, 3, ac, offload))
    ref = _fsdp_single(3, 2)
    for k in ref:
        assert torch.equal(outs[0][k], outs[1][k]), f"{k}: ranks diverged"
        assert torch.allclose(outs[0][k], ref[k], atol=3e-5, rtol=1e-4), (k, (outs[0][k] - ref[k]).abs().max())


def test_ddp_three_ranks_matches_single_process():
    """An odd world size (buckets and the 1/world factor are not powers of two)."""
    outs = run_multiprocess(_ddp_worker, world=3, args=(2, 0.05, 2, 4))
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]), "ranks diverged"
    ref = _single_worker_equiv(2, 3, GA=4)
    assert torch.allclose(outs[0][0], ref, atol=2e-5, rtol=1e-4), (outs[0][0] - ref).abs().max()


@pytest.mark.parametrize("strategy,world,local", [("FULL_SHARD", 3, 3), ("HYBRID_SHARD", 4, 2)])
def test_fsdp_wider_worlds_match_single_process(strategy, world, local):
    """FULL_SHARD over 3 ranks (no unit divides evenly: shard padding on every unit) and
    HYBRID_SHARD as a 2 x 2 mesh (shard inside each "node" of 2, all-reduce across)."""
    outs = run_multiprocess(_fsdp_worker, world=world, args=(strategy, 2, True, False),
                            env={"LOCAL_WORLD_SIZE": str(local)})
    ref = _fsdp_single(2, world)
    for k in ref:
        for r in range(1, world):
            assert torch.equal(outs[0][k], outs[r][k]), f"{k}: rank {r} diverged"
        assert torch.allclose(outs[0][k], ref[k], atol=3e-5, rtol=1e-4), (k, (outs[0][k] - ref[k]).abs().max())


def test_fsdp_micro_step_fusion_matches_single_process():
    """FULL_SHARD with both micro-steps fused into one chain (one reduce-scatter per
    chain instead of per micro-step): same parameters as the unfused single process."""
    outs = run_multiprocess(_fsdp_worker, world=2, args=("FULL_SHARD", 3, True, False, 2))
    ref = _fsdp_single(3, 2)
    for k in ref:
        assert torch.equal(outs[0][k], outs[1][k]), f"{k}: ranks diverged"
        assert torch.allclose(outs[0][k], ref[k], atol=3e-5, rtol=1e-4), (k, (outs[0][k] - ref[k]).abs().max())


def _fsdp_ckpt_worker(rank, world, path):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, learning_rate=1e-2)
    fc = FSDPConfig(reduce_dtype="fp32")
    tr = FSDPTrainer(cfg, tc, fc)
    for s in range(2):
        tr.train_step({"input_ids": _data(s, rank, n=4)})
    tr.save_checkpoint(path)
    tr2 = FSDPTrainer(cfg, tc, fc)
    tr2.load_checkpoint(path)
    same = torch.equal(tr.runtime.master_flat, tr2.runtime.master_flat) and \
        torch.equal(tr.optimizer.exp_avg, tr2.optimizer.exp_avg) and tr2.global_step == 2
    # one more identical step on both -> identical params
    b = _data(5, rank, n=4)
    tr.train_step({"input_ids": b})
    tr2.train_step({"input_ids": b})
    return same, torch.equal(tr.runtime.master_flat, tr2.runtime.master_flat)


def test_fsdp_checkpoint_roundtrip(tmp_path):
    path = str(tmp_path / "fsdp.pt")
    outs = run_multiprocess(_fsdp_ckpt_worker, world=2, args=(path,))
    for same, same_after in outs:
        assert same and same_after
    from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint
    c = load_checkpoint(path)
    assert set(c) == {"model", "optimizer", "global_step", "tokens_seen", "model_config", "training_config",
                      "fsdp_config"}
    assert isinstance(next(iter(c["optimizer"]["state"])), str)  # FQN keys (FSDP optim_state_dict format)
    assert len(c["optimizer"]["param_groups"]) == 1
    assert c["model"]["embed_tokens.weight"].shape == (384, 64)


def test_fsdp_single_matches_ddp_engine():
    """Guards against common-mode bugs in the FSDP-vs-FSDP comparisons above: one-rank
    FSDP must equal the DDP trainer with the FSDP trainer's optimizer grouping."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    from distributed_llm_trainer_amd.training.optim import flat_store_optimizer
    os.environ.pop("RANK", None)
    cfg = GPTConfig(**TINY)
    tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=1, max_steps=100,
                        learning_rate=1e-2, lr_schedule_fix=True)
    tr = DistributedTrainer(cfg, tc)
    tr.optimizer = flat_store_optimizer(tr.store, tc.learning_rate, (0.9, 0.95), 1e-8, 0.1, split_no_decay=False)
    for s in range(3):
        tr.train_step({"input_ids": torch.cat([_data(s, r, n=4) for r in range(2)], dim=0)})
    ddp_sd = {k: v for k, v in tr.model.state_dict().items() if "rotary" not in k}
    fsdp_sd = _fsdp_single(3, 2)
    for k in fsdp_sd:
        assert torch.allclose(fsdp_sd[k], ddp_sd[k], atol=3e-5, rtol=1e-4), k


def _replica_worker(rank, world):
    import torch
    from distributed_llm_trainer_amd.training.common import setup_distributed
    from distributed_llm_trainer_amd.utils import debug
    setup_distributed()
    flat = torch.arange(1000, dtype=torch.float32) * 0.01
    debug.check_replicas(flat)  # identical replicas pass
    if rank == 1:
        flat[123] += 1e-6  # one ulp-scale divergence on one rank
    try:
        debug.check_replicas(flat)
        return "no error"
    except RuntimeError as e:
        return str(e)


def test_replica_divergence_detected():
    out = run_multiprocess(_replica_worker, world=2)
    assert all("ranks [1]" in o for o in out), out


def _fsdp_reshard_load_worker(rank, world, path):
    """Load a checkpoint written by a 2-rank FSDP job into a job of a different size."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, learning_rate=1e-2)
    tr = FSDPTrainer(cfg, tc, FSDPConfig(reduce_dtype="fp32"))
    tr.load_checkpoint(path)
    sd = tr._full_state()
    return {k: v.clone() for k, v in sd.items()}, tr.global_step


def test_fsdp_checkpoint_loads_at_other_world_size(tmp_path):
    """FULL_STATE_DICT checkpoints are world-size independent: written by 2 ranks, read
    back by 1 and by 3 ranks with identical full parameters."""
    path = str(tmp_path / "fsdp2.pt")
    run_multiprocess(_fsdp_ckpt_worker, world=2, args=(path,))
    from distributed_llm_trainer_amd.utils.checkpoint import load_checkpoint
    ref = load_checkpoint(path)["model"]
    for world in (1, 3):
        outs = run_multiprocess(_fsdp_reshard_load_worker, world=world, args=(path,))
        for sd, step in outs:
            assert step == 2
            for k, v in ref.items():
                assert torch.equal(sd[k].float(), v.float()), (world, k)


def _fsdp_sharded_ckpt_worker(rank, world, path, full_path, strategy):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, learning_rate=1e-2)
    fc = FSDPConfig(sharding_strategy=strategy, reduce_dtype="fp32")
    tr = FSDPTrainer(cfg, tc, fc)
    for s in range(2):
        tr.train_step({"input_ids": _data(s, rank, n=4)})
    tr.save_sharded_checkpoint(path)
    tr.save_checkpoint(full_path)   # the same state through the FULL_STATE_DICT path
    tr2 = FSDPTrainer(cfg, tc, fc)
    tr2.load_checkpoint(path)       # a directory -> sharded load
    same = torch.equal(tr.runtime.master_flat, tr2.runtime.master_flat) and \
        torch.equal(tr.optimizer.exp_avg_sq, tr2.optimizer.exp_avg_sq) and tr2.global_step == 2 and \
        tr2.optimizer.step_count == tr.optimizer.step_count
    b = _data(5, rank, n=4)
    tr.train_step({"input_ids": b})
    tr2.train_step({"input_ids": b})
    return same, torch.equal(tr.runtime.master_flat, tr2.runtime.master_flat)


@pytest.mark.parametrize("strategy", ["FULL_SHARD", "HYBRID_SHARD"])
def test_fsdp_sharded_checkpoint_roundtrip_and_consolidate(tmp_path, strategy):
    """SHARDED_STATE_DICT: per-rank save/load resumes bit-exactly, and the offline
    consolidation reproduces the FULL_STATE_DICT file of the same state."""
    path, full_path = str(tmp_path / "sharded"), str(tmp_path / "full.pt")
    outs = run_multiprocess(_fsdp_sharded_ckpt_worker, world=2, args=(path, full_path, strategy))
    for same, same_after in outs:
        assert same and same_after
    assert sorted(os.listdir(path)) == ["extra.pt", "meta.json", "shard_00000.pt", "shard_00001.pt"]
    from distributed_llm_trainer_amd.utils.checkpoint import consolidate_sharded, load_checkpoint
    cons = consolidate_sharded(path, str(tmp_path / "cons.pt"))
    full = load_checkpoint(full_path)
    again = load_checkpoint(str(tmp_path / "cons.pt"))
    assert set(again) == set(full)
    assert list(again["model"]) == list(full["model"])
    for k, v in full["model"].items():
        assert torch.equal(cons["model"][k], v), k
    assert list(full["optimizer"]["state"]) == list(cons["optimizer"]["state"])
    for n, st in full["optimizer"]["state"].items():
        for f in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(cons["optimizer"]["state"][n][f], st[f]), (n, f)
    assert cons["optimizer"]["param_groups"] == full["optimizer"]["param_groups"]
    assert (cons["global_step"], cons["tokens_seen"]) == (full["global_step"], full["tokens_seen"])
    assert cons["model_config"] == full["model_config"] and cons["fsdp_config"] == full["fsdp_config"]


def test_fsdp_sharded_checkpoint_rejects_other_world_size(tmp_path):
    path = str(tmp_path / "sharded")
    run_multiprocess(_fsdp_sharded_ckpt_worker, world=2, args=(path, str(tmp_path / "f.pt"), "FULL_SHARD"))
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    tr = FSDPTrainer(GPTConfig(**TINY), FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2),
                     FSDPConfig(reduce_dtype="fp32"))
    with pytest.raises(ValueError, match="consolidate_sharded"):
        tr.load_checkpoint(path)


def _forced_worker(rank, world, mode, strategy="FULL_SHARD"):
    """One rank; with DLT_FORCE_COLLECTIVES=1 every bucket / gather / reduce-scatter is
    still issued through the process group (the multi-GPU code path)."""
    from distributed_llm_trainer_amd.models.config import GPTConfig
    cfg = GPTConfig(**TINY)
    if mode == "ddp":
        from distributed_llm_trainer_amd.training.configs import TrainingConfig
        from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=1, max_steps=100,
                            learning_rate=1e-2, bucket_cap_mb=0.05, micro_step_fusion=2)
        tr = DistributedTrainer(cfg, tc)
    else:
        from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
        from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
        tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=4, warmup_steps=1, max_steps=100,
                                learning_rate=1e-2, micro_step_fusion=2)
        tr = FSDPTrainer(cfg, tc, FSDPConfig(sharding_strategy=strategy, reduce_dtype="fp32"))
    for s in range(2):
        tr.train_step({"input_ids": _data(s, 0, n=8)})
    launched = tr.ddp.launched if mode == "ddp" else 0
    sd = tr._full_state() if mode != "ddp" else {"flat": tr.flat_params().detach().cpu().clone()}
    return {k: v.detach().float().cpu() for k, v in sd.items() if "rotary" not in k}, launched


@pytest.mark.parametrize("mode,strategy", [("ddp", None), ("fsdp", "FULL_SHARD"), ("fsdp", "NO_SHARD")])
def test_forced_collectives_on_one_rank_are_identity(mode, strategy):
    a, _ = run_multiprocess(_forced_worker, world=1, args=(mode, strategy))[0]
    b, launched = run_multiprocess(_forced_worker, world=1, args=(mode, strategy),
                                   env={"DLT_FORCE_COLLECTIVES": "1"})[0]
    if mode == "ddp":
        assert launched > 2
    for k in a:
        assert torch.equal(a[k], b[k]), k


def _loss_worker(rank, world):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import TrainingConfig
    from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
    tr = DistributedTrainer(GPTConfig(**TINY), TrainingConfig(batch_size=2, gradient_accumulation_steps=2,
                                                              warmup_steps=1, max_steps=10))
    m = tr.train_step({"input_ids": _data(0, rank, n=4)})
    return m["loss"], m["loss_global"]


def test_logged_global_loss_is_the_rank_mean():
    """the log line keeps rank 0's local loss; the metrics also carry the
    mean over ranks (one scalar all-reduce on logged steps)."""
    (l0, g0), (l1, g1) = run_multiprocess(_loss_worker, world=2)
    assert g0 == g1 and abs(g0 - (l0 + l1) / 2) < 1e-6 and l0 != l1


def _rank0_only_worker(rank, world):
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
    from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
    cfg = GPTConfig(**TINY)
    tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, learning_rate=1e-2)
    tr = FSDPTrainer(cfg, tc, FSDPConfig(reduce_dtype="fp32"))
    tr.train_step({"input_ids": _data(0, rank, n=4)})
    full = tr._full_state()  # every rank
    r0 = tr._full_state(rank0_only=True)
    o0 = tr._full_optim_state(rank0_only=True)
    same = r0 is not None and all(torch.equal(r0[k], full[k]) for k in full)
    return rank, r0 is None, o0 is None, same


def test_fsdp_full_state_dict_rank0_only():
    """FULL_STATE_DICT at save time is gathered to rank 0 only (the reference's
    FullStateDictConfig(offload_to_cpu=True, rank0_only=True)): the other ranks take part
    in the collectives but never hold the host copy."""
    outs = sorted(run_multiprocess(_rank0_only_worker, world=2))
    (r0, none0, onone0, same0), (r1, none1, onone1, _) = outs
    assert not none0 and not onone0 and same0
    assert none1 and onone1


def test_fsdp_limit_all_gathers_bounds_prefetch():
    """limit_all_gathers (reference fsdp_trainer.py:296): at most two prefetched
    all-gathers (one per pipelined chain) are in flight; without the limit the same
    prefetch requests are all issued."""
    from distributed_llm_trainer_amd.models import GPT
    from distributed_llm_trainer_amd.models.config import GPTConfig
    from distributed_llm_trainer_amd.parallel.fsdp import FSDPRuntime

    class _Work:
        def wait(self):
            pass

    for limit, want in ((True, 2), (False, 4)):
        rt = FSDPRuntime(GPT(GPTConfig(**dict(TINY, num_layers=4))), "cpu", limit_all_gathers=limit)
        rt.force = True  # behave like a sharded job: prefetches are real (async) gathers
        issued = []

        def fake_gather(u, async_op, issued=issued):
            u.full = torch.empty(u.padded)
            u.ag_work = _Work() if async_op else None
            issued.append(u.uid)
        rt._gather = fake_gather
        for uid in range(4):
            rt._prefetch(rt.units[uid])
        assert len(issued) == want, (limit, issued)


def _count_worker(rank, world, mode, strategy="FULL_SHARD", sparse_rows=None):
    """One warm step, then the collectives of one optimizer step (GA = 2 micro-steps),
    counted by wrapping torch.distributed: [(name, numel, element size)]."""
    import torch.distributed as dist
    if sparse_rows is not None:
        os.environ["DLT_DDP_SPARSE_ROWS"] = str(sparse_rows)
    from distributed_llm_trainer_amd.models.config import GPTConfig
    cfg = GPTConfig(**TINY)
    if mode == "ddp":
        from distributed_llm_trainer_amd.training.configs import TrainingConfig
        from distributed_llm_trainer_amd.training.ddp_trainer import DistributedTrainer
        tc = TrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                            learning_rate=1e-2, bucket_cap_mb=0.05, micro_step_fusion=1)
        tr = DistributedTrainer(cfg, tc)
    else:
        from distributed_llm_trainer_amd.training.configs import FSDPConfig, FSDPTrainingConfig
        from distributed_llm_trainer_amd.training.fsdp_trainer import FSDPTrainer
        tc = FSDPTrainingConfig(batch_size=2, gradient_accumulation_steps=2, warmup_steps=1, max_steps=100,
                                learning_rate=1e-2, micro_step_fusion=1)
        tr = FSDPTrainer(cfg, tc, FSDPConfig(sharding_strategy=strategy, reduce_dtype="fp32"))
    tr.train_step({"input_ids": _data(0, rank, n=4)})
    log = []
    names = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast", "all_gather",
             "reduce_scatter", "barrier")
    orig = {n: getattr(dist, n) for n in names}

    def wrap(n):
        def f(*a, **kw):
            # the full-size operand: all_gather_into_tensor's output, reduce_scatter_tensor's input
            t = a[1] if n == "reduce_scatter_tensor" else (a[0] if a and torch.is_tensor(a[0]) else kw.get("tensor"))
            log.append((n, t.numel() if torch.is_tensor(t) else 0, t.element_size() if torch.is_tensor(t) else 0))
            return orig[n](*a, **kw)
        return f
    for n in names:
        setattr(dist, n, wrap(n))
    try:
        tr.train_step({"input_ids": _data(1, rank, n=4)})
    finally:
        for n in names:
            setattr(dist, n, orig[n])
    if mode == "ddp":
        lay = tr.store.layout
        info = dict(buckets=[b - a for a, b in tr.ddp.buckets], total=tr.store.flat.numel(), embed=lay.embed_offset,
                    decay_end=lay.decay_end, H=cfg.hidden_size, Vp=cfg.vocab_size_padded, head=tr.ddp.last_head)
        return log, info, None
    units = {str(uid): (u.padded, u.shard) for uid, u in tr.runtime.units.items()}
    return log, units, cfg.num_layers


@pytest.mark.parametrize("sparse", [False, True])
def test_ddp_collective_pattern_per_step(sparse):
    """SURVEY §2.4 X3/X4 on 2 gloo ranks: one optimizer step (2 micro-steps) issues its
    gradient all-reduces only in the last micro-step (no_sync): one fp32 all-reduce per
    layer bucket, the lm_head part of the tied gradient ([Vp, H], handed over by the engine
    at the start of the last backward), the embedding part -- dense by default, row-sparse
    with DLT_DDP_SPARSE_ROWS (one byte per row MAX-reduced, then only the union of non-zero
    rows, or dense when the union exceeds that share of the rows) -- the norm weights, plus
    the logged global loss (one scalar).  No per-step buffer broadcast (X3 is dropped by
    design)."""
    for log, d, _ in run_multiprocess(_count_worker, world=2,
                                      args=("ddp", "FULL_SHARD", 0.5 if sparse else None)):
        ar = [x for x in log if x[0] == "all_reduce"]
        assert len(log) == len(ar), log  # no broadcast / gather / reduce-scatter per step
        H, Vp = d["H"], d["Vp"]
        layer = [b for b in d["buckets"] if b <= d["embed"]]
        sizes = [x[1] for x in ar]
        # layer buckets first, in backward order, fp32, covering the layer region once
        assert sum(x[1] for x in ar if x[1] in layer and x[2] == 4) >= d["embed"]
        assert Vp * H in sizes  # the lm_head part (or a dense embedding part too)
        # the union bitmap (row-sparse mode only)
        assert [x for x in ar if x[2] == 1] == ([("all_reduce", Vp, 1)] if sparse else [])
        head = d["head"]
        if not sparse:
            assert head == "dense"
        assert head == "dense" or (head[0] == "rows" and 0 < head[1] <= Vp // 2 and head[2] == Vp), head
        if head != "dense":
            assert head[1] * H in sizes
        assert d["total"] - d["decay_end"] in sizes  # the norm weights
        assert sizes.count(1) == 1  # the global-loss scalar


@pytest.mark.parametrize("strategy", ["FULL_SHARD", "SHARD_GRAD_OP"])
def test_fsdp_collective_pattern_per_step(strategy):
    """SURVEY §2.4 X5-X8 on 2 gloo ranks, per optimizer step of 2 micro-steps: every
    micro-step all-gathers each block for its forward (X5; the root unit once per step),
    FULL_SHARD gathers each block again for its backward (X6; SHARD_GRAD_OP keeps the
    forward's gather), reduce-scatters
    every unit's gradient once (X7), and the step ends with one scalar all-reduce for the
    gradient clip (X8) plus the logged global loss."""
    for log, units, L in run_multiprocess(_count_worker, world=2, args=("fsdp", strategy)):
        ag = [x for x in log if x[0] == "all_gather_into_tensor"]
        rs = [x for x in log if x[0] == "reduce_scatter_tensor"]
        ar = [x for x in log if x[0] == "all_reduce"]
        assert len(ag) + len(rs) + len(ar) == len(log), log
        full = {uid: p for uid, (p, _) in units.items()}
        head, block = full["head"], full["0"]
        # the root unit (embedding / tied lm_head / final norm) is gathered once and kept for
        # the step (the reference's root FSDP unit is never resharded after forward); every
        # block is gathered for each micro-step's forward and, under FULL_SHARD, again for
        # its backward
        per_block = 4 if strategy == "FULL_SHARD" else 2
        assert [x[1] for x in ag].count(head) == 1
        assert [x[1] for x in ag].count(block) == per_block * L and len(ag) == 1 + per_block * L
        assert sorted(x[1] for x in rs) == sorted(2 * list(full.values()))  # every unit, every micro-step
        assert [x[1] for x in ar] == [1, 1]  # clip sum of squares + the logged loss


def test_comm_env_is_set_before_the_process_group(monkeypatch):
    """parallel/comm_env.py: the RCCL xGMI defaults are exported before
    init_process_group creates a communicator, and a user's own value wins."""
    import torch.distributed as dist
    from distributed_llm_trainer_amd.parallel import comm_env
    from distributed_llm_trainer_amd.training import common
    if dist.is_initialized():
        pytest.skip("process group already initialised in this process")
    for k in list(comm_env.COMMON) + list(comm_env.SINGLE_NODE):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_DEBUG", "INFO")  # user-set: kept
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    seen = {}

    def fake_init(**kw):
        seen.update({k: os.environ.get(k) for k in list(comm_env.COMMON) + list(comm_env.SINGLE_NODE)})
        raise RuntimeError("stop")  # nothing to rendezvous with
    monkeypatch.setattr(dist, "init_process_group", fake_init)
    with pytest.raises(RuntimeError, match="stop"):
        common.setup_distributed(require=True)
    assert seen["NCCL_DEBUG"] == "INFO"
    assert seen["NCCL_IB_DISABLE"] == "1" and seen["NCCL_MIN_NCHANNELS"] == "32"
    assert seen["TORCH_NCCL_HIGH_PRIORITY"] == "1" and seen["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # several nodes: no NCCL_IB_DISABLE
    monkeypatch.delenv("NCCL_IB_DISABLE")
    assert "NCCL_IB_DISABLE" not in comm_env.apply(world_size=16, local_world_size=8)
    monkeypatch.setenv("DLT_COMM_ENV", "0")
    assert comm_env.apply() == {}
