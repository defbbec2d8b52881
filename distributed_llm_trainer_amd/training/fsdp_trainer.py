"""Fully-sharded trainer (CLI- and API-compatible with the reference's
``src/training/fsdp_trainer.py``; call stack SURVEY §3.2).

Differences from the reference by design:
* The sharding runtime is ``parallel/fsdp.py`` (flat units per TransformerBlock +
  root, bf16 all-gather with forward/backward prefetch, reduce-scatter into fp32
  shards) driving the fused HIP executor; torch FSDP is not used.
* Activation checkpointing (default ON, like the reference) recomputes each block
  from its saved fp32 input; dropout masks replay bit-exactly (counter RNG).
* ``HYBRID_SHARD`` is implemented (the reference documents but does not map it).
* Precision (``FSDPConfig.mixed_precision``): see ``_setup_model`` for the bf16 /
  fp16 / fp32 policies.
* Seeded init, so every rank shards the same initial model (Q13).
* Checkpoints: FULL_STATE_DICT format of the reference (fp32 params with the same
  keys + FQN-keyed, unflattened optimizer state, one param group); loading reads
  the file on rank 0 and broadcasts flat units (no pickled broadcast, X11).
  ``--state_dict_type sharded`` adds SHARDED_STATE_DICT (per-rank shard files, no
  gather; the reference only discusses it at ``fsdp_trainer.py:416-418``).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist

from ..models.config import GPTConfig
from ..models.gpt import GPT, count_parameters
from ..parallel.fsdp import FSDPRuntime
from ..utils import checkpoint as ckpt
from ..utils import debug as dbg
from ..utils.profiling import Profiler
from .common import cosine_lr, gemm_plan_hook, global_mean_loss, memory_stats, micro_step_fusion, seed_all, select_device, setup_distributed, unwrap_batch
from .configs import FSDPConfig, FSDPTrainingConfig
from .optim import FlatAdamW

TrainingConfig = FSDPTrainingConfig  # name parity with the reference module

_DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


class FSDPTrainer:
    def __init__(self, model_config: GPTConfig, training_config: FSDPTrainingConfig, fsdp_config: FSDPConfig):
        self.model_config = model_config
        self.training_config = training_config
        self.fsdp_config = fsdp_config
        self.distributed, self.rank, self.world_size, self.local_rank = setup_distributed(require=False)
        self.is_main_process = self.rank == 0
        if self.is_main_process:
            print(f"Initialized FSDP: world_size={self.world_size}")
        self.device = select_device(self.local_rank)
        mp = fsdp_config.mixed_precision
        cuda = self.device.type == "cuda"
        # Precision policies (reference fsdp_trainer.py:223-234: bf16 -> MixedPrecision(bf16,
        # bf16, bf16), fp16 -> all fp16, otherwise none).  Master shards are always fp32;
        # the gathered compute copy, the activations and the reduce-scatter wire take the
        # policy dtype.  bf16 and fp16 run the HIP kernels (fp16: IEEE-half instances,
        # hand weight / data gradient GEMMs, hipBLASLt fp16 forwards); fp32 (reference / debug mode) runs the same schedule with
        # PyTorch ops on the GPU + hipBLASLt GEMMs (GPT.enable_engine).  fp16 adds a
        # dynamic loss scale the reference lacks (Q11): the global grad sumsq is
        # all-reduced anyway for clipping, so an inf/nan on ANY rank's shard skips the step
        # on every rank and halves the scale (x2 after 2000 good steps).
        self.compute_dtype = _DT.get(mp, torch.bfloat16) if cuda else torch.float32
        self.loss_scale = 2.0 ** 16 if self.compute_dtype == torch.float16 else None
        self._good_steps = 0
        if self.is_main_process:
            print(f"Device: {self.device} | compute dtype: {self.compute_dtype}")
        self._setup_model()
        self._setup_optimizer()
        self.global_step = 0
        self.tokens_seen = 0
        self._last_norm = None

    def _setup_model(self):
        fc, tc = self.fsdp_config, self.training_config
        seed_all(tc.seed)
        if self.is_main_process:
            print("Building model...")
        model = GPT(self.model_config)
        if self.is_main_process:
            print(f"Model parameters: {count_parameters(model):,}")
        red = _DT.get(fc.reduce_dtype, torch.bfloat16) if self.device.type == "cuda" else torch.float32
        if self.compute_dtype != torch.bfloat16 and fc.reduce_dtype == "bf16":
            red = self.compute_dtype  # the policy's reduce dtype (fp16 -> fp16, fp32 -> fp32)
        self.runtime = FSDPRuntime(model, self.device, sharding_strategy=fc.sharding_strategy,
                                   compute_dtype=self.compute_dtype, reduce_dtype=red, cpu_offload=fc.cpu_offload,
                                   backward_prefetch=fc.backward_prefetch, limit_all_gathers=fc.limit_all_gathers,
                                   sync_every_micro_step=fc.sync_every_micro_step)
        self.model = model.to(self.device)
        self.model.gradient_checkpointing = bool(fc.activation_checkpointing)
        self.model.enable_engine(provider=self.runtime, act_dtype=self.compute_dtype,
                                 seed=tc.seed + 1000003 * self.rank)
        if self.is_main_process:
            if fc.activation_checkpointing:
                print("Activation checkpointing enabled")
            print(f"FSDP sharding strategy: {fc.sharding_strategy}")

    def _setup_optimizer(self):
        tc = self.training_config
        rt = self.runtime
        shadow = None if (self.fsdp_config.cpu_offload or rt.shard_c_flat is rt.master_flat) else rt.shard_c_flat
        # reference: one group, weight decay on everything (fsdp_trainer.py:338-343)
        self.optimizer = FlatAdamW(rt.master_flat, rt.grad_flat, shadow,
                                   [(0, rt.master_flat.numel(), tc.weight_decay)], tc.learning_rate,
                                   (tc.beta1, tc.beta2), tc.adam_eps)
        if self.fsdp_config.cpu_offload:
            self.optimizer.is_cuda = False  # host AdamW on the offloaded shards

    def fusion_factor(self, GA: int, micro_bs: int, seq_len: int) -> int:
        gpu = self.device.type == "cuda"
        return micro_step_fusion(getattr(self.training_config, "micro_step_fusion", 0), GA, micro_bs, seq_len, gpu)

    def chains_per_step(self) -> int:
        """Engine forwards per optimizer step (dropout streams are keyed by this count)."""
        tc = self.training_config
        GA = tc.gradient_accumulation_steps
        return GA // self.fusion_factor(GA, tc.batch_size, self.model_config.max_seq_len)

    def get_lr(self, step: int) -> float:
        tc = self.training_config
        return cosine_lr(step, tc.learning_rate, tc.warmup_steps, tc.max_steps, clamp=True)

    def train_step(self, batch, sync_loss: bool = True) -> dict:
        tc = self.training_config
        rt = self.runtime
        self.model.train()
        if tc.lr_schedule_fix:
            lr = self.get_lr(self.global_step)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
        input_ids = unwrap_batch(batch).to(self.device, non_blocking=True)
        GA = tc.gradient_accumulation_steps
        micro_bs = input_ids.shape[0] // GA
        # F micro-steps per executed chain (micro_step_fusion); losses stay normalised
        # per micro-step, so the gradient is the reference's GA average
        F = self.fusion_factor(GA, micro_bs, input_ids.shape[1])
        chains, chain_bs = GA // F, micro_bs * F
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        rt.zero_grad()
        defer = not self.fsdp_config.sync_every_micro_step
        eng = self.model.engine
        eng.set_loss_segments(F)
        # micro-step pipelining (GPTEngine.train_window) from the second step on (the
        # first runs the GEMM autotuning); units are shared by the two chains through
        # the runtime's reference-counted residency
        pipelined = (chains > 1 and getattr(tc, "pipeline_micro_steps", True) and getattr(self, "_engine_warm", False)
                     and (self.device.type != "cuda" or getattr(eng.gemm, "stream_safe", False))
                     and os.environ.get("DLT_PIPELINE", "1") != "0")
        ls = self.loss_scale or 1.0
        # fp16: the cross-entropy gradient is stored pre-scaled by the loss scale (no fp16
        # underflow); the engine divides it out where dloss (= ls / chains) is applied
        eng.ce_grad_scale = float(ls)
        if pipelined:
            from ..models.engine import shift_targets
            ids_l = [input_ids[m * chain_bs:(m + 1) * chain_bs] for m in range(chains)]
            rt.require_sync(False)
            losses = eng.train_window(ids_l, [shift_targets(x) for x in ids_l],
                                      torch.full((), ls / chains, dtype=torch.float32, device=self.device),
                                      recompute=bool(self.model.gradient_checkpointing),
                                      before_last=lambda: rt.require_sync(True), defer=defer,
                                      sync_hook=rt.require_sync)
            for loss in losses:
                total += (loss / chains).detach().float()
        for micro in range(chains if pipelined else 0, chains):
            ids = input_ids[micro * chain_bs:(micro + 1) * chain_bs]
            rt.require_sync(micro == chains - 1)
            eng.set_accumulation(micro, chains, defer=defer)
            _, loss = self.model(ids, labels=ids)
            loss = loss / chains
            (loss * ls).backward() if self.loss_scale else loss.backward()
            total += loss.detach().float()
        eng.set_loss_segments(1)
        self._engine_warm = True
        rt.finish()
        # global grad norm: local shard sumsq -> scalar all-reduce (reference X8)
        ss = self.optimizer.local_sumsq()
        if self.distributed and rt.strategy != "NO_SHARD":
            ss_dev = ss.to(self.device)
            dist.all_reduce(ss_dev)
            ss = ss_dev.to(ss.device)
        scale = self.optimizer.compute_scale(tc.grad_clip, grad_div=float(self.world_size) * ls, sumsq=ss)
        skip = False
        if self.loss_scale is not None:  # ss is global: every rank takes the same decision
            if not torch.isfinite(scale[0]).item():
                self.loss_scale /= 2.0
                self._good_steps = 0
                skip = True
            else:
                self._good_steps += 1
                if self._good_steps % 2000 == 0:
                    self.loss_scale *= 2.0
        if not skip:
            self.optimizer.step(scale)
        if self.fsdp_config.cpu_offload:
            rt.refresh_shadow()
        self._last_norm = scale[0]
        rt.zero_grad()
        if not tc.lr_schedule_fix:
            lr = self.get_lr(self.global_step)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
        else:
            lr = self.optimizer.param_groups[0]["lr"]
        self.global_step += 1
        self.tokens_seen += input_ids.numel() * self.world_size
        if self.global_step >= 2:
            gemm_plan_hook()
        out = {"loss": total.item() if sync_loss else total, "lr": lr, "tokens": self.tokens_seen}
        if sync_loss and self.distributed and self.world_size > 1:
            out["loss_global"] = global_mean_loss(total, self.world_size)
        return out

    # ------------------------------------------------------------ checkpoints
    def _full_state(self, rank0_only: bool = False):
        """FULL_STATE_DICT (collective).  ``rank0_only``: None on ranks > 0, which never
        hold a host copy (what save_checkpoint uses, like the reference's
        ``FullStateDictConfig(offload_to_cpu=True, rank0_only=True)``)."""
        rt = self.runtime
        sd = rt.state_dict_full(rank0_only=rank0_only)
        if sd is None:
            return None
        # RoPE buffers (reference checkpoints carry them) in module order
        out = {}
        for k, v in self.model.state_dict().items():
            if k in sd:
                out[k] = sd[k]
            elif k == "lm_head.weight":
                out[k] = sd["embed_tokens.weight"]
            else:
                out[k] = v.detach().cpu().clone()
        return out

    def _full_optim_state(self, rank0_only: bool = False):
        rt, opt = self.runtime, self.optimizer
        state, names = {}, []
        order = [n for n, _ in self.model.named_parameters()]
        pieces = {}
        for uid, u in rt.units.items():
            a, b = rt.unit_offsets[uid]
            m = rt.gather_shard_tensor(uid, opt.exp_avg[a:b], rank0_only=rank0_only)
            v = rt.gather_shard_tensor(uid, opt.exp_avg_sq[a:b], rank0_only=rank0_only)
            if m is None:
                continue
            for s in u.segs:
                pieces[s.name] = (m[s.offset:s.offset + s.numel].view(s.shape).clone(),
                                  v[s.offset:s.offset + s.numel].view(s.shape).clone())
        for n in order:
            if n not in pieces:
                continue
            state[n] = {"step": torch.tensor(float(opt.step_count)), "exp_avg": pieces[n][0],
                        "exp_avg_sq": pieces[n][1]}
            names.append(n)
        if not pieces:
            return None  # rank > 0 under rank0_only
        g = {k: v for k, v in opt.param_groups[0].items()}
        g["params"] = names
        return {"state": state, "param_groups": [g]}

    def save_checkpoint(self, path: str):
        model_sd = self._full_state(rank0_only=True)          # collective; None on ranks > 0
        optim_sd = self._full_optim_state(rank0_only=True)    # collective
        if self.is_main_process:
            ckpt.save_checkpoint(path, {
                "model": model_sd, "optimizer": optim_sd, "global_step": self.global_step,
                "tokens_seen": self.tokens_seen, "model_config": self.model_config,
                "training_config": self.training_config, "fsdp_config": self.fsdp_config})
        if self.distributed:
            dist.barrier()

    # ------------------------------------------------------- SHARDED_STATE_DICT
    @torch.no_grad()
    def save_sharded_checkpoint(self, path: str):
        """SHARDED_STATE_DICT (the reference only discusses it, ``fsdp_trainer.py:416-418``):
        every rank writes its own fp32 master / exp_avg / exp_avg_sq shards into the
        directory ``path`` -- no all-gather, no rank-0 host copy of the full model, so a
        save costs one local write per rank regardless of model size.  Rank 0 adds
        ``meta.json`` (counters, configs, unit layout) and ``extra.pt`` (RoPE buffers and
        the state-dict key order) so ``utils.checkpoint.consolidate_sharded`` can rebuild
        the reference FULL_STATE_DICT file offline."""
        rt, opt = self.runtime, self.optimizer
        os.makedirs(path, exist_ok=True)
        units = {}
        for uid, u in rt.units.items():
            a, b = rt.unit_offsets[uid]
            units[str(uid)] = {"param": u.master.detach().to("cpu", copy=True),
                               "exp_avg": opt.exp_avg[a:b].to("cpu", copy=True),
                               "exp_avg_sq": opt.exp_avg_sq[a:b].to("cpu", copy=True)}
        ckpt.save_checkpoint(os.path.join(path, f"shard_{self.rank:05d}.pt"), {
            "rank": self.rank, "shard_rank": rt.shard_rank, "shard_world": rt.shard_world, "units": units})
        if self.is_main_process:
            sd_keys = list(self.model.state_dict().keys())
            params = {n for n, _ in self.model.named_parameters()}
            extra = {k: v.detach().to("cpu", copy=True) for k, v in self.model.state_dict().items()
                     if k not in params and k != "lm_head.weight"}
            ckpt.save_checkpoint(os.path.join(path, "extra.pt"), {"buffers": extra})
            g = {k: v for k, v in opt.param_groups[0].items() if k != "params"}
            meta = {
                "format": ckpt.SHARDED_FORMAT, "world_size": self.world_size, "shard_world": rt.shard_world,
                "strategy": rt.strategy, "global_step": self.global_step, "tokens_seen": self.tokens_seen,
                "optimizer_step": opt.step_count, "param_group": g,
                "state_dict_keys": sd_keys, "param_order": [n for n, _ in self.model.named_parameters()],
                "model_config": ckpt.config_to_dict(self.model_config),
                "training_config": ckpt.config_to_dict(self.training_config),
                "fsdp_config": ckpt.config_to_dict(self.fsdp_config),
                "units": {str(uid): {"numel": u.numel, "padded": u.padded, "shard": u.shard,
                                     "segs": [[s.name, s.offset, s.numel, list(s.shape)] for s in u.segs]}
                          for uid, u in rt.units.items()},
            }
            ckpt.write_json_atomic(os.path.join(path, "meta.json"), meta)
        if self.distributed:
            dist.barrier()

    @torch.no_grad()
    def load_sharded_checkpoint(self, path: str):
        """Load a SHARDED_STATE_DICT directory written at the same shard layout; for a
        different world size, consolidate it to a full checkpoint first."""
        rt, opt = self.runtime, self.optimizer
        meta = ckpt.read_sharded_meta(path)
        if meta["world_size"] != self.world_size or meta["shard_world"] != rt.shard_world:
            raise ValueError(f"sharded checkpoint was written by {meta['world_size']} ranks "
                             f"(shard world {meta['shard_world']}); this job has {self.world_size} "
                             f"(shard world {rt.shard_world}). Run utils.checkpoint.consolidate_sharded first.")
        c = ckpt.load_checkpoint(os.path.join(path, f"shard_{self.rank:05d}.pt"))
        if c["shard_rank"] != rt.shard_rank:
            raise ValueError(f"shard file of rank {self.rank} holds shard {c['shard_rank']}, expected {rt.shard_rank}")
        for uid, u in rt.units.items():
            e = c["units"][str(uid)]
            if e["param"].numel() != u.shard:
                raise ValueError(f"unit {uid}: shard has {e['param'].numel()} elements, expected {u.shard}")
            a, b = rt.unit_offsets[uid]
            u.master.copy_(e["param"].to(u.master.device))
            opt.exp_avg[a:b].copy_(e["exp_avg"].to(opt.exp_avg.device))
            opt.exp_avg_sq[a:b].copy_(e["exp_avg_sq"].to(opt.exp_avg_sq.device))
        rt.refresh_shadow()
        self.global_step, self.tokens_seen = int(meta["global_step"]), int(meta["tokens_seen"])
        opt.step_count = int(meta["optimizer_step"])
        self.model.engine.micro_counter = self.global_step * self.chains_per_step()
        if self.is_main_process:
            print(f"Loaded sharded checkpoint from {path} (step {self.global_step})")

    @torch.no_grad()
    def load_checkpoint(self, path: str):
        if os.path.isdir(path):
            return self.load_sharded_checkpoint(path)
        rt, opt = self.runtime, self.optimizer
        c = ckpt.load_checkpoint(path, map_location="cpu") if (self.is_main_process or not self.distributed) else None
        meta = [None]
        if self.is_main_process or not self.distributed:
            c["model"] = ckpt.normalize_state_dict_keys(c["model"])
            osd = c["optimizer"]
            steps = [int(float(s["step"])) for s in osd["state"].values()] if osd.get("state") else [0]
            meta[0] = (int(c["global_step"]), int(c["tokens_seen"]), max(steps) if steps else 0)
        if self.distributed:
            dist.broadcast_object_list(meta, src=0)
        for uid, u in rt.units.items():
            full = torch.zeros(u.padded, dtype=torch.float32, device=self.device)
            fm = torch.zeros_like(full)
            fv = torch.zeros_like(full)
            if c is not None:
                st = c["optimizer"]["state"]
                for s in u.segs:
                    full[s.offset:s.offset + s.numel].copy_(c["model"][s.name].reshape(-1))
                    if s.name in st:
                        fm[s.offset:s.offset + s.numel].copy_(st[s.name]["exp_avg"].reshape(-1))
                        fv[s.offset:s.offset + s.numel].copy_(st[s.name]["exp_avg_sq"].reshape(-1))
            if self.distributed:
                for t in (full, fm, fv):
                    dist.broadcast(t, src=0)
            rt.load_full_flat(uid, full.cpu() if rt.cpu_offload else full)
            a, b = rt.unit_offsets[uid]
            la, lb = u.local_slice()
            opt.exp_avg[a:b].copy_(fm[la:lb].to(opt.exp_avg.device))
            opt.exp_avg_sq[a:b].copy_(fv[la:lb].to(opt.exp_avg_sq.device))
        self.global_step, self.tokens_seen, opt.step_count = meta[0]
        self.model.engine.micro_counter = self.global_step * self.chains_per_step()
        if self.is_main_process:
            print(f"Loaded Checkpoint from {path} (step {self.global_step})")

    def get_memory_stats(self) -> dict:
        return memory_stats(self.device)


def build_parser():
    p = argparse.ArgumentParser(description="MI355X FSDP trainer (reference-compatible CLI)")
    p.add_argument("--model_size", default="medium", choices=["small", "medium", "large", "xl"])
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--max_steps", type=int, default=1000)
    p.add_argument("--sharding", default="FULL_SHARD", choices=["FULL_SHARD", "SHARD_GRAD_OP", "NO_SHARD",
                                                                  "HYBRID_SHARD"])
    p.add_argument("--cpu_offload", action="store_true")
    p.add_argument("--no_activation_checkpointing", action="store_true")
    # additions
    p.add_argument("--config", type=str, default=None)
    p.add_argument("--resume_from", type=str, default=None)
    p.add_argument("--checkpoint_dir", type=str, default=None)
    p.add_argument("--save_interval", type=int, default=None)
    p.add_argument("--log_interval", type=int, default=None)
    p.add_argument("--seq_len", type=int, default=None)
    p.add_argument("--gradient_accumulation_steps", type=int, default=None)
    p.add_argument("--reduce_dtype", choices=["bf16", "fp32"], default=None)
    p.add_argument("--no_final_save", action="store_true")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--profile", type=str, default=None, help="write a torch.profiler trace to this dir")
    p.add_argument("--metrics_jsonl", type=str, default=None)
    p.add_argument("--state_dict_type", choices=["full", "sharded"], default="full",
                   help="full: reference FULL_STATE_DICT file (rank-0 gather); sharded: per-rank shard "
                        "directory, no gather (resume with --resume_from DIR)")
    return p


def main(argv=None):
    from ..data import create_dummy_dataloader
    from ..utils.config_loader import explicit_args, load_yaml_config
    parser = build_parser()
    args = parser.parse_args(argv)
    given = explicit_args(parser, argv)
    model_config = GPTConfig.from_preset(args.model_size)
    tc = FSDPTrainingConfig(batch_size=args.batch_size, max_steps=args.max_steps)
    fc = FSDPConfig(sharding_strategy=args.sharding, cpu_offload=args.cpu_offload,
                    activation_checkpointing=not args.no_activation_checkpointing)
    if args.config:
        model_config, tc, fc, _ = load_yaml_config(args.config, model_config, tc, fc,
                                                   keep_model_preset="model_size" in given)
        if "batch_size" in given:
            tc.batch_size = args.batch_size
        if "max_steps" in given:
            tc.max_steps = args.max_steps
        if "sharding" in given:
            fc.sharding_strategy = args.sharding
        if "cpu_offload" in given:
            fc.cpu_offload = True
        if "no_activation_checkpointing" in given:
            fc.activation_checkpointing = False
    for k in ("resume_from", "checkpoint_dir", "save_interval", "log_interval", "gradient_accumulation_steps",
              "seed"):
        v = getattr(args, k)
        if v is not None:
            setattr(tc, k, v)
    if args.reduce_dtype:
        fc.reduce_dtype = args.reduce_dtype
    if args.seq_len:
        model_config.max_seq_len = args.seq_len

    trainer = FSDPTrainer(model_config, tc, fc)
    if tc.resume_from:
        trainer.load_checkpoint(tc.resume_from)
    total_batch = tc.batch_size * tc.gradient_accumulation_steps
    dataloader = create_dummy_dataloader(batch_size=total_batch, seq_len=model_config.max_seq_len,
                                         vocab_size=model_config.vocab_size, distributed=trainer.distributed,
                                         rank=trainer.rank, world_size=trainer.world_size,
                                         num_batches=int(os.environ.get("DLT_DUMMY_BATCHES", "64")), seed=tc.seed,
                                         device=trainer.device)
    if hasattr(dataloader, "seek") and trainer.global_step:
        dataloader.seek(trainer.global_step)
    if trainer.is_main_process:
        print("\n" + "=" * 60)
        print("Starting FSDP training...")
        print("=" * 60 + "\n")
        mem = trainer.get_memory_stats()
        print(f"Initial memory: {mem['allocated_gb']:.2f} GB allocated")
    def save(stem):
        if args.state_dict_type == "sharded":
            trainer.save_sharded_checkpoint(stem)
        else:
            trainer.save_checkpoint(stem + ".pt")

    metrics_f = open(args.metrics_jsonl, "a") if (args.metrics_jsonl and trainer.is_main_process) else None
    prof = Profiler(args.profile, enabled=bool(args.profile) and trainer.is_main_process)
    data_iter = iter(dataloader)
    start_time = time.time()
    start_step = trainer.global_step
    tokens0 = trainer.tokens_seen  # tokens of a resumed run's earlier steps are not this run's throughput
    steady_t0, steady_tok0, steady_ckpt = None, 0, 0.0
    for step in range(start_step, tc.max_steps):
        dbg.maybe_inject_fault(step, trainer.rank)
        try:
            batch = next(data_iter)
        except StopIteration:
            data_iter = iter(dataloader)
            batch = next(data_iter)
        do_log = step % tc.log_interval == 0
        metrics = trainer.train_step({"input_ids": unwrap_batch(batch)}, sync_loss=do_log)
        prof.step()
        if step - start_step == 10:
            steady_t0, steady_tok0 = time.time(), trainer.tokens_seen
        if do_log and trainer.is_main_process:
            elapsed = time.time() - start_time
            tps = (metrics["tokens"] - tokens0) / max(elapsed, 1e-9)
            mem = trainer.get_memory_stats()
            print(f"Step {step:6d} | Loss: {metrics['loss']:.4f} | LR: {metrics['lr']:.2e} | "
                  f"Tokens/s: {tps:,.0f} | Mem: {mem['allocated_gb']:.1f}GB", flush=True)
            if metrics_f:
                rec = {"step": step, "loss": metrics["loss"], "lr": metrics["lr"], "tokens": metrics["tokens"],
                       "elapsed_s": elapsed,
                       **({"loss_global": metrics["loss_global"]} if "loss_global" in metrics else {}),
                       "tokens_per_sec": tps, **mem}
                if trainer._last_norm is not None:
                    rec["grad_norm"] = float(trainer._last_norm)
                metrics_f.write(json.dumps(rec) + "\n")
                metrics_f.flush()
        if step > 0 and step % tc.save_interval == 0:
            t_ck = time.time()
            save(f"{tc.checkpoint_dir}/step_{step}")
            if steady_t0 is not None:  # checkpoint I/O is not training throughput
                steady_ckpt += time.time() - t_ck
    if trainer.device.type == "cuda":
        torch.cuda.synchronize(trainer.device)
    steady_t1 = time.time()
    prof.close()
    if not args.no_final_save:
        save(f"{tc.checkpoint_dir}/final")
    if trainer.is_main_process:
        total_time = time.time() - start_time
        print(f"\nTraining complete! Total time: {total_time:.2f}s")
        print(f"Tokens processed: {trainer.tokens_seen:,}")
        print(f"Peak memory: {trainer.get_memory_stats()['max_allocated_gb']:.2f} GB")
        if steady_t0 is not None:
            from .ddp_trainer import PEAK_BF16_FLOPS
            dt = max(steady_t1 - steady_t0 - steady_ckpt, 1e-9)
            sps = (trainer.tokens_seen - steady_tok0) / dt
            fpt = model_config.flops_per_token(model_config.max_seq_len, recompute=fc.activation_checkpointing)
            mfu = sps / trainer.world_size * fpt / PEAK_BF16_FLOPS
            print(f"Steady-state tokens/s (after step 10): {sps:,.0f} "
                  f"({sps / trainer.world_size:,.0f}/GPU, MFU {100 * mfu:.1f}% of {PEAK_BF16_FLOPS / 1e15:.1f} PF dense bf16)")
            if metrics_f:
                metrics_f.write(json.dumps({"summary": True, "steady_tokens_per_sec": sps,
                                            "tokens_per_sec_per_gpu": sps / trainer.world_size, "mfu": mfu,
                                            **trainer.get_memory_stats()}) + "\n")
    if metrics_f:
        metrics_f.close()
    if trainer.distributed:
        dist.destroy_process_group()
    return trainer


if __name__ == "__main__":
    main()
