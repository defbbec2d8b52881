"""Single-GPU / data-parallel trainer (CLI- and API-compatible with the reference's
``src/training/ddp_trainer.py``).

Reference call stack: torchrun -> main() -> DistributedTrainer ->
DDP(GPT) + fused AdamW -> train_step (GA micro-loop, no_sync, autocast, clip, step).

MI355X design:
* bf16 (the default and the headline config) runs the fused executor
  (``models/engine.py``) on the HIP kernels; weights are views into a flat fp32
  master buffer with a bf16 shadow (``parallel/flat.py``).
* Data parallelism is ``parallel/ddp.py``: zero-copy 64 MB buckets all-reduced over
  RCCL as soon as each group of layers finishes its backward.
* Loss is accumulated on the device; the only host sync per optimizer step is the
  logged loss value (the reference syncs on every micro-step, Q10).
* fp32 / fp16 run the same fused executor with fp32 master weights and a shadow in the
  compute dtype (fp16 with dynamic loss scaling, GradScaler's defaults); on CPU the
  fused executor runs with the PyTorch reference ops in fp32.

Intentional fixes (documented in README "Divergences"): LR is set before the
optimizer step and the cosine is clamped (Q5/Q6, switch off with
``lr_schedule_fix=False``), seeded init (Q13), working ``--resume_from`` (Q8) and
``--config`` YAML (Q1).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..models.config import GPTConfig
from ..models.gpt import GPT, count_parameters
from ..parallel.ddp import DDPRuntime
from ..parallel.flat import FlatParamStore
from ..utils import checkpoint as ckpt
from ..utils import debug as dbg
from ..utils.profiling import Profiler, range_push, range_pop
from .common import cosine_lr, gemm_plan_hook, global_mean_loss, memory_stats, micro_step_fusion, seed_all, select_device, setup_distributed, unwrap_batch
from .configs import TrainingConfig
from .optim import flat_store_optimizer


PEAK_BF16_FLOPS = 2.5e15  # MI355X dense bf16 MFMA peak (no sparsity), for MFU reporting


class DistributedTrainer:
    """DDP trainer.  ``train_step(batch) -> {"loss", "lr", "tokens"}``."""

    def __init__(self, model_config: GPTConfig, training_config: TrainingConfig, use_engine: Optional[bool] = None):
        self.model_config = model_config
        self.training_config = training_config
        self._setup_distributed()
        self._setup_device(use_engine)
        self._setup_model()
        self._setup_optimizer()
        self.global_step = 0
        self.tokens_seen = 0
        self._last_norm = None
        self._grads_zeroed = False
        self._engine_warm = False

    # ------------------------------------------------------------------ setup
    def _setup_distributed(self):
        self.distributed, self.rank, self.world_size, self.local_rank = setup_distributed()
        self.is_main_process = self.rank == 0
        if self.is_main_process:
            print(f"Distributed training: {self.distributed}")
            print(f"World size: {self.world_size}")

    def _setup_device(self, use_engine):
        self.device = select_device(self.local_rank)
        mp = self.training_config.mixed_precision
        cuda = self.device.type == "cuda"
        if use_engine is None:
            use_engine = True
        self.use_engine = use_engine
        self.autocast_ctx = contextlib.nullcontext()
        self.loss_scale = None
        self._good_steps = 0
        # reference ddp_trainer.py:129-152: bf16 autocast, fp16 autocast + GradScaler, or
        # fp32.  Here every mode runs the fused engine with fp32 master weights and a
        # compute-dtype shadow: bf16 and fp16 on the HIP kernels (fp16: the same kernels
        # instantiated for IEEE half, the hand weight / data gradient GEMMs in fp16 and
        # hipBLASLt fp16 forward GEMMs, dynamic loss scaling -- 2^16,
        # x0.5 and skip on inf/nan, x2 after 2000 good steps: GradScaler defaults); fp32
        # (the reference / debug mode) with PyTorch ops on the GPU + hipBLASLt GEMMs
        if cuda and mp == "bf16":
            self.dtype = torch.bfloat16
        elif cuda and mp == "fp16":
            self.dtype = torch.float16
            self.loss_scale = 2.0 ** 16
            if not use_engine:
                self.autocast_ctx = torch.autocast(device_type="cuda", dtype=torch.float16)
        else:
            self.dtype = torch.float32
        if self.is_main_process:
            path = ("fused HIP engine" if self.dtype in (torch.bfloat16, torch.float16) else
                    "fused engine (PyTorch ops + hipBLASLt on the GPU: fp32 reference mode)") if (use_engine and cuda) \
                else ("fused engine (CPU reference ops)" if use_engine else "eager")
            print(f"Device: {self.device}")
            print(f"Mixed precision: {mp} (dtype: {self.dtype}) | execution: {path}")

    def _setup_model(self):
        seed_all(self.training_config.seed)
        model = GPT(self.model_config)
        self.model = model.to(self.device)
        if self.is_main_process:
            print(f"Model parameters: {count_parameters(self.model):,}")
        if self.use_engine:
            act = self.dtype if self.device.type == "cuda" else None
            eng = self.model.enable_engine(seed=self.training_config.seed + 1000003 * self.rank, act_dtype=act)
            if self.training_config.memory_first:
                if self.training_config.defer_roles == "all":
                    # memory-first defers no weight gradient unless the config names roles
                    self.training_config.defer_roles = LEAN_DEFER_ROLES
                eng.s_refill = os.environ.get("DLT_S_REFILL", "1") != "0"
            eng.defer_roles = parse_defer_roles(self.training_config.defer_roles)
            if "head" not in eng.defer_roles and not eng.head_chunks_env:
                # memory-lean: chunked lm_head run in the forwards (GPTEngine); memory-first
                # (unfused 8192-row micro-steps) takes each micro-step's rows in one chunk:
                # +0.4 GB, +3 % (tools/ab/r6/memfirst_ab.sh)
                eng.head_chunks = 1 if self.training_config.memory_first else 2
            self.store = self.model.store
        else:
            self.store = FlatParamStore(self.model, self.device, compute_dtype=torch.float32)
        self.ddp = None
        if self.distributed:
            rd = torch.bfloat16 if self.training_config.reduce_dtype == "bf16" else torch.float32
            self.ddp = DDPRuntime(self.store, bucket_cap_mb=self.training_config.bucket_cap_mb, reduce_dtype=rd)

    def _setup_optimizer(self):
        c = self.training_config
        self.optimizer = flat_store_optimizer(self.store, c.learning_rate, (c.beta1, c.beta2), c.adam_eps,
                                              c.weight_decay, split_no_decay=True)

    def fusion_factor(self, GA: int, micro_bs: int, seq_len: int) -> int:
        gpu_engine = self.use_engine and self.device.type == "cuda"
        req = self.training_config.micro_step_fusion
        if self.training_config.memory_first and req == 0:
            req = 1  # one micro-step's activations per chain
        return micro_step_fusion(req, GA, micro_bs, seq_len, gpu_engine)

    def chains_per_step(self) -> int:
        """Engine forwards per optimizer step (dropout streams are keyed by this count)."""
        c = self.training_config
        GA = c.gradient_accumulation_steps
        return GA // self.fusion_factor(GA, c.batch_size, self.model_config.max_seq_len)

    # --------------------------------------------------------------- schedule
    def get_lr(self, step: int) -> float:
        c = self.training_config
        return cosine_lr(step, c.learning_rate, c.warmup_steps, c.max_steps, clamp=c.lr_schedule_fix)

    # ------------------------------------------------------------------- step
    def train_step(self, batch, sync_loss: bool = True) -> dict:
        cfg = self.training_config
        self.model.train()
        if cfg.lr_schedule_fix:
            lr = self.get_lr(self.global_step)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
        if not self._grads_zeroed:  # the previous step already zeroed them (saves a 600 MB memset)
            self.optimizer.zero_grad(set_to_none=True)
        self._grads_zeroed = False
        input_ids = unwrap_batch(batch).to(self.device, non_blocking=True)
        GA = cfg.gradient_accumulation_steps
        micro_bs = input_ids.shape[0] // GA
        # F micro-steps per executed chain (see TrainingConfig.micro_step_fusion); the
        # gradient is still the average of GA per-micro-step mean losses
        F = self.fusion_factor(GA, micro_bs, input_ids.shape[1])
        chains, chain_bs = GA // F, micro_bs * F
        if self.use_engine:
            self.model.engine.set_loss_segments(F)
            # fp16: the cross-entropy gradient is stored pre-scaled by the loss scale (no
            # fp16 underflow); the engine divides it out where dloss is applied
            self.model.engine.ce_grad_scale = float(self.loss_scale or 1.0)
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        # micro-step pipelining (engine.train_window): from the second step on, so the
        # first one runs the GEMM autotuning on a quiet GPU
        window_ok = (self.use_engine and chains > 1 and cfg.pipeline_micro_steps
                     and (self.device.type != "cuda" or getattr(self.model.engine.gemm, "stream_safe", False))
                     and os.environ.get("DLT_PIPELINE", "1") != "0")
        pipelined = window_ok and self._engine_warm
        # first step: the GEMM races time on a quiet GPU, so no stream pipelining -- but
        # when the window would run ffbb, its single-stream form (same block order, same
        # dY slot ring) keeps the first step's memory at the steady state's
        serial = (window_ok and not self._engine_warm and self.device.type == "cuda"
                  and self.model.engine.window_schedule(chains, cfg.defer_wgrad)[1] == "ffbb")
        pipelined = pipelined or serial
        if pipelined:
            ids_l = [input_ids[m * chain_bs:(m + 1) * chain_bs] for m in range(chains)]
            from ..models.engine import shift_targets
            tg_l = [shift_targets(x) for x in ids_l]
            if self.ddp is not None:
                self.ddp.require_sync(False)
            # fp16: the backward seed carries the loss scale, as (loss * scale).backward() does
            dloss = torch.full((), (self.loss_scale or 1.0) / chains, dtype=torch.float32, device=self.device)
            range_push("window")
            # defer_wgrad=False: each chain's weight gradients run in its own backward, so no
            # [GA*M, N] slot buffers and no window-wide dlogits are kept (defer_roles: per role)
            losses = self.model.engine.train_window(
                ids_l, tg_l, dloss, recompute=bool(self.model.gradient_checkpointing),
                before_last=(lambda: self.ddp.require_sync(True)) if self.ddp is not None else None,
                sync_hook=self.ddp.require_sync if self.ddp is not None else None,
                defer=cfg.defer_wgrad, serial=serial)
            range_pop()
            for loss in losses:
                total += (loss / chains).detach().float()
        for micro in range(0 if not pipelined else chains, chains):
            ids = input_ids[micro * chain_bs:(micro + 1) * chain_bs]
            if self.ddp is not None:
                self.ddp.require_sync(micro == chains - 1)
            if self.use_engine:
                self.model.engine.set_accumulation(micro, chains, defer=cfg.defer_wgrad)
            range_push(f"micro{micro}")
            with self.autocast_ctx:
                _, loss = self.model(ids, labels=ids)
                loss = loss / chains
            if self.loss_scale is not None:
                (loss * self.loss_scale).backward()
            else:
                loss.backward()
            range_pop()
            total += loss.detach().float()
        if self.use_engine:
            self.model.engine.set_loss_segments(1)
        self._engine_warm = self.use_engine
        if not self.use_engine:
            self.store.sync_grads_from_params()
            if self.ddp is not None:
                self.ddp.reduce_all_now()
        elif self.ddp is not None:
            self.ddp.finish()
        div = float(self.world_size) * (self.loss_scale or 1.0)
        scale = self.optimizer.compute_scale(cfg.grad_clip, grad_div=div)
        skip = False
        if self.loss_scale is not None:  # fp16 dynamic loss scaling (the all-reduced grads: one decision)
            if not torch.isfinite(scale[0]).item():
                self.loss_scale /= 2.0
                self._good_steps = 0
                skip = True
            else:
                self._good_steps += 1
                if self._good_steps % 2000 == 0:
                    self.loss_scale *= 2.0
        lazy = self._lazy_mode()
        if not skip and lazy != "off":
            # recorded, applied per unit by the next forward's pre_forward hooks (which
            # also zero each unit's gradient): the update overlaps the next step's compute
            if self.store.pending is not None and not self.store.pending.complete:
                self.store.flush_pending()
            self.store.pending = self.optimizer.step_lazy(scale, self.store.unit_ranges(), mode=lazy)
        else:
            if not skip:
                self.optimizer.step(scale)
                if not self.use_engine:
                    self.store.refresh_shadow()
            self.optimizer.zero_grad(set_to_none=True)
        self._last_norm = scale[0]
        self._grads_zeroed = True
        if not cfg.lr_schedule_fix:  # reference order: LR for the *next* step set after this one
            lr = self.get_lr(self.global_step)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
        else:
            lr = self.optimizer.param_groups[0]["lr"]
        self.global_step += 1
        self.tokens_seen += input_ids.numel() * self.world_size
        if self.use_engine and self.global_step >= 2:
            gemm_plan_hook()
        out = {"loss": total.item() if sync_loss else total, "lr": lr, "tokens": self.tokens_seen}
        if sync_loss and self.distributed and self.world_size > 1:
            out["loss_global"] = global_mean_loss(total, self.world_size)
        return out

    def _lazy_mode(self) -> str:
        """The optimizer-step mode of TrainingConfig.lazy_optimizer (engine path only;
        DLT_LAZY_OPT overrides): "inline", "stream" or "off"."""
        mode = os.environ.get("DLT_LAZY_OPT") or getattr(self.training_config, "lazy_optimizer", "inline")
        mode = {"0": "off", "1": "inline", "": "off"}.get(str(mode), str(mode))
        if mode not in ("inline", "stream", "off"):
            raise ValueError(f"lazy_optimizer must be inline / stream / off, got {mode!r}")
        return mode if self.use_engine else "off"

    def flush_optimizer(self) -> None:
        """Apply a recorded (lazy) optimizer step now: after this the parameters, the
        16-bit shadow and the zeroed gradients are what the reference's end-of-step
        ``optimizer.step(); zero_grad()`` leaves (``ddp_trainer.py:352-358``)."""
        self.store.flush_pending()

    def flat_params(self) -> torch.Tensor:
        """The flat fp32 master weights after every recorded optimizer step is applied."""
        self.flush_optimizer()
        return self.store.flat

    # ------------------------------------------------------------ checkpoints
    def save_checkpoint(self, path: str):
        self.flush_optimizer()
        if not self.is_main_process:
            return
        payload = {
            "model": ckpt.model_state_dict_cpu(self.model),
            "optimizer": self.optimizer.state_dict(),
            "global_step": self.global_step,
            "tokens_seen": self.tokens_seen,
            "model_config": self.model_config,
            "training_config": self.training_config,
        }
        ckpt.save_checkpoint(path, payload)

    def load_checkpoint(self, path: str):
        self.flush_optimizer()
        c = ckpt.load_checkpoint(path, map_location="cpu")
        ckpt.load_model_state(self.model, c["model"])
        self.store.refresh_shadow()
        self.optimizer.load_state_dict(c["optimizer"])
        self.global_step = int(c["global_step"])
        self.tokens_seen = int(c["tokens_seen"])
        if self.use_engine:  # dropout streams continue exactly where the saved run was
            self.model.engine.micro_counter = self.global_step * self.chains_per_step()
        if self.is_main_process:
            print(f"Loaded Checkpoint from {path} (step {self.global_step})")

    def get_memory_stats(self) -> dict:
        return memory_stats(self.device)


# --------------------------------------------------------------------------- CLI
# --memory_lean: no weight gradient deferred to the window -- every chain runs its own
# (no [GA*M, N] slot buffers), the lm_head in row chunks in the forwards: 11.9 GB at the
# headline shape vs 14.9 GB deferring qkv / o ("qkv,o", the round-3 choice), -0.7 %
# (profiles/r4_memory_lean.md)
LEAN_DEFER_ROLES = "none"


def parse_defer_roles(text: str) -> frozenset:
    """TrainingConfig.defer_roles -> the engine's role set ("all", "none" or a comma list)."""
    from ..models.engine import GPTEngine
    if text.strip() in ("", "all"):
        return frozenset(GPTEngine.ROLES)
    if text.strip() == "none":
        return frozenset()
    roles = frozenset(r.strip() for r in text.split(",") if r.strip())
    bad = roles - set(GPTEngine.ROLES)
    if bad:
        raise ValueError(f"defer_roles: unknown roles {sorted(bad)} (choose from {GPTEngine.ROLES})")
    return roles


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X DDP trainer (reference-compatible CLI)")
    p.add_argument("--model_size", type=str, default="small", choices=["small", "medium", "large", "xl"])
    p.add_argument("--batch_size", type=int, default=8)
    p.add_argument("--max_steps", type=int, default=1000)
    p.add_argument("--mixed_precision", type=str, default="bf16", choices=["fp32", "fp16", "bf16"])
    p.add_argument("--gradient_checkpointing", action="store_true")
    p.add_argument("--dataset", type=str, default="dummy", choices=["dummy", "tinystories", "openwebtext"])
    p.add_argument("--data_path", type=str, default=None)
    p.add_argument("--max_tokens", type=int, default=None)
    p.add_argument("--streaming", action="store_true")
    p.add_argument("--cache_max_tokens", type=int, default=None)
    # additions
    p.add_argument("--config", type=str, default=None, help="YAML config (configs/*.yaml); CLI flags override it")
    p.add_argument("--resume_from", type=str, default=None)
    p.add_argument("--checkpoint_dir", type=str, default=None)
    p.add_argument("--save_interval", type=int, default=None)
    p.add_argument("--log_interval", type=int, default=None)
    p.add_argument("--learning_rate", type=float, default=None)
    p.add_argument("--warmup_steps", type=int, default=None)
    p.add_argument("--gradient_accumulation_steps", type=int, default=None)
    p.add_argument("--seq_len", type=int, default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--tokenizer", type=str, default="gpt2")
    p.add_argument("--profile", type=str, default=None, help="write a torch.profiler trace to this dir")
    p.add_argument("--metrics_jsonl", type=str, default=None)
    p.add_argument("--no_final_save", action="store_true")
    p.add_argument("--memory_first", action="store_true",
                   help="peak memory first: --memory_lean + unfused micro-steps + the SwiGLU output rewritten "
                        "by the backward (TrainingConfig.memory_first; ~7 GB at the headline shape, "
                        "profiles/r6_memory.md)")
    p.add_argument("--memory_lean", action="store_true",
                   help="no weight gradient deferred to the end of the accumulation window: every micro-step "
                        "chain runs its own (no [GA*M, N] slot buffers, no window-wide dlogits; lm_head in row "
                        "chunks): ~56 %% of the default peak memory at -3 %% tok/s")
    return p


def main(argv=None):
    from ..utils.config_loader import explicit_args, load_yaml_config
    parser = build_parser()
    args = parser.parse_args(argv)
    given = explicit_args(parser, argv)

    model_config = GPTConfig.from_preset(args.model_size)
    tc = TrainingConfig(batch_size=args.batch_size, max_steps=args.max_steps, mixed_precision=args.mixed_precision)
    if args.config:
        model_config, tc, _, data_cfg = load_yaml_config(args.config, model_config, tc, None,
                                                         keep_model_preset="model_size" in given)
        # CLI flags that were explicitly given still win
        for k in ("batch_size", "max_steps", "mixed_precision"):
            if k in given:
                setattr(tc, k, getattr(args, k))
        if "dataset" not in given and data_cfg.get("dataset") in ("dummy", "tinystories", "openwebtext"):
            args.dataset = data_cfg["dataset"]
    if args.gradient_checkpointing:
        model_config.gradient_checkpointing = True
    for k in ("resume_from", "checkpoint_dir", "save_interval", "log_interval", "learning_rate", "warmup_steps",
              "gradient_accumulation_steps", "seed"):
        v = getattr(args, k)
        if v is not None:
            setattr(tc, k, v)
    if args.seq_len:
        model_config.max_seq_len = args.seq_len
    if args.memory_lean:
        tc.defer_roles = LEAN_DEFER_ROLES
    if args.memory_first:
        tc.memory_first = True

    trainer = DistributedTrainer(model_config, tc)
    if tc.resume_from:
        trainer.load_checkpoint(tc.resume_from)

    loader_bs = tc.batch_size * tc.gradient_accumulation_steps
    seq_len = model_config.max_seq_len
    if args.dataset in ("tinystories", "openwebtext"):
        if args.data_path is None:
            raise ValueError(f"{args.dataset} dataset requires --data_path")
        from ..data import create_openwebtext_dataloader, create_tinystories_dataloader
        fn = create_tinystories_dataloader if args.dataset == "tinystories" else create_openwebtext_dataloader
        dataloader = fn(path=args.data_path, batch_size=loader_bs, seq_len=seq_len, distributed=trainer.distributed,
                        rank=trainer.rank, world_size=trainer.world_size, tokenizer_name=args.tokenizer,
                        max_tokens=args.max_tokens, streaming=args.streaming,
                        cache_max_tokens=args.cache_max_tokens, num_workers=0 if args.streaming else 2,
                        seed=tc.seed, device=trainer.device)
    else:
        from ..data import create_dummy_dataloader
        dataloader = create_dummy_dataloader(batch_size=loader_bs, seq_len=seq_len,
                                             vocab_size=model_config.vocab_size, distributed=trainer.distributed,
                                             rank=trainer.rank, world_size=trainer.world_size,
                                             num_batches=int(os.environ.get("DLT_DUMMY_BATCHES", "64")),
                                             seed=tc.seed, device=trainer.device)
    if hasattr(dataloader, "seek") and trainer.global_step:
        dataloader.seek(trainer.global_step)  # native loader: resume the exact batch stream

    if trainer.is_main_process:
        print("\n" + "=" * 60)
        print("Starting training...")
        print("=" * 60 + "\n")
    metrics_f = open(args.metrics_jsonl, "a") if (args.metrics_jsonl and trainer.is_main_process) else None
    prof = Profiler(args.profile, enabled=bool(args.profile) and trainer.is_main_process)
    data_iter = iter(dataloader)
    check_every = dbg.replica_check_interval()
    if check_every:
        dbg.check_replicas(trainer.store.flat)
    start_time = time.time()
    start_step = trainer.global_step
    tokens0 = trainer.tokens_seen  # tokens of a resumed run's earlier steps are not this run's throughput
    steady_t0, steady_tok0, steady_ckpt = None, 0, 0.0
    for step in range(start_step, tc.max_steps):
        dbg.maybe_inject_fault(step, trainer.rank)
        try:
            batch = next(data_iter)
        except StopIteration:
            if hasattr(dataloader.sampler, "set_epoch"):
                dataloader.sampler.set_epoch(step)
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
            print(f"Step {step:6d} | Loss: {metrics['loss']:.4f} | LR: {metrics['lr']:.2e} | Tokens/sec: {tps:,.0f}",
                  flush=True)
            if metrics_f:
                rec = {"step": step, "loss": metrics["loss"], "lr": metrics["lr"], "tokens": metrics["tokens"],
                       "elapsed_s": elapsed,
                       **({"loss_global": metrics["loss_global"]} if "loss_global" in metrics else {}),
                       "tokens_per_sec": tps, **trainer.get_memory_stats()}
                if trainer._last_norm is not None:
                    rec["grad_norm"] = float(trainer._last_norm)
                metrics_f.write(json.dumps(rec) + "\n")
                metrics_f.flush()
        if check_every and (step + 1) % check_every == 0:
            dbg.check_replicas(trainer.store.flat)
        if step > 0 and step % tc.save_interval == 0:
            t_ck = time.time()
            trainer.save_checkpoint(f"{tc.checkpoint_dir}/step_{step}.pt")
            if steady_t0 is not None:  # checkpoint I/O is not training throughput
                steady_ckpt += time.time() - t_ck
    if trainer.device.type == "cuda":
        torch.cuda.synchronize(trainer.device)
    steady_t1 = time.time()
    prof.close()
    if not args.no_final_save:
        trainer.save_checkpoint(f"{tc.checkpoint_dir}/final.pt")
    if trainer.distributed:
        dist.barrier()
        dist.destroy_process_group()
    if trainer.is_main_process:
        total_time = time.time() - start_time
        print(f"\nTraining complete! Total time: {total_time:.2f}s")
        print(f"Total tokens processed: {trainer.tokens_seen:,}")
        if steady_t0 is not None:
            dt = max(steady_t1 - steady_t0 - steady_ckpt, 1e-9)
            sps = (trainer.tokens_seen - steady_tok0) / dt
            fpt = model_config.flops_per_token(seq_len, recompute=bool(model_config.gradient_checkpointing))
            mfu = sps / trainer.world_size * fpt / PEAK_BF16_FLOPS
            print(f"Steady-state tokens/sec (after step 10): {sps:,.0f} "
                  f"({sps / trainer.world_size:,.0f}/GPU, MFU {100 * mfu:.1f}% of {PEAK_BF16_FLOPS / 1e15:.1f} PF dense bf16)")
            if metrics_f:
                metrics_f.write(json.dumps({"summary": True, "steady_tokens_per_sec": sps,
                                            "tokens_per_sec_per_gpu": sps / trainer.world_size, "mfu": mfu,
                                            **trainer.get_memory_stats()}) + "\n")
        ms = trainer.get_memory_stats()
        print(f"Peak memory: {ms['max_allocated_gb']:.2f} GB")
    if metrics_f:
        metrics_f.close()
    return trainer


if __name__ == "__main__":
    main()
