"""Byte model of the gradient / parameter collectives per optimizer step on one 8x MI355X
node (xGMI full mesh), for the configs BASELINE.json names.

For each config: bytes each rank moves per collective kind, the wire time at a given
bus bandwidth, how much of it the schedule can hide behind compute, and the exposed
remainder as a share of the measured 1-GPU step time.

Ring collectives on W ranks (RCCL's default for these sizes): all-reduce moves
2 (W-1)/W x S per rank, reduce-scatter and all-gather (W-1)/W x S.  On a fully connected
8-GPU xGMI mesh RCCL builds several rings over distinct links; the bus bandwidth is
modelled as eff x links x per-direction link bandwidth (7 links x 76.5 GB/s per direction
= 535 GB/s peak injection per GPU) and reported for a range of eff.

What is exposed:
* DDP: the engine issues each 64 MB bucket when its last layer's weight gradients are
  final (layer-granular post_backward) and the side stream keeps computing the remaining
  layers' weight gradients, so all buckets but the last overlap the backward.  The last
  ("head") bucket -- the tied embedding / lm_head gradient (Vp x H fp32) plus every norm
  weight -- is final only after the embedding scatter-add of the residual gradient at the
  model input, i.e. at the very end of the backward; only layer 0's weight gradients
  remain to overlap it.  Its all-reduce is the exposed part (the clip norm needs it).
* FSDP: all-gathers are prefetched one unit ahead and reduce-scatters trail by one unit;
  the exposed part is modelled as the first unit's all-gather plus the last unit's
  reduce-scatter per micro-step, and any excess of total wire time over compute time.

usage: python tools/comm_model.py [--link_gbs 76.5] [--links 7] > profiles/r5_comm_model.md
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_trainer_amd.models.config import GPTConfig  # noqa: E402

# measured 1-GPU step times (ms) of the same per-GPU work (weak scaling), from the bench
# tables: DDP small = BENCH_r04 (32 x 1024 tokens); FSDP from profiles/r3b_bench_table.md
# (bs 4 x GA 8 x 1024 tokens per step: 757k / 279k / 64.8k tok/s)
STEP_MS = {"ddp_small": 41.3, "fsdp_small": 32768 / 757e3 * 1e3, "fsdp_medium": 32768 / 279e3 * 1e3,
           "fsdp_xl": 32768 / 64.8e3 * 1e3}


def param_counts(cfg: GPTConfig):
    H, I, L, Vp = cfg.hidden_size, cfg.intermediate_size, cfg.num_layers, cfg.vocab_size_padded
    block = 4 * H * H + 3 * H * I + 2 * H
    root = Vp * H + H
    return block, root, L


def ddp_model(cfg, W, bus, bucket_mb=64.0, reduce_bytes=4):
    block, root, L = param_counts(cfg)
    total = (block * L + root) * reduce_bytes
    head = (cfg.vocab_size_padded * cfg.hidden_size + (2 * L + 1) * cfg.hidden_size) * reduce_bytes
    ring = 2 * (W - 1) / W
    t_total = ring * total / bus * 1e3
    t_head = ring * head / bus * 1e3
    return {"bytes_per_rank_GB": ring * total / 1e9, "wire_ms": t_total, "exposed_ms": t_head,
            "buckets": int(-(-(total - head) // (bucket_mb * 2 ** 20))) + 1}


def fsdp_model(cfg, W, bus, GA=8, ac=True, shard="FULL_SHARD"):
    block, root, L = param_counts(cfg)
    f = (W - 1) / W
    # bf16 unit all-gathers: forward (root + every block), backward again for the blocks
    # under FULL_SHARD (resharded after forward), reduce-scatter of bf16 grads per unit,
    # every micro-step (the reference reduces on every micro-step: no no_sync)
    ag_units = (root + block * L) + (block * L if shard == "FULL_SHARD" else 0)
    ag = f * ag_units * 2 * GA
    rs = f * (root + block * L) * 2 * GA
    t_ag, t_rs = ag / bus * 1e3, rs / bus * 1e3
    exposed_first = (f * (root * 2) / bus + f * (block * 2) / bus) * 1e3 * GA  # first AG + last RS per micro-step
    return {"bytes_per_rank_GB": (ag + rs) / 1e9, "wire_ms": t_ag + t_rs, "ag_ms": t_ag, "rs_ms": t_rs,
            "exposed_floor_ms": exposed_first}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--link_gbs", type=float, default=76.5, help="xGMI bandwidth per link per direction (GB/s)")
    ap.add_argument("--links", type=int, default=7)
    a = ap.parse_args(argv)
    peak = a.link_gbs * a.links * 1e9
    effs = (0.4, 0.6, 0.8)
    print("# Collective byte model per optimizer step, 8x MI355X (xGMI full mesh)\n")
    print(f"`python tools/comm_model.py` -- peak injection {a.links} links x {a.link_gbs} GB/s = "
          f"{peak / 1e9:.0f} GB/s per GPU per direction; bus bandwidth = eff x peak.  Step times: the "
          "measured 1-GPU step of the same per-GPU work (weak scaling).  Model assumptions in the tool's "
          "docstring.\n")
    small, medium, xl = (GPTConfig.from_preset(p) for p in ("small", "medium", "xl"))
    print("## DDP (GPT-2 small, micro-batch 8 x GA 4 per GPU, fp32 gradients, 64 MB buckets)\n")
    print("| W | eff | bus GB/s | bytes/rank/step | wire ms | exposed (head bucket) ms | step ms | exposed % |"
          " bf16 wire: exposed ms |")
    print("|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for W in (2, 4, 8):
        for e in effs:
            bus = e * peak
            d = ddp_model(small, W, bus)
            d16 = ddp_model(small, W, bus, reduce_bytes=2)
            st = STEP_MS["ddp_small"]
            print(f"| {W} | {e} | {bus / 1e9:.0f} | {d['bytes_per_rank_GB']:.2f} GB | {d['wire_ms']:.2f} | "
                  f"{d['exposed_ms']:.2f} | {st:.1f} | {100 * d['exposed_ms'] / st:.1f} % | {d16['exposed_ms']:.2f} |")
    print()
    print("## FSDP FULL_SHARD (bs 4 x GA 8 per GPU, bf16 all-gather / reduce-scatter every micro-step)\n")
    print("| config | W | eff | bytes/rank/step | AG ms | RS ms | wire ms | step ms | wire / step | "
          "exposed floor ms |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, cfg, Ws in (("small", small, (8,)), ("medium", medium, (4, 8)), ("xl", xl, (8,))):
        for W in Ws:
            for e in effs:
                bus = e * peak
                d = fsdp_model(cfg, W, bus)
                st = STEP_MS[f"fsdp_{name}"]
                print(f"| {name} | {W} | {e} | {d['bytes_per_rank_GB']:.2f} GB | {d['ag_ms']:.1f} | {d['rs_ms']:.1f} | "
                      f"{d['wire_ms']:.1f} | {st:.0f} | {d['wire_ms'] / st:.2f} | {d['exposed_floor_ms']:.2f} |")
    print()
    d8 = [ddp_model(small, 8, e * peak)["exposed_ms"] for e in effs]
    fx = [fsdp_model(xl, 8, e * peak)["wire_ms"] / STEP_MS["fsdp_xl"] for e in effs]
    print(f"Reading: DDP small exposes only the head bucket's all-reduce (the 154 MB tied embedding "
          f"gradient + every norm weight): {min(d8):.2f}-{max(d8):.2f} ms at W = 8, "
          f"{100 * min(d8) / STEP_MS['ddp_small']:.1f}-{100 * max(d8) / STEP_MS['ddp_small']:.1f} % of the step; "
          "a bf16 wire (TrainingConfig.reduce_dtype) halves it.  Splitting that bucket (the lm_head "
          "weight-gradient part early, the embedding scatter part late) does not shrink the exposed "
          "part: both parts are dense [Vp, H] tensors, so the late all-reduce moves the same bytes.  "
          f"FSDP moves the most: xl's wire time is {min(fx):.2f}-{max(fx):.2f} x its step's compute "
          "(every micro-step all-gathers every unit twice and reduce-scatters it once), so the "
          "prefetch / trailing reduce-scatter overlap carries FSDP scaling; small and medium stay "
          "under 0.75 x.")


if __name__ == "__main__":
    main()
