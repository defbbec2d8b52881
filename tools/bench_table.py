"""Benchmark harness: run bench.py over a set of configurations and write a
BASELINE.md-style markdown table.

Each configuration runs in its own process (N > 1 through torch.distributed.run, one
rank per GPU, 127.0.0.1 rendezvous).  Usage:
  python tools/bench_table.py --gpus 1 --out profiles/r1_bench_table.md
  python tools/bench_table.py --gpus 1,2,4,8 --configs ddp_small,fsdp_small
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = {("ddp", "small", 1): 12500, ("ddp", "small", 2): 24100, ("ddp", "small", 4): 46800,
       ("fsdp", "small", 4): 44200}  # BASELINE.md (reference README.md:191-197)

CONFIGS = {
    "ddp_small": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4"],
    "ddp_small_lean": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4", "--memory_lean"],
    "ddp_small_memfirst": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4", "--memory_first"],
    "ddp_small_fp16": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4", "--precision", "fp16"],
    "ddp_small_fp32": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4", "--precision", "fp32"],
    # head_dim 128 (6 heads of the small model's 768): the D = 128 MFMA attention kernels
    "ddp_small_hd128": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4",
                        "--model_override", "num_heads=6"],
    # head_dim 96 (8 heads of 768): no flash kernel, attention as 16-bit GEMMs (ops/attn_gemm.py)
    "ddp_small_hd96": ["--model_size", "small", "--batch_size", "8", "--grad_accum", "4",
                       "--model_override", "num_heads=8"],
    "fsdp_small": ["--mode", "fsdp", "--model_size", "small", "--batch_size", "8", "--grad_accum", "4"],
    "ddp_medium": ["--model_size", "medium", "--batch_size", "4", "--grad_accum", "8"],
    "fsdp_medium": ["--mode", "fsdp", "--model_size", "medium", "--batch_size", "4", "--grad_accum", "8"],
    "fsdp_medium_noac": ["--mode", "fsdp", "--model_size", "medium", "--batch_size", "4", "--grad_accum", "8",
                         "--no_ac"],
    "ddp_xl": ["--model_size", "xl", "--batch_size", "4", "--grad_accum", "8"],
    "fsdp_xl": ["--mode", "fsdp", "--model_size", "xl", "--batch_size", "4", "--grad_accum", "8"],
}


def run(n, args, steps, warmup, timeout):
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup), *args]
    if n > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(29600 + n), *cmd[1:]]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    for line in reversed(r.stdout.splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise RuntimeError(f"{' '.join(cmd)} failed (rc {r.returncode}):\n{r.stderr[-2000:]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1")
    ap.add_argument("--configs", default="ddp_small,fsdp_small,ddp_medium,fsdp_medium,fsdp_medium_noac,ddp_xl,fsdp_xl")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = ["| GPUs | config | tokens/s | ms / step | peak GB/GPU | final loss | vs reference |",
             "|---:|---|---:|---:|---:|---:|---|"]
    for n in [int(x) for x in a.gpus.split(",")]:
        for name in a.configs.split(","):
            res = run(n, CONFIGS[name], a.steps, a.warmup, a.timeout)
            mode, size = name.split("_")[0], name.split("_")[1]
            ref = REF.get((mode, size, n)) if name.count("_") == 1 else None  # variants: no reference row
            vs = f"{res['value'] / ref:.1f}x ({ref:,})" if ref else "--"
            lines.append(f"| {n} | {name} | {res['value']:,.0f} | {res['ms_per_step']:.1f} | "
                         f"{res['peak_gb_per_gpu']:.1f} | {res['final_loss']:.3f} | {vs} |")
            print(lines[-1], flush=True)
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(f"# bench.py table ({a.steps} timed steps after {a.warmup} warmup, synthetic data)\n\n" + text)
    print(text)


if __name__ == "__main__":
    main()
