"""Per-step kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV.

Takes the kernels of the LAST optimizer step (between the last two ``k_sumsq``
dispatches), so warmup / GEMM-planner autotuning does not pollute the numbers, and
groups them into categories.  Also reports the step's wall span (first kernel start to
last kernel end) vs the summed kernel time -> GPU idle (launch gaps).

usage: python tools/step_profile.py run_kernel_trace.csv [micro_steps]
"""
import csv
import os
import re
import sys
from collections import defaultdict

CATS = [
    ("attn fwd", r"k_attn_fwd"),
    ("attn bwd dkdv", r"k_attn_bwd_dkdv"),
    ("attn bwd dq", r"k_attn_bwd_dq"),
    ("attn bwd delta", r"k_attn_bwd_delta"),
    ("dropout mask", r"k_dropout_bits"),
    ("rmsnorm fwd", r"k_add_dropout_rmsnorm_fwd"),
    ("rmsnorm bwd", r"k_rmsnorm_bwd"),
    ("swiglu", r"k_swiglu"),
    ("rope", r"k_rope"),
    ("cross entropy", r"k_ce_"),
    ("embedding", r"k_embedding"),
    ("optimizer", r"k_adamw|k_sumsq|k_clip|k_cast"),
    ("GEMM (hipBLASLt)", r"^Cijk|^Custom_Cijk"),
    ("GEMM (hand-written)", r"k_wgrad_gemm|k_gemm"),
    ("RCCL", r"ncclDevKernel|ncclKernel|rccl"),
    ("torch elementwise/copy", r"at::native|__amd_rocclr"),
]


def cat_of(name):
    for c, pat in CATS:
        if re.search(pat, name):
            return c
    return "other"


def main(path, micro=4):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_sumsq" in r["Kernel_Name"]]
    if len(adam) < 2:
        sys.exit("need >= 2 optimizer steps in the trace")
    lo, hi = adam[-2] + 1, adam[-1] + 1
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    by = defaultdict(lambda: [0.0, 0])
    names = defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        c = cat_of(r["Kernel_Name"])
        by[c][0] += d
        by[c][1] += 1
        n = r["Kernel_Name"]
        names[n[:90]][0] += d
        names[n[:90]][1] += 1
    span = (t1 - t0) / 1e3
    # union of kernel intervals: time with >= 1 kernel running (rest = GPU idle)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            union += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    union += ce - cs
    print(f"Last optimizer step: span {span / 1e3:.2f} ms, kernel-busy {busy / 1e3:.2f} ms "
          f"({100 * busy / span:.1f}% busy), {len(step)} kernels; per micro-step ({micro}): {busy / 1e3 / micro:.2f} ms")
    print(f"GPU occupied (>=1 kernel running) {union / 1e6:.2f} ms = {100 * union / 1e3 / span:.1f}% of the span; "
          f"idle {span / 1e3 - union / 1e6:.2f} ms")
    print()
    print("| category | ms/step | % | launches |")
    print("|---|---:|---:|---:|")
    for c, (t, n) in sorted(by.items(), key=lambda kv: -kv[1][0]):
        print(f"| {c} | {t / 1e3:.2f} | {100 * t / busy:.1f} | {n} |")
    print()
    print("| kernel | ms/step | launches | avg us |")
    print("|---|---:|---:|---:|")
    for n, (t, k) in sorted(names.items(), key=lambda kv: -kv[1][0])[:int(os.environ.get("STEP_PROFILE_TOP", "25"))]:
        print(f"| `{n.replace('|', '/')}` | {t / 1e3:.3f} | {k} | {t / k:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
