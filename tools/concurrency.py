"""Concurrency view of one optimizer step from a rocprofv3 --kernel-trace CSV.

For the last step (between the last two k_sumsq dispatches, as tools/step_profile.py):
splits the step's span into intervals by kernel start/end events and attributes each
interval's length equally to the kernels running in it ("attributed" time: what a
kernel costs the step when others share the GPU), and reports how much of the span had
exactly 0 / 1 / 2 / 3+ kernels in flight, plus the kernels that ran ALONE the longest
(alone time is fully on the critical path).

usage: python tools/concurrency.py run_kernel_trace.csv [top]
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from step_profile import cat_of  # noqa: E402


def short(n):
    n = n.split("(")[0].replace("void ", "")
    return n[:70]


def main(path, top=20):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_sumsq" in r["Kernel_Name"]]
    if len(adam) < 2:
        sys.exit("need >= 2 optimizer steps in the trace")
    step = rows[adam[-2] + 1:adam[-1] + 1]
    ev = []
    for k, r in enumerate(step):
        ev.append((int(r["Start_Timestamp"]), 1, k))
        ev.append((int(r["End_Timestamp"]), -1, k))
    ev.sort()
    live = set()
    t_prev = ev[0][0]
    span = ev[-1][0] - ev[0][0]
    by_n = defaultdict(float)
    attr = defaultdict(float)
    alone = defaultdict(float)
    cat_attr = defaultdict(float)
    cat_alone = defaultdict(float)
    for t, kind, k in ev:
        dt = (t - t_prev) / 1e3
        if dt > 0:
            n = len(live)
            by_n[min(n, 3)] += dt
            for j in live:
                nm = short(step[j]["Kernel_Name"])
                attr[nm] += dt / n
                cat_attr[cat_of(step[j]["Kernel_Name"])] += dt / n
                if n == 1:
                    alone[nm] += dt
                    cat_alone[cat_of(step[j]["Kernel_Name"])] += dt
        t_prev = t
        if kind == 1:
            live.add(k)
        else:
            live.discard(k)
    print(f"step span {span / 1e6:.2f} ms; kernels in flight: " +
          ", ".join(f"{'3+' if n == 3 else n}: {v / 1e3:.2f} ms ({100 * v * 1e3 / span:.1f}%)"
                    for n, v in sorted(by_n.items())))
    print("\n| category | attributed ms | alone ms |\n|---|---:|---:|")
    for c, v in sorted(cat_attr.items(), key=lambda x: -x[1]):
        print(f"| {c} | {v / 1e3:.2f} | {cat_alone[c] / 1e3:.2f} |")
    print("\n| kernel | attributed ms | alone ms |\n|---|---:|---:|")
    for nm, v in sorted(attr.items(), key=lambda x: -x[1])[:top]:
        print(f"| `{nm}` | {v / 1e3:.2f} | {alone[nm] / 1e3:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
