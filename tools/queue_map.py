"""Kernels per (HSA queue, stream) of the last optimizer step of a rocprofv3 kernel trace.

HIP binds a stream to a hardware queue at its first dispatch; which queue a compute stream
lands on decides what it shares (profiles/r4_opt_overlap.md).  Prints, per (queue, stream):
kernel count, summed kernel time (ms) and the two most frequent kernels.

usage: python tools/queue_map.py run_kernel_trace.csv
"""
import csv
import sys
from collections import Counter, defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "k_sumsq" in r["Kernel_Name"]]
    step = rows[opt[-2] + 1:opt[-1] + 1] if len(opt) >= 2 else rows
    busy, count, names = defaultdict(float), Counter(), defaultdict(Counter)
    for r in step:
        k = (int(r["Queue_Id"]), int(r["Stream_Id"]))
        busy[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        count[k] += 1
        names[k][r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]] += 1
    for k in sorted(busy):
        print(f"queue {k[0]:2d} stream {k[1]:2d}: {count[k]:4d} kernels {busy[k]:7.2f} ms  {names[k].most_common(2)}")


if __name__ == "__main__":
    main(sys.argv[1])
