"""Summarise rocprofv3 --pmc passes (tools/ab/pmc.sh) into per-kernel hardware metrics.

Per kernel name (averaged over its dispatches; counters of different passes are joined
by kernel name, so each metric is an average over the same kind of dispatch):
  * MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs * CUs * 4 SIMDs)
    (GRBM_GUI_ACTIVE is summed over the 8 XCDs on MI355X: calibrated against the
    kernel's own duration -- 887k for a 43 us kernel at 2.4 GHz)
  * VALU / MFMA / LDS instructions per wave, LDS bank-conflict cycles per LDS instruction
  * FETCH / WRITE bytes (TCC <-> fabric/HBM), achieved bandwidth over the kernel's duration
  * L2 (TCC) hit rate
usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [top] [CUs]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    return n[:60]


def load(d):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("SQ_WAVES", "FETCH_SIZE"):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def avg(v):
    return sum(v) / len(v) if v else float("nan")


def main(d, top=25, cus=256, only=None):
    per, dur = load(d)
    rows = []
    for k, c in per.items():
        if only and not re.search(only, k):
            continue
        t = avg(dur[k])
        n = len(c.get("SQ_WAVES", [])) or len(c.get("FETCH_SIZE", []))
        rows.append((t * n, k, c, t, n))
    rows.sort(reverse=True)
    print("| kernel | calls | us | MFMA busy | VALU/wave | MFMA/wave | LDS/wave | LDS confl/LDS inst | fetch MB | write MB | GB/s | L2 hit |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for _, k, c, t, n in rows[:top]:
        waves = avg(c.get("SQ_WAVES", []))
        gui = avg(c.get("GRBM_GUI_ACTIVE", []))
        mb = avg(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        mfma = 100 * mb / (gui / 8 * cus * 4) if gui == gui and gui > 0 else float("nan")
        valu = avg(c.get("SQ_INSTS_VALU", [])) / waves if waves else float("nan")
        mf = avg(c.get("SQ_INSTS_MFMA", [])) / waves if waves else float("nan")
        lds = avg(c.get("SQ_INSTS_LDS", [])) / waves if waves else float("nan")
        li = avg(c.get("SQ_INSTS_LDS", []))
        conf = avg(c.get("SQ_LDS_BANK_CONFLICT", [])) / li if li else float("nan")
        fe = avg(c.get("FETCH_SIZE", [])) / 1024  # KB -> MB
        wr = avg(c.get("WRITE_SIZE", [])) / 1024
        bw = (fe + wr) / t * 1e3 if t else float("nan")  # MB / us -> GB/s
        h, m = avg(c.get("TCC_HIT_sum", [])), avg(c.get("TCC_MISS_sum", []))
        hit = 100 * h / (h + m) if (h + m) else float("nan")
        print(f"| `{k}` | {n} | {t:.1f} | {mfma:.1f}% | {valu:.0f} | {mf:.0f} | {lds:.0f} | {conf:.2f} | {fe:.1f} | {wr:.1f} | "
              f"{bw:.0f} | {hit:.1f}% |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25, int(sys.argv[3]) if len(sys.argv) > 3 else 256,
         sys.argv[4] if len(sys.argv) > 4 else None)
