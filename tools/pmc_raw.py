"""Per-kernel averages of raw rocprofv3 --pmc counters over every pass directory
(gpurun_out/<tag>/p*/run_counter_collection.csv): one row per (kernel, counter).
usage: python tools/pmc_raw.py gpurun_out/<tag> [name-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
pats = sys.argv[2:]
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    per = defaultdict(float)  # (dispatch, kernel, counter) summed over dimensions
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:70]
        per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (disp, k, c), v in per.items():
        vals[k][c].append(v)
for k in sorted(vals):
    if pats and not any(p in k for p in pats):
        continue
    print(k)
    for c in sorted(vals[k]):
        v = vals[k][c]
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
