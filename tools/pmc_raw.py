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
        per[(r["Dispatch_Id"], k, "_duration_us")] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for (disp, k, c), v in per.items():
        vals[k][c].append(v)
for k in sorted(vals):
    if pats and not any(p in k for p in pats):
        continue
    print(k)
    g, d = vals[k].get("GRBM_GUI_ACTIVE"), vals[k].get("_duration_us")
    if g and d:  # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back)
        print(f"   {'effective clock GHz':28s} {sum(g) / len(g) / 8 / (sum(d) / len(d)) / 1e3:16.3f}")
    for c in sorted(vals[k]):
        v = vals[k][c]
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
