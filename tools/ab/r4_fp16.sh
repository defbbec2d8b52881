# round 4: --precision fp16 (HIP kernels for IEEE half): bench + kernel trace of the step (which kernels are at::native)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --precision fp16 > gpurun_out/f16_bench.log 2> gpurun_out/f16_bench.err || { tail -20 gpurun_out/f16_bench.err; exit 1; }
tail -1 gpurun_out/f16_bench.log
bash tools/ab/prof_step.sh f16 --precision fp16 > gpurun_out/step_f16_full.md 2>&1 || { tail -20 gpurun_out/step_f16_full.md; exit 1; }
head -40 gpurun_out/step_f16_full.md
f=$(find gpurun_out/prof_f16 -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
from collections import Counter
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
opt = [i for i, r in enumerate(rows) if "k_sumsq" in r["Kernel_Name"]]
step = rows[opt[-2] + 1:opt[-1] + 1]
c, t = Counter(), Counter()
for r in step:
    n = r["Kernel_Name"]
    if "at::native" in n or "rocprim" in n:
        k = n.split("(")[0][:150]
        c[k] += 1
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("at::native / rocprim kernels in the last fp16 step:", sum(c.values()), "launches,", round(sum(t.values()), 1), "us")
for k, v in t.most_common(20):
    print(f"{v:9.1f} us {c[k]:4d}  {k}")
PY
