# round 5 batch 11: wait / LDS-utilisation counters of the forward GEMMs (lib, persistent
# hand kernel, four-wave tn4 BK 64) -- one rocprofv3 --pmc pass, 8 SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pmc_e11
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM"
DLT_TN4_BK=64 timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmc_e11/p1 -o run --output-format csv -- python3 tools/bench_gemm_fwd.py --iters 5 \
  > gpurun_out/pmc_e11/p1.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc_e11/p1.log; exit 1; }
python - <<'PY'
import csv, glob, re
from collections import defaultdict
per = defaultdict(lambda: defaultdict(list))
for f in glob.glob("gpurun_out/pmc_e11/p1/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:50]
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in per.items():
    if "gemm" not in k and "Cijk" not in k:
        continue
    a = {n: sum(v) / len(v) for n, v in c.items()}
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(f"{k:50s} wait_any {a['SQ_WAIT_ANY']/wc:.2f} wait_inst_any {a['SQ_WAIT_INST_ANY']/wc:.2f} "
          f"wait_inst_lds {a['SQ_WAIT_INST_LDS']/wc:.2f} lds_active/busy_cu {a['SQ_LDS_IDX_ACTIVE']/max(a['SQ_BUSY_CU_CYCLES'],1):.2f} "
          f"active_lds/wave {a['SQ_ACTIVE_INST_LDS']/wc:.2f} vmem_level/wave {a['SQ_INST_LEVEL_VMEM']/wc:.2f}")
PY
