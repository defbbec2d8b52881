#!/bin/bash
# LDS-array utilisation of the hand-written GEMMs (is the main loop LDS-bound?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out/pmc_lds
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/pmc_lds/avail.txt 2>&1 || true
P="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
GW_SPLITS=8 timeout -s KILL 60 rocprofv3 --pmc $P -d $R/gpurun_out/pmc_lds/wg -o run --output-format csv -- $R/tools/cpp/gemm_bench wgrad 32768 6144 768 > $R/gpurun_out/pmc_lds/wg.log 2>&1 || { tail -5 $R/gpurun_out/pmc_lds/wg.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc $P -d $R/gpurun_out/pmc_lds/fw -o run --output-format csv -- $R/tools/cpp/gemm_bench bf16,nostore 16384 6144 768 > $R/gpurun_out/pmc_lds/fw.log 2>&1 || { tail -5 $R/gpurun_out/pmc_lds/fw.log; exit 1; }
cd $R
python - <<'PY'
import csv, glob, collections
for tag in ("wg", "fw"):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/pmc_lds/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in per.items():
        a = {n: sum(v) / len(v) for n, v in c.items()}
        g = a.get("GRBM_GUI_ACTIVE", float("nan"))
        print(tag, k, " ".join(f"{n}={v:.3g}" for n, v in sorted(a.items())))
PY
