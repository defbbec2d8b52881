# round 4: attention keep-bit masks regenerated in the backward (DLT_ATTN_MASK_BUDGET_GB=0) vs kept; serial profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/m_$n.log 2> gpurun_out/m_$n.err || { tail -20 gpurun_out/m_$n.err; exit 1; }; }
for rep in 1 2; do
  run keep.$rep DLT_X=0 && run regen.$rep DLT_ATTN_MASK_BUDGET_GB=0 || exit 1
done
for f in gpurun_out/m_*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
bash tools/ab/r4_serial.sh && bash tools/ab/r4_coll.sh
