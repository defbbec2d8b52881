#!/bin/bash
# A/B of the hand-written GEMM choices on one box (same process image, back to back),
# then a rocprofv3 kernel trace of the default configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$name.log 2> gpurun_out/ab_$name.err \
    || { tail -20 gpurun_out/ab_$name.err; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$name.log)"
}
# the round-2 library split-K picks, for the no-hand-wgrad arm
python - <<'PY'
import json
p = json.load(open("configs/gemm_plan_mi355x.json"))
p["splitk"] = {"32768x50304x768": 1, "32768x768x3072": 4, "32768x6144x768": 2, "32768x768x768": 16, "32768x2304x768": 4}
json.dump(p, open("gpurun_out/plan_libwgrad.json", "w"))
PY
run default X=1
run nohandwgrad DLT_GEMM_PLAN=gpurun_out/plan_libwgrad.json
run nohand DLT_GEMM_PLAN=gpurun_out/plan_libwgrad.json DLT_GEMM_TN=0 DLT_GEMM_FUSED=0
run default2 X=1
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r3" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r3.log" 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/prof_r3 -name '*kernel_trace.csv' | head -1)
  python tools/step_profile.py "$f" > gpurun_out/r3_step_breakdown.md && cat gpurun_out/r3_step_breakdown.md
fi
