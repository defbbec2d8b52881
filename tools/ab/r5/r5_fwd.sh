# round 5: forward projection GEMMs on the hand kernel in the step -- persistent vs one tile per
# workgroup vs the library plan, ffbb and fb windows; then a kernel trace of the hand plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
H=tools/ab/r5/plan_r5_fwdhand.json
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/f5_$n.log 2> gpurun_out/f5_$n.err || { tail -20 gpurun_out/f5_$n.err; exit 1; }; python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" gpurun_out/f5_$n.log $n; }
for rep in 1 2; do
  run lib.$rep DLT_X=0 &&
  run hand.$rep DLT_GEMM_PLAN=$H &&
  run hand1t.$rep DLT_GEMM_PLAN=$H DLT_GEMM_FWD_FLAGS=256 &&
  run handnocap.$rep DLT_GEMM_PLAN=$H DLT_FFBB_GEMM_GRID=0 &&
  run libfb.$rep DLT_WINDOW_SCHED=fb &&
  run handfb.$rep DLT_GEMM_PLAN=$H DLT_WINDOW_SCHED=fb || exit 1
done
R0=$PWD
cd /tmp && export TMPDIR=/tmp
for v in lib hand1t; do
  if [ $v = lib ]; then E="DLT_X=0"; else E="DLT_GEMM_PLAN=$R0/$H DLT_GEMM_FWD_FLAGS=256"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace -d "$R0/gpurun_out/prof_f5_$v" -o run --output-format csv \
    -- python3 "$R0/bench.py" --steps 3 --warmup 2 > "$R0/gpurun_out/prof_f5_$v.log" 2>&1 || { tail -20 "$R0/gpurun_out/prof_f5_$v.log"; exit 1; }
done
cd "$R0"
for v in lib hand1t; do
  f=$(find gpurun_out/prof_f5_$v -name '*kernel_trace.csv' | head -1)
  python tools/step_profile.py "$f" > gpurun_out/step_f5_$v.md && python tools/concurrency.py "$f" 30 >> gpurun_out/step_f5_$v.md && head -12 gpurun_out/step_f5_$v.md
done
