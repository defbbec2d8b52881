# round 5: memory vs throughput of the two-chain ffbb window without (or with fewer)
# deferred weight gradients -- can the default reach <= 18 GB at unchanged tok/s?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
run() {  # name, env (comma list or -), bench args...
  local name=$1 kv=$2; shift 2
  [ "$kv" = "-" ] && kv=""
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 20 --warmup 3 "$@" \
    > gpurun_out/mf_$name.log 2> gpurun_out/mf_$name.err || { tail -20 gpurun_out/mf_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'], d.get('window'))" gpurun_out/mf_$name.log $name
}
for rep in 1 2; do
  run default - || exit 1
  run lean_ffbb DLT_WINDOW_SCHED=ffbb --memory_lean || exit 1
  run lean - --memory_lean || exit 1
  run dgh_ffbb DLT_WINDOW_SCHED=ffbb --defer_roles gu,down,head || exit 1
  run qo_ffbb DLT_WINDOW_SCHED=ffbb --defer_roles qkv,o,head || exit 1
done
