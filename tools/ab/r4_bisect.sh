# round 4: which change slowed convergence? 30-step engine runs with single knobs off
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in "base:" "nodgrad:DLT_GEMM_DGRAD=0" "flags0:DLT_GEMM_FLAGS=0" "noring:DLT_SLOT_RING=0" "nopipe:DLT_PIPELINE=0" "fb:DLT_WINDOW_SCHED=fb"; do
  name=${v%%:*}; kv=${v#*:}
  env $kv timeout -k 10 300 python -u tools/converge.py --steps 21 --log 10 > gpurun_out/bis_$name.log 2>&1 || { tail -20 gpurun_out/bis_$name.log; exit 1; }
  echo "$name $(grep '"step": 20' gpurun_out/bis_$name.log)"
done
