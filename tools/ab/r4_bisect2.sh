set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in none all only_qkv only_o only_gu only_down only_head; do
  DLT_GEMM_PLAN=gpurun_plans/$v.json timeout -k 10 300 python -u tools/converge.py --steps 21 --log 10 > gpurun_out/bis2_$v.log 2>&1 || { tail -20 gpurun_out/bis2_$v.log; exit 1; }
  echo "$v $(grep '"step": 20' gpurun_out/bis2_$v.log)"
done
