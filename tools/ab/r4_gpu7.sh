# round 4: nf-slot race fix -> convergence (3 seeds, engine vs eager), ffbb tests, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "ffbb or pipelined_window or reproducible" > gpurun_out/r4_t7.log 2>&1 || { tail -60 gpurun_out/r4_t7.log; exit 1; }
tail -1 gpurun_out/r4_t7.log
for v in all only_head; do
  DLT_GEMM_PLAN=gpurun_plans/$v.json timeout -k 10 300 python -u tools/converge.py --steps 21 --log 10 > gpurun_out/bis3_$v.log 2>&1 || { tail -20 gpurun_out/bis3_$v.log; exit 1; }
  echo "$v $(grep '"step": 20' gpurun_out/bis3_$v.log)"
done
for seed in 1234 1 2; do
  timeout -k 10 300 python -u tools/converge.py --steps 150 --seed $seed > gpurun_out/conv_engine_$seed.log 2>&1 || { tail -20 gpurun_out/conv_engine_$seed.log; exit 1; }
  tail -1 gpurun_out/conv_engine_$seed.log
done
