# round 4: 150-step full-size convergence, engine vs eager autocast, 3 seeds each (variance band)
set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for seed in 1234 1 2; do
  timeout -k 10 300 python -u tools/converge.py --steps 150 --seed $seed > gpurun_out/conv_engine_$seed.log 2>&1 || { tail -20 gpurun_out/conv_engine_$seed.log; exit 1; }
  tail -1 gpurun_out/conv_engine_$seed.log
  timeout -k 10 300 python -u tools/converge.py --steps 150 --seed $seed --eager > gpurun_out/conv_eager_$seed.log 2>&1 || { tail -20 gpurun_out/conv_eager_$seed.log; exit 1; }
  tail -1 gpurun_out/conv_eager_$seed.log
done
