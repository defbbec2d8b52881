# round 4: bench.py through torch.distributed.run (the driver's N > 1 launch form) with one rank
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29655 \
  bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/tr1.log 2> gpurun_out/tr1.err || { tail -30 gpurun_out/tr1.err; exit 1; }
tail -1 gpurun_out/tr1.log | cut -c1-300
