# FSDP trainer on one GPU: medium (AC on, reference default) and xl, throughput + peak memory.
set -o pipefail
timeout -k 10 400 python bench.py --mode fsdp --model_size medium --batch_size 4 --grad_accum 8 --steps 3 --warmup 1 2>&1 | grep metric
timeout -k 10 400 python bench.py --mode fsdp --model_size medium --batch_size 4 --grad_accum 8 --steps 3 --warmup 1 --no_ac 2>&1 | grep metric
timeout -k 10 600 python bench.py --mode fsdp --model_size xl --batch_size 4 --grad_accum 8 --steps 2 --warmup 1 2>&1 | grep metric
