mkdir -p gpurun_out/abl
run() { name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/abl/$name.log 2>&1 || { echo "$name failed"; return 1; }; echo "$name $(tail -1 gpurun_out/abl/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
run base python bench.py --steps 10 --warmup 3 && \
run nodrop python bench.py --steps 10 --warmup 3 --dropout 0 && \
run nowgstream env DLT_WGRAD_STREAM=0 python bench.py --steps 10 --warmup 3 && \
run maskstream env DLT_MASK_STREAM=1 python bench.py --steps 10 --warmup 3 && \
run base2 python bench.py --steps 10 --warmup 3
