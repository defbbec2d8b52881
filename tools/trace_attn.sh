export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_trace -o t --output-format csv -- python3 tools/bench_attn.py --iters 5 > gpurun_out/attn_trace.log 2>&1
