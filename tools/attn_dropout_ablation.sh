for p in 0.0 0.1; do timeout -k 10 120 python tools/bench_attn.py --p $p --iters 30 || exit 1; done
