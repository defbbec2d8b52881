set -o pipefail
timeout -k 10 200 python -u tools/bench_gemm_fwd.py --iters 30 --impls lib,fw4,fw4s1 > gpurun_out/fw4_3.log 2>&1 || exit 1
tail -5 gpurun_out/fw4_3.log
REPS=1 STEPS=8 bash tools/ab/r6/mem_ab.sh "first:--memory_first;f2np:--memory_first --fusion 2 --no_pipeline;f1np:--memory_first --no_pipeline" || exit 1
timeout -k 10 300 python -u tools/mem_breakdown.py --memory_first --top 30 > gpurun_out/memfirst_breakdown.txt 2>&1; echo mb rc=$?
