for i in 1 2; do
DLT_GEMM_TN=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 2>/dev/null | grep metric | cut -c1-110 || exit 1
DLT_GEMM_TN=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 2>/dev/null | grep metric | cut -c1-110 || exit 1
done
