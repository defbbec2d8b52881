set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_roles.py 16384 2 > gpurun_out/gemm_roles_16k.log 2>&1; echo rc=$?; head -12 gpurun_out/gemm_roles_16k.log
M=16384 timeout -k 10 300 python -u tools/gemm_tn8_bench.py > gpurun_out/tn8_16k.log 2>&1; echo rc=$?; cat gpurun_out/tn8_16k.log
