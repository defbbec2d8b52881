# round 4: next-tile DMA hoist in k_gemm_bf16 (flags 4096 = old order): kernel tests,
# isolated timings (forward / dgrad), cycle stamps, in-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 200 --timeout-method thread \
  > gpurun_out/h_t.log 2>&1 || { tail -40 gpurun_out/h_t.log; exit 1; }
tail -1 gpurun_out/h_t.log
timeout -k 10 200 tools/cpp/gemm_bench xbsc1,xbsc1nh,blas 16384 6144 768 16384 2304 768 16384 768 3072 16384 768 768 16384 50304 768 \
  > gpurun_out/h_fwd.log 2>&1 || { cat gpurun_out/h_fwd.log; exit 1; }
cat gpurun_out/h_fwd.log
timeout -k 10 200 tools/cpp/gemm_bench dgrad 16384 768 2304 16384 768 768 16384 768 6144 16384 3072 768 16384 768 50304 \
  > gpurun_out/h_dg.log 2>&1 || { cat gpurun_out/h_dg.log; exit 1; }
cat gpurun_out/h_dg.log
timeout -k 10 120 tools/cpp/gemm_stamps 16384 6144 768 3084 7180 > gpurun_out/h_st.log 2>&1 &&
timeout -k 10 120 tools/cpp/gemm_stamps 16384 50304 768 3084 7180 >> gpurun_out/h_st.log 2>&1 || { cat gpurun_out/h_st.log; exit 1; }
cat gpurun_out/h_st.log
run() { n=$1; shift; timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 3 > gpurun_out/h_$n.log 2> gpurun_out/h_$n.err || { tail -20 gpurun_out/h_$n.err; exit 1; }; }
for rep in 1 2; do
  run hoist.$rep DLT_GEMM_FLAGS=3084 && run nohoist.$rep DLT_GEMM_FLAGS=7180 || exit 1
done
for f in gpurun_out/h_*hoist*.log; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['peak_gb_per_gpu'])" $f; done
