# round 5 batch 10: four-wave forward GEMM, k-step-pipelined, BK 32 (ring of 4) vs 64 (ring
# of 2): numerics both depths, isolated timing, counters of lib / hand / tn4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/e10_avail.txt 2>&1 || echo "list-avail rc=$?"
for bk in 64 32; do
  DLT_TN4_BK=$bk timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_tn4" \
    > gpurun_out/e10_tests$bk.log 2>&1 || { tail -40 gpurun_out/e10_tests$bk.log; exit 1; }
  tail -1 gpurun_out/e10_tests$bk.log
  DLT_TN4_BK=$bk timeout -k 10 300 python -u tools/bench_gemm_fwd.py > gpurun_out/e10_iso$bk.log 2>&1 || { tail -20 gpurun_out/e10_iso$bk.log; exit 1; }
  echo "BK=$bk"; grep -v amdgpu.ids gpurun_out/e10_iso$bk.log | grep -v HW_QUEUES
done
bash tools/ab/pmc.sh e10 tools/bench_gemm_fwd.py --iters 5 && python tools/pmc_summary.py gpurun_out/pmc_e10 12
