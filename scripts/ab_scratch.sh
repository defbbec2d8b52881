set -u
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dgrad_swiglu" --timeout 120 --timeout-method thread 2>&1 | tail -1
python - <<'PY'
import torch, time, sys
sys.path.insert(0, '.')
from distributed_llm_trainer_amd.ops import hip, gemm
g = gemm.HipGemm()
M, H, I = 16384, 768, 3072
dd = torch.randn(M, H, device='cuda').bfloat16(); w = (torch.randn(H, I, device='cuda')/30).bfloat16()
gu = torch.randn(M, 2*I, device='cuda').bfloat16(); out = torch.empty(M, 2*I, device='cuda', dtype=torch.bfloat16)
wt = w.t().contiguous()
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/it*1e6
print("fused kernel       %.1f us" % bench(lambda: hip.dgrad_swiglu_bwd(dd, wt, gu, out=out)))
print("plain tn8          %.1f us" % bench(lambda: hip.gemm_tn(dd, wt, 5)))
print("unfused total      %.1f us" % bench(lambda: hip.swiglu_bwd(gu, g.linear_dgrad(dd, w), out=out)))
PY
