import torch, sys
sys.path.insert(0, '.')
from distributed_llm_trainer_amd.ops import hip, gemm
torch.manual_seed(0)
g = gemm.HipGemm()
for (M, Nout, Nred) in [(16384, 768, 2304), (16384, 768, 768), (16384, 768, 6144), (16384, 3072, 768), (16384, 768, 50304)]:
    dy = ((torch.rand(M, Nred, device='cuda') * 2 - 1) * (1e-3 if Nred == 50304 else 1)).bfloat16()
    w = ((torch.rand(Nred, Nout, device='cuda') * 2 - 1) / Nred ** 0.5).bfloat16()
    a = hip.gemm_dgrad(dy, w)
    b = torch.empty_like(a)
    g._lib_dgrad(dy, w, b)
    torch.cuda.synchronize()
    d = (a.float() - b.float())
    rel = (d.norm() / b.float().norm()).item()
    # per row-tile max relative error
    rt = d.abs().view(M // 256, 256, Nout).amax(dim=(1, 2)) / b.float().abs().max()
    print(M, Nout, Nred, 'rel', rel, 'worst tile rows', rt.argmax().item(), rt.max().item(), flush=True)
# dswiglu fused vs unfused
M, H, I = 16384, 768, 3072
dd = (torch.rand(M, H, device='cuda') * 2 - 1).bfloat16()
wd = ((torch.rand(H, I, device='cuda') * 2 - 1) / H ** 0.5).bfloat16()
gu = (torch.randn(M, 2 * I, device='cuda') * 2).bfloat16()
f = hip.gemm_down_swiglu_bwd(dd, wd, gu)
ds = torch.empty(M, I, dtype=torch.bfloat16, device='cuda'); g._lib_dgrad(dd, wd, ds)
u = hip.swiglu_bwd(gu, ds)
torch.cuda.synchronize()
print('dswiglu rel', ((f.float() - u.float()).norm() / u.float().norm()).item())
