"""Hand data-gradient GEMM at the step's shapes: capped (ffbb: 192 workgroups) vs full
persistent grid, bitwise; and on two concurrent streams."""
import sys
import torch
sys.path.insert(0, '.')
from distributed_llm_trainer_amd.ops import hip
torch.manual_seed(0)
for (M, Nout, Nred) in [(16384, 768, 2304), (16384, 768, 6144), (16384, 768, 50304), (16384, 3072, 768)]:
    dy = ((torch.rand(M, Nred, device='cuda') * 2 - 1) * 1e-3).bfloat16()
    w = ((torch.rand(Nred, Nout, device='cuda') * 2 - 1) / Nred ** 0.5).bfloat16()
    hip.gemm_grid_cap(0)
    a = hip.gemm_dgrad(dy, w)
    res = []
    for cap in (192, 128, 64):
        hip.gemm_grid_cap(cap)
        b = hip.gemm_dgrad(dy, w)
        torch.cuda.synchronize()
        res.append((cap, torch.equal(a, b), (a.float() - b.float()).abs().max().item()))
    hip.gemm_grid_cap(0)
    # two streams concurrently (same inputs)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream()); s2.wait_stream(torch.cuda.current_stream())
    hip.gemm_grid_cap(192)
    with torch.cuda.stream(s1):
        c1 = hip.gemm_dgrad(dy, w)
    with torch.cuda.stream(s2):
        c2 = hip.gemm_dgrad(dy, w)
    hip.gemm_grid_cap(0)
    torch.cuda.synchronize()
    print(M, Nout, Nred, res, 'concurrent', torch.equal(a, c1), torch.equal(a, c2), flush=True)
