import torch, sys
sys.path.insert(0, '.')
from distributed_llm_trainer_amd.ops import gemm
x = torch.randn(8192, 768, device='cuda').bfloat16(); w = torch.randn(6144, 768, device='cuda').bfloat16()
g = gemm.HipGemm(); g._race = False
y = g.linear(x, w); torch.cuda.synchronize()
print(gemm.report())
