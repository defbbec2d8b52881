DLT_GEMM_TUNE=exhaustive DLT_GEMM_VERBOSE=1 DLT_GEMM_PLAN=none timeout -k 10 300 python - <<'PY'
import torch, sys
sys.path.insert(0, '.')
from distributed_llm_trainer_amd.ops import gemm
g = gemm.HipGemm(); g._race = False
x = torch.randn(16384, 768, device='cuda').bfloat16(); w = torch.randn(2304, 768, device='cuda').bfloat16()
y = g.linear(x, w); torch.cuda.synchronize()
PY
