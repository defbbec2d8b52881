"""wgrad (dW += dY^T X, fp32 accumulate) variants on the model's shapes."""
import time
import torch
M = 8192
shapes = [("qkv", 2304, 768), ("o", 768, 768), ("gu", 6144, 768), ("down", 768, 3072), ("lm", 50304, 768)]
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e6
for name, n, k in shapes:
    x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16); dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
    dw = torch.zeros(n, k, device="cuda")
    a = bench(lambda: torch.addmm(dw, dy.t(), x, out_dtype=torch.float32, out=dw))
    b = bench(lambda: dw.add_(torch.matmul(dy.t(), x)))
    c = bench(lambda: torch.matmul(dy.t(), x))
    xt = x.t().contiguous(); dyt = dy.t().contiguous()
    d = bench(lambda: torch.matmul(dyt, xt.t()))
    e = bench(lambda: torch.addmm(dw, dyt, xt.t(), out_dtype=torch.float32, out=dw))
    fl = 2 * M * n * k
    print(f"{name:5s} addmm_f32 {a:7.1f}  mm_bf16+add {b:7.1f}  mm_bf16 {c:7.1f}  mm(contig T) {d:7.1f} addmm(contigT) {e:7.1f} us | best {fl/min(a,b)/1e6:.0f} TF")
