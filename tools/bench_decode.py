"""Decode throughput of GPT.generate (KV cache) with and without the HIP-graph step.
usage: python tools/bench_decode.py [model_size] [batch] [new_tokens]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_trainer_amd.models import GPT, GPTConfig  # noqa: E402

size = sys.argv[1] if len(sys.argv) > 1 else "small"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
N = int(sys.argv[3]) if len(sys.argv) > 3 else 200
torch.manual_seed(0)
m = GPT(GPTConfig.from_preset(size)).to("cuda")
m.enable_engine()
ids = torch.randint(0, 50257, (B, 32), device="cuda")
for mode, graph, loop in (("eager", "0", "0"), ("graph, host sampling", "1", "0"), ("graph, device loop", "1", "1")):
    os.environ["DLT_DECODE_GRAPH"] = graph
    os.environ["DLT_DECODE_DEVICE_LOOP"] = loop
    m.generate(ids, max_new_tokens=8)
    torch.cuda.synchronize()
    t = time.perf_counter()
    m.generate(ids, max_new_tokens=N)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"{size} B={B} {mode}: {N / dt:.1f} steps/s, {B * N / dt:.1f} tokens/s ({dt / N * 1e3:.2f} ms/token)",
          flush=True)

# replay-only cost of the captured step (no sampling / Python in the loop)
from distributed_llm_trainer_amd.eval.decode import DecodeGraph, KVCache, forward_cached  # noqa: E402
with torch.no_grad():
    c = KVCache(m.config, B, "cuda", m.engine.act_dtype)
    forward_cached(m, ids, c)
    g = DecodeGraph(m, c, c.len)
    nxt = ids[:, -1:].clone()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        g.graph.replay()
    torch.cuda.synchronize()
    print(f"graph replay only: {(time.perf_counter() - t) / 100 * 1e3:.3f} ms/step")
    lg = g(nxt)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(100):
        v, _ = torch.topk(lg, 50)
        l2 = lg.masked_fill(lg < v[:, [-1]], float("-inf"))
        p = torch.softmax(l2, dim=-1)
        s = torch.multinomial(p, 1)
    torch.cuda.synchronize()
    print(f"sampling only: {(time.perf_counter() - t) / 100 * 1e3:.3f} ms/step")
