"""Peak-memory breakdown of the training step (one GPU).

Records the caching allocator's history (torch.cuda.memory._record_memory_history) over a
few bench-config steps, replays the alloc / free trace to the moment of the peak, and
groups the blocks live at that moment by the innermost stack frame inside this package
(file:line function).  usage:
    python tools/mem_breakdown.py [bench.py args, e.g. --memory_lean --fusion 1] [--top 25]
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def site(frames):
    for f in frames:
        fn = f.get("filename", "")
        if "distributed_llm_trainer_amd" in fn and "/ops/" not in fn.split("distributed_llm_trainer_amd")[-1][:5]:
            return f"{fn.split('distributed_llm_trainer_amd/')[-1]}:{f.get('line')} {f.get('name')}"
    for f in frames:
        fn = f.get("filename", "")
        if "distributed_llm_trainer_amd" in fn:
            return f"{fn.split('distributed_llm_trainer_amd/')[-1]}:{f.get('line')} {f.get('name')}"
    return "(outside the package)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=25)
    args, rest = ap.parse_known_args()
    import bench
    torch.cuda.memory._record_memory_history(max_entries=2_000_000)
    sys.argv = ["bench.py", "--steps", "2", "--warmup", "2"] + rest
    bench.main()
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    live, cur, peak, at_peak = {}, 0, 0, {}
    for trace in snap["device_traces"]:
        for ev in trace:
            a, sz = ev["action"], ev["size"]
            if a == "alloc":
                live[ev["addr"]] = (sz, site(ev.get("frames", [])))
                cur += sz
                if cur > peak:
                    peak, at_peak = cur, dict(live)
            elif a in ("free_requested", "free_completed") and ev["addr"] in live and a == "free_completed":
                cur -= live.pop(ev["addr"])[0]
    groups = collections.defaultdict(lambda: [0, 0])
    for sz, where in at_peak.values():
        groups[where][0] += sz
        groups[where][1] += 1
    print(f"peak of the recorded window (live tensor bytes, allocator view): {peak / 1e9:.3f} GB; "
          f"max_allocated {torch.cuda.max_memory_allocated() / 1e9:.3f} GB")
    print(f"| site | GB | blocks |\n|---|---:|---:|")
    for where, (sz, n) in sorted(groups.items(), key=lambda kv: -kv[1][0])[:args.top]:
        print(f"| `{where}` | {sz / 1e9:.3f} | {n} |")


if __name__ == "__main__":
    main()
