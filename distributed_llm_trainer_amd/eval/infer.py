"""Text generation from a checkpoint (CLI parity with ``src/eval/infer.py:34-70``).

Differences: checkpoints load with ``weights_only=True`` (config classes are
registered safe globals, including the reference's module paths -- no arbitrary
unpickling, and no placeholder-class hack needed); generation runs the KV-cached
decoder on the fused engine when a GPU is present; the tokenizer resolves offline
(``--tokenizer byte`` works without any downloaded files).
"""
from __future__ import annotations

import argparse

import torch

from ..data.tokenizer import get_tokenizer
from ..models.config import GPTConfig
from ..models.gpt import GPT
from ..utils.checkpoint import load_checkpoint, load_model_state


def pick_device(name: str) -> torch.device:
    if name != "auto":
        return torch.device(name)
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def load_model(path: str, model_size: str = None, device="cpu"):
    ckpt = load_checkpoint(path, map_location="cpu")
    cfg = ckpt.get("model_config")
    if model_size is not None or not isinstance(cfg, GPTConfig):
        cfg = GPTConfig.from_preset(model_size or "small")
    model = GPT(cfg)
    load_model_state(model, ckpt["model"])
    model = model.to(device)
    if torch.device(device).type == "cuda":
        model.enable_engine()
    model.eval()
    return model


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--checkpoint", required=True)
    p.add_argument("--model_size", default=None, choices=["small", "medium", "large", "xl"])
    p.add_argument("--prompt", default="Once upon a time,")
    p.add_argument("--max_new_tokens", type=int, default=50)
    p.add_argument("--device", default="auto")
    p.add_argument("--temperature", type=float, default=1.0)
    p.add_argument("--top_k", type=int, default=50)
    p.add_argument("--tokenizer", default="gpt2")
    p.add_argument("--seed", type=int, default=None)
    args = p.parse_args(argv)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    dev = pick_device(args.device)
    model = load_model(args.checkpoint, args.model_size, dev)
    tok = get_tokenizer(args.tokenizer)
    ids = torch.tensor([tok.encode(args.prompt)], dtype=torch.long, device=dev)
    out = model.generate(ids, max_new_tokens=args.max_new_tokens, temperature=args.temperature, top_k=args.top_k)
    text = tok.decode(out[0].tolist())
    print(text)
    return text


if __name__ == "__main__":
    main()
