"""Reference-path shim for ``models.gpt`` (``src/models/gpt.py``)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_llm_trainer_amd.models.gpt import (  # noqa: E402,F401
    GPT, MLP, CausalSelfAttention, RMSNorm, RotaryPositionEmbedding, TransformerBlock, apply_rotary_pos_emb,
    count_parameters, rotate_half)

if __name__ == "__main__":
    import torch
    from distributed_llm_trainer_amd.models.config import GPTConfig
    config = GPTConfig.gpt2_small()
    model = GPT(config)
    print(f"Model config: {config}")
    print(f"Estimated parameters (reference formula): {config.num_parameters_legacy():,}")
    print(f"Actual parameters: {count_parameters(model):,}")
    ids = torch.randint(0, config.vocab_size, (2, 128))
    logits, loss = model(ids, labels=ids)
    print(f"Logits shape: {logits.shape}")
    print(f"Loss: {loss.item():.4f}")
