"""The counter-based dropout RNG contract (ops/rng.py)."""
import torch

from distributed_llm_trainer_amd.ops import rng


def test_lowbias32_vectorised_matches_scalar():
    xs = [0, 1, 2, 12345, 0xFFFFFFFF, 0x80000000]
    t = rng.lowbias32_t(torch.tensor(xs, dtype=torch.int64))
    assert t.tolist() == [rng.lowbias32(x) for x in xs]


def test_keep_rate_and_independence():
    key = rng.site_key(1, 2, 3, rng.SITE_RESID)
    m = rng.keep_mask((1000, 1000), key, 0.1)
    rate = 1 - m.float().mean().item()
    assert abs(rate - 0.1) < 0.002
    m2 = rng.keep_mask((1000, 1000), rng.site_key(1, 3, 3, rng.SITE_RESID), 0.1)
    both = (~m & ~m2).float().mean().item()
    assert abs(both - 0.01) < 0.002  # different steps -> independent masks
    assert rng.keep_mask((10,), key, 0.0).all()


def test_attention_mask_rate():
    m = rng.attn_keep_mask(4, 128, 128, rng.site_key(7, 0, 0, rng.SITE_ATTN), 0.1)
    assert abs((1 - m.float().mean().item()) - 0.1) < 0.01
