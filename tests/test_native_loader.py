"""Native C++ token loader (runtime/csrc/loader.cpp): sharding, ordering, resume."""
import numpy as np
import pytest
import torch

from distributed_llm_trainer_amd.runtime import loader as nl

pytestmark = pytest.mark.skipif(not nl.available(), reason="native runtime not built")


def _file(tmp_path, n, dtype=np.uint16):
    p = tmp_path / f"tok_{np.dtype(dtype).name}.bin"
    np.arange(n, dtype=np.int64).astype(dtype).tofile(p)
    return str(p)


def test_windows_are_contiguous_and_ranks_disjoint(tmp_path):
    S, B, W = 16, 3, 2
    path = _file(tmp_path, 16 * 200 + 1)
    loaders = [nl.NativeTokenLoader(path, S, B, rank=r, world_size=W, seed=5) for r in range(W)]
    spe = loaders[0].steps_per_epoch
    assert loaders[0].num_windows == 200 and spe == 200 // W // B
    seen = []
    for L in loaders:
        for _ in range(spe):
            b = next(L)
            assert b.shape == (B, S) and b.dtype == torch.int64
            assert torch.all(b[:, 0] % S == 0) and torch.all(b[:, 1:] - b[:, :-1] == 1)
            seen += (b[:, 0] // S).tolist()
        L.close()
    assert len(seen) == len(set(seen)) == W * B * spe  # one epoch: every window at most once


def test_seeded_order_epochs_and_resume(tmp_path):
    path = _file(tmp_path, 8 * 64 + 1)
    a = nl.NativeTokenLoader(path, 8, 2, seed=1)
    stream = [next(a) for _ in range(3 * a.steps_per_epoch)]
    b = nl.NativeTokenLoader(path, 8, 2, seed=1, start_step=7)
    assert all(torch.equal(next(b), stream[7 + i]) for i in range(10))
    b.seek(2)
    assert torch.equal(next(b), stream[2])
    assert all(torch.equal(a.batch_at(i), stream[i]) for i in range(len(stream)))
    spe = a.steps_per_epoch
    e0 = torch.cat(stream[:spe])[:, 0].tolist()
    e1 = torch.cat(stream[spe:2 * spe])[:, 0].tolist()
    assert e0 != e1 and sorted(e0) == sorted(e1)  # reshuffled every epoch
    c = nl.NativeTokenLoader(path, 8, 2, seed=2)
    assert not torch.equal(next(c), stream[0])
    d = nl.NativeTokenLoader(path, 8, 2, seed=1, shuffle=False)
    assert next(d)[:, 0].tolist() == [0, 8]
    for L in (a, b, c, d):
        L.close()


@pytest.mark.parametrize("dtype,nbytes", [(np.uint16, 2), (np.uint32, 4), (np.int64, 8)])
def test_token_widths(tmp_path, dtype, nbytes):
    n = 70000 if nbytes > 2 else 60000
    p = tmp_path / "t.bin"
    (np.arange(n, dtype=np.int64) * 7 % 65000).astype(dtype).tofile(p)
    L = nl.NativeTokenLoader(str(p), 32, 4, token_bytes=nbytes, shuffle=False)
    b = next(L)
    assert b[0].tolist() == [(i * 7) % 65000 for i in range(32)]
    L.close()


def test_max_tokens_and_errors(tmp_path):
    path = _file(tmp_path, 1000)
    L = nl.NativeTokenLoader(path, 10, 1, max_tokens=101)
    assert L.num_windows == 10
    L.close()
    with pytest.raises(ValueError):
        nl.NativeTokenLoader(path, 10, 200)
    with pytest.raises(ValueError):
        nl.NativeTokenLoader(str(tmp_path / "missing.bin"), 10, 1)


def test_dummy_mode():
    a = nl.NativeTokenLoader(None, 64, 4, vocab_size=1000, seed=3, rank=0, world_size=2)
    b = nl.NativeTokenLoader(None, 64, 4, vocab_size=1000, seed=3, rank=1, world_size=2)
    a2 = nl.NativeTokenLoader(None, 64, 4, vocab_size=1000, seed=3, rank=0, world_size=2)
    xs = [next(a) for _ in range(20)]
    assert all(torch.equal(x, next(a2)) for x in xs)
    assert not torch.equal(xs[0], next(b))
    allv = torch.cat(xs)
    assert allv.min() >= 0 and allv.max() < 1000
    assert abs(allv.float().mean().item() - 499.5) < 15
    assert len(torch.unique(allv)) > 900
    for L in (a, b, a2):
        L.close()


def test_text_dataloader_uses_native_for_bin(tmp_path):
    from distributed_llm_trainer_amd.data import create_tinystories_dataloader
    path = _file(tmp_path, 4096)
    dl = create_tinystories_dataloader(path, batch_size=2, seq_len=32)
    assert isinstance(dl, nl.NativeTokenLoader)
    it = iter(dl)
    assert next(it).shape == (2, 32)
    dl.close()
