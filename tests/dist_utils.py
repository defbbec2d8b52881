"""Helpers to run a function in N processes over gloo (127.0.0.1 rendezvous); CPU by
default, or all ranks sharing one GPU."""
import io
import os
import socket
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q, env):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world),
                       "DLT_BACKEND": "gloo", "DLT_FORCE_CPU": "1"})
    for k, v in (env or {}).items():  # None removes a variable
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        out = fn(rank, world, *args)
        buf = io.BytesIO()
        torch.save(out, buf)  # plain bytes: no fd-shared storages outliving the child
        q.put((rank, "ok", buf.getvalue()))
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def run_multiprocess(fn, world: int = 2, args=(), timeout: float = 300.0, env=None):
    """``env`` overrides the child environment (e.g. ``{"DLT_FORCE_CPU": None,
    "DLT_SHARE_GPU": "1"}`` runs every rank on the one GPU, still over gloo)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, status, out = q.get(timeout=timeout)
        if status != "ok":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {rank} failed:\n{out}")
        results[rank] = torch.load(io.BytesIO(out), weights_only=False)
    for p in procs:
        p.join(timeout=60)
    return [results[r] for r in range(world)]
