"""world_size-2 gloo test of the multi-GPU record gather (the bench's only collective)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gpdemod_loader
    gpd = gpdemod_loader.load()
    from gpdemod import shard
    P = 8
    off = shard.weak_offset(P, rank)
    rec = np.zeros(P, dtype=gpd.PARAM_DTYPE)
    rec["b"] = off + np.arange(P)          # global series id encoded in b
    rec["nfev"] = rank
    local = torch.from_numpy(rec.view(np.uint8).reshape(P, 64).copy())
    out = shard.gather_records(local, world, rank)
    if rank == 0:
        got = shard.records_to_numpy(out, gpd.PARAM_DTYPE)
        q.put((got["b"].tolist(), got["nfev"].tolist()))
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_records_gloo_world2():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    b, nfev = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert b == list(range(16))
    assert nfev == [0] * 8 + [1] * 8
