"""Multi-rank fit sharding + result gather on CPU (gloo, world size 2)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    from sglm_hip import grid
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total = 23
    mine = grid.shard_indices(total, rank, world)
    local = {i: (np.full(3, float(i)), float(i) * 2, rank) for i in mine}
    merged = grid.merge_results(local, dist)
    q.put((rank, sorted(merged), {i: merged[i][2] for i in merged},
           all(np.all(merged[i][0] == i) and merged[i][1] == 2 * i for i in merged)))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_and_gather_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, keys, owner, ok in out:
        assert keys == list(range(23))
        assert ok
        assert all(owner[i] == i % 2 for i in keys)


def test_shard_indices_cover_exactly_once():
    from sglm_hip import grid
    for world in (1, 2, 3, 8):
        allidx = sorted(i for r in range(world) for i in grid.shard_indices(120, r, world))
        assert allidx == list(range(120))
