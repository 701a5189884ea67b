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


def test_shard_plan_mask_major_balanced():
    """C4's table (20 lambdas x (5 folds + refit)) over 1..8 ranks: every fit on exactly one
    rank, per-rank row cost balanced, each rank spanning at most one mask more than its share
    needs (round-robin gives every rank all 6), and each rank mixes weakly and strongly penalised fits."""
    from sglm_hip import grid
    nlam, K = 20, 5
    table = [(j, k) for j in range(nlam) for k in list(range(K)) + [K]]   # (lambda, mask)
    rows = [800_000] * K + [1_000_000]
    keys = [(k, 0, grid.snake(j, nlam), 0, j) for j, k in table]
    costs = [rows[k] for _, k in table]
    for world in (1, 2, 3, 4, 8):
        plan = [grid.shard_plan(keys, costs, r, world) for r in range(world)]
        assert sorted(i for p in plan for i in p) == list(range(len(table)))
        load = [sum(costs[i] for i in p) for p in plan]
        assert max(load) - min(load) <= 2 * max(rows)
        per_rank = -(-len(table) // world)
        assert max(len({table[i][1] for i in p}) for p in plan) <= -(-per_rank // nlam) + 1
        for p in plan:
            if len(p) >= 4:
                lams = [table[i][0] for i in p]
                assert min(lams) < nlam // 2 <= max(lams)
    assert [grid.snake(j, 5) for j in range(5)] == [0, 2, 4, 3, 1]
    assert sorted(grid.snake(j, 6) for j in range(6)) == list(range(6))
