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


def _grid_worker(rank, world, port, q):
    """One rank of a sharded CV grid with the product's host plan (grid.plan_fits /
    rank_share / merge_results / assemble); each rank's per-fit solves come from the float64
    oracle, in the exact per-fit result format grid.run_multi gathers."""
    import sys
    import torch.distributed as dist
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    from oracle import glm_ref
    from sglm_hip import engine as E, grid, synth
    from sglm_hip.estimators import Objective
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = synth.make(N=1500, m=3, L=3, family="poisson", rho=0.1, seed=5, beta_scale=0.3)
    X, y = s.dense_X(), s.y
    rng = np.random.default_rng(1)
    cv_idx = []
    for _ in range(3):
        perm = rng.permutation(s.N)
        cv_idx.append((np.sort(perm[300:]), np.sort(perm[:300])))
    alphas = [0.01, 0.1, 1.0]
    groups = [{"cv_idx": cv_idx, "rolls": [0, 0, 0],
               "objectives": [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, a, "n", True, 100)
                              for a in alphas]}]
    plan = grid.plan_fits(groups, s.N)
    specs, gm, counts, table, roll_list = plan
    mine = grid.rank_share(plan, groups, rank, world)
    local = {}
    for i in mine:
        _, j, k, m, r, mt = table[i]
        rows = np.arange(s.N) if k < 0 else cv_idx[k][0]
        c, b = glm_ref.fit_tweedie_newton(X[rows], y[rows], alphas[j], 1.0)
        sc = {}
        if k >= 0:
            te = cv_idx[k][1]
            mu_tr = np.exp(X[rows] @ c + b)
            mu_te = np.exp(X[te] @ c + b)
            sc = {"train": -np.mean((y[rows] - mu_tr) ** 2), "test": -np.mean((y[te] - mu_te) ** 2),
                  "ss_res": float(np.sum((y[te] - mu_te) ** 2)),
                  "sst": float(np.sum((y[te] - y[te].mean()) ** 2)), "cnt_te": float(te.size)}
        local[i] = (c, b, 1, True, sc)
    merged = grid.merge_results(local, dist)
    out = grid.assemble(groups, plan, merged, s.p)[0]
    q.put((rank, sorted(mine), sorted(merged), out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_grid_plan_gather_assemble(world):
    """shard_plan over real fit tables, merge_results over gloo, assemble into the
    reference's per-param dicts: every rank ends with the same dicts, equal to the oracle's
    unsharded cv_glm_mult_params (backend/sglm_cv.py:42-206)."""
    import sys
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    from oracle import cv_ref
    from sglm_hip import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shares = [m for _, m, _, _ in outs]
    assert sorted(i for m in shares for i in m) == list(range(12))
    assert all(len(m) > 0 for m in shares)
    s = synth.make(N=1500, m=3, L=3, family="poisson", rho=0.1, seed=5, beta_scale=0.3)
    X, y = s.dense_X(), s.y
    rng = np.random.default_rng(1)
    cv_idx = []
    for _ in range(3):
        perm = rng.permutation(s.N)
        cv_idx.append((np.sort(perm[300:]), np.sort(perm[:300])))
    ref = cv_ref.cv_mult(X, y, cv_idx, [{"model_name": "Poisson", "alpha": a}
                                        for a in (0.01, 0.1, 1.0)])["full_cv_results"]
    for _, _, keys, out in outs:
        assert keys == list(range(12))
        for d, r in zip(out, ref):
            np.testing.assert_allclose(d["cv_coefs"], r["cv_coefs"], rtol=0, atol=1e-10)
            np.testing.assert_allclose(d["refit_coef"], r["coef"], rtol=0, atol=1e-10)
            np.testing.assert_allclose(d["cv_scores_test"], r["cv_scores_test"], rtol=1e-12)
            assert abs(d["cv_R2_score"] - r["cv_R2_score"]) < 1e-12
            assert abs(d["cv_mse_score"] - r["cv_mse_score"]) < 1e-12 * r["cv_mse_score"]


def _rowcomm_worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    from sglm_hip.comm import RowComm, row_slab
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = RowComm(dist)
    # slab partials of a Gram-like sum, a maximum and a minimum over rows
    n = 1000
    s0, s1 = row_slab(n, rank, world)
    rows = torch.arange(s0, s1, dtype=torch.float64)
    g = torch.stack([rows.sum(), (rows ** 2).sum()])
    c.sum_(g)
    mx = torch.tensor([rows.max().item()], dtype=torch.float32)
    c.max_(mx)
    mn = torch.tensor([rows.min().item()], dtype=torch.float64)
    c.min_(mn)
    # round-robin factorisation owners, then directions combined by one sum
    own = c.owners(7, 3)
    delta = torch.zeros((7, 4), dtype=torch.float32)
    for k in range(7):
        if own[k] == rank:
            delta[k] = float(k + 1)
    c.directions_(delta)
    q.put((rank, g.tolist(), float(mx), float(mn), own.tolist(), delta[:, 0].tolist(),
           c.calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_collectives(world):
    """comm.RowComm over a gloo group: slab sums / maxima / minima equal the whole-row values
    on every rank, the factorisation owners agree and cover every rank, and the directions
    each owner solved reach every rank (the others add zeros) -- the collectives of the
    row-sharded grid (engine.irls with comm=RowComm)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rowcomm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 1000
    for rank, g, mx, mn, own, d0, calls in out:
        assert g == [float(sum(range(n))), float(sum(i * i for i in range(n)))]
        assert mx == n - 1 and mn == 0
        assert own == [(k + 3) % world for k in range(7)]
        assert d0 == [float(k + 1) for k in range(7)]
        assert calls == 4
