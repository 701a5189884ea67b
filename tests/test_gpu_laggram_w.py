"""The weighted Gram of a time-shifted 0/1 event design from its events (sglm_lag_gram_w,
csrc/lagw.hip) against the dense bit-plane Gram (sglm_syrk_cbits) of the same design: bitwise
equal with integer weights (exact f32 sums below 2^24 -- the Gaussian path's mask Grams), and
within f32 summation-order noise with bf16-rounded IRLS weights; shift-major and event-major
columns, a row window (row0 > 0), one and two 32-event halves, both launch shapes (<= 64 and
> 64 fit-shift columns), and fits on masked rows (weights 0 there); an irregular shift set
takes the dense path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_mod(engine):
    import torch
    return torch


def _events(rng, N, m, rho):
    E = (rng.random((N, m)) < rho).astype(np.float32)
    E[:, 0] = 0
    E[rng.integers(0, N, 5), 0] = 1                   # a sparse event
    return E


def _dense(engine, torch, d, W, fits):
    """H via the row-compacted bit-plane Gram over every row (weights carry the masks)."""
    from sglm_hip import _lib
    prob = engine.Problem(d, [np.zeros(d.n)], [np.ones(d.n, np.uint8)])
    bits, nr, rows = prob.compact(0)
    B = len(fits)
    stride = max(64, (nr + 63) // 64 * 64)
    wc = torch.zeros(B * stride, dtype=torch.bfloat16, device="cuda")
    desc = torch.tensor([[bits.data_ptr(), nr, wc.data_ptr() + 2 * k * stride, 0]
                         for k in range(B)], dtype=torch.int64).cuda()
    fits_d = torch.tensor(fits, dtype=torch.int32, device="cuda")
    _lib.call("sglm_gather_w", W.data_ptr(), d.ld, fits_d.data_ptr(), B, desc.data_ptr(), nr, 0)
    H = torch.zeros((int(max(fits)) + 1, d.P, d.P), dtype=torch.float32, device="cuda")
    _lib.call("sglm_syrk_cbits", desc.data_ptr(), d.P, fits_d.data_ptr(), B, 1, H.data_ptr(),
              0, 0)
    return H


def _lag(engine, torch, d, W, fits):
    from sglm_hip import _lib
    lg = engine._lagw(d)
    assert lg is not None
    fits_d = torch.tensor(fits, dtype=torch.int32, device="cuda")
    H = torch.full((int(max(fits)) + 1, d.P, d.P), float("nan"), dtype=torch.float32,
                   device="cuda")
    wk = torch.empty(_lib.query("sglm_lag_gram_w_work_bytes", lg.n_raw, lg.K, len(fits), d.P),
                     dtype=torch.uint8, device="cuda")
    _lib.call("sglm_lag_gram_w", lg.R.data_ptr(), lg.occ.data_ptr(), lg.ev_off.data_ptr(), lg.m,
              lg.n_raw, lg.shifts.data_ptr(), lg.bidx.data_ptr(), lg.K, lg.smin, lg.smax,
              lg.layout, lg.row0, lg.n, W.data_ptr(), d.ld, fits_d.data_ptr(), len(fits),
              H.data_ptr(), d.P, d.p, wk.data_ptr(), 0)
    return H


@pytest.mark.parametrize("m,shifts,row0,event_major,nf", [
    (13, list(range(-5, 5)), 5, False, 3),              # one half, shift-major, NT = 2
    (40, list(range(0, 12)), 11, True, 2),              # two halves, event-major
    (20, list(range(3, -4, -1)), 7, False, 14),         # descending shifts, two column groups
    (50, list(range(-20, 20)), 20, False, 5),           # the C4 layout, 200 columns
    (30, list(range(-8, 8)), 8, False, 17),             # 272 columns: three column blocks
    (45, list(range(5, -5, -1)), 9, True, 1),           # event-major, descending, one fit
])
def test_lag_gram_w_matches_dense(engine, torch_mod, m, shifts, row0, event_major, nf):
    torch = torch_mod
    rng = np.random.default_rng(m + nf)
    N = 6000
    E = _events(rng, N, m, 0.03)
    n = N - row0 - max(0, max(shifts))
    d = engine.Design.from_events(E, shifts, row0, n, event_major=event_major)
    assert d.lag is not None and d.p == m * len(shifts)
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))
    fits = [2 * k + 1 for k in range(nf)]                # non-contiguous slots
    nslot = max(fits) + 1
    # integer weights (mask multiplicities): exact sums, bitwise equal
    Wi = torch.zeros((nslot, d.ld), dtype=torch.float32, device="cuda")
    for k in fits:
        Wi[k, :n] = torch.from_numpy((rng.random(n) < 0.8).astype(np.float32)
                                     * rng.integers(1, 3, n).astype(np.float32))
    Hd, Hl = _dense(engine, torch, d, Wi, fits), _lag(engine, torch, d, Wi, fits)
    for k in fits:
        a, b = Hd[k].cpu().numpy()[blk], Hl[k].cpu().numpy()[blk]
        assert np.array_equal(a, b), (k, np.flatnonzero(a != b)[:5])
    # IRLS-like weights on masked rows (bf16-rounded in both): summation-order noise only
    Wf = torch.zeros((nslot, d.ld), dtype=torch.float32, device="cuda")
    for k in fits:
        Wf[k, :n] = torch.from_numpy(((rng.random(n) < 0.7) * np.exp(rng.normal(0, 1, n)))
                                     .astype(np.float32))
    Hd, Hl = _dense(engine, torch, d, Wf, fits), _lag(engine, torch, d, Wf, fits)
    for k in fits:
        a, b = Hd[k].cpu().numpy()[blk], Hl[k].cpu().numpy()[blk]
        assert np.all(np.isfinite(b))
        assert np.max(np.abs(a - b)) <= 2e-6 * max(1.0, float(np.max(np.abs(a)))), k


@pytest.mark.parametrize("split", ["0", "1"])
def test_lag_gram_w_split_pieces(engine, torch_mod, monkeypatch, split):
    """With and without the load-balancing split (the heaviest pieces run as two
    half-occurrence jobs whose second halves the symmetrize pass adds): integer weights bitwise
    the dense Gram, IRLS-like weights within f32 summation noise; the C4 layout (two event
    halves) at 5 fits and one fit."""
    torch = torch_mod
    monkeypatch.setenv("SGLM_LAGW_SPLIT", split)
    rng = np.random.default_rng(21)
    N, m, shifts, row0 = 20000, 50, list(range(-20, 20)), 20
    E = _events(rng, N, m, 0.02)
    n = N - row0 - 19
    d = engine.Design.from_events(E, shifts, row0, n)
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))
    for nf in (5, 1):
        fits = list(range(nf))
        Wi = torch.zeros((nf, d.ld), dtype=torch.float32, device="cuda")
        Wf = torch.zeros((nf, d.ld), dtype=torch.float32, device="cuda")
        for k in fits:
            Wi[k, :n] = torch.from_numpy(rng.integers(0, 3, n).astype(np.float32))
            Wf[k, :n] = torch.from_numpy(np.exp(rng.normal(0, 1, n)).astype(np.float32))
        Hd, Hl = _dense(engine, torch, d, Wi, fits), _lag(engine, torch, d, Wi, fits)
        for k in fits:
            a, b = Hd[k].cpu().numpy()[blk], Hl[k].cpu().numpy()[blk]
            assert np.array_equal(a, b), (nf, k, np.flatnonzero(a != b)[:5])
        Hd, Hl = _dense(engine, torch, d, Wf, fits), _lag(engine, torch, d, Wf, fits)
        for k in fits:
            a, b = Hd[k].cpu().numpy()[blk], Hl[k].cpu().numpy()[blk]
            assert np.max(np.abs(a - b)) <= 2e-6 * float(np.max(np.abs(a))), (nf, k)


def test_lag_gram_w_cost_model(engine, torch_mod):
    """The structured Gram is chosen for the C4 shape (2000 lag columns, 2 % events) and not
    for a small design whose dense Gram costs microseconds."""
    from sglm_hip import synth
    s = synth.make(N=200_000, m=50, L=40, family="poisson", rho=0.02, seed=0)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    lg = engine._lagw(d)
    assert lg is not None and engine._lagw_pays(d, lg, 5)
    s2 = synth.make(N=20_000, m=6, L=5, family="poisson", rho=0.05, seed=1)
    d2 = engine.Design.from_events(s2.E, s2.shifts, s2.L - 1, s2.N)
    lg2 = engine._lagw(d2)
    assert lg2 is not None and not engine._lagw_pays(d2, lg2, 5)


def test_lag_gram_w_irregular_shifts_fall_back(engine, torch_mod):
    rng = np.random.default_rng(3)
    E = _events(rng, 3000, 9, 0.05)
    d = engine.Design.from_events(E, [-7, -2, 0, 1, 6], 7, 2980)
    assert d.lag is not None and engine._lagw(d) is None


def test_lag_gram_w_in_grid_matches_dense_path(engine, torch_mod, monkeypatch):
    """A Poisson CV grid solved with the structured Gram equals the dense-Gram grid (the same
    fixed point; Hessians differ by f32 summation order only)."""
    from sglm_hip import grid, synth, folds
    from sglm_hip.estimators import Objective
    import pandas as pd
    s = synth.make(N=30000, m=12, L=8, family="poisson", rho=0.03, seed=5)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(1)
    cv = folds.cv_idx_from_bucket_ids(codes, num_folds=3)
    objs = [Objective("irls", engine.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in (1e-3, 1e-2, 1e-1)]
    out = {}
    monkeypatch.setattr(engine, "_lagw_pays", lambda d, lg, nact: True)   # small: force it
    for flag in (True, False):
        monkeypatch.setattr(engine, "LAG_GRAM_W", flag)
        out[flag] = grid.run(d, s.y, cv, objs, [0] * len(objs))
    for a, b in zip(out[True], out[False]):
        assert np.allclose(a["refit_coef"], b["refit_coef"], rtol=1e-4, atol=1e-6)
        assert np.allclose(a["cv_coefs"], b["cv_coefs"], rtol=1e-4, atol=1e-6)
        assert abs(a["cv_mean_score"] - b["cv_mean_score"]) <= 1e-6 * max(1, abs(b["cv_mean_score"]))


def test_lag_gram_w_scratch_budget_chunks_fits(engine, torch_mod, monkeypatch):
    """The launch's scratch (8 bf16 weight copies and a split-half image per fit) is bounded:
    with a budget of two fits the seven fits run as four launches and give bitwise the same
    Hessians (integer weights: exact sums, whichever pieces each launch shape splits)."""
    from types import SimpleNamespace
    torch = torch_mod
    rng = np.random.default_rng(7)
    E = _events(rng, 5000, 20, 0.04)
    d = engine.Design.from_events(E, list(range(-6, 6)), 6, 4988)
    lg = engine._lagw(d)
    fits = np.array([0, 2, 3, 5, 6, 8, 9], dtype=np.int32)
    W = torch.randint(0, 4, (10, d.ld), device="cuda").float()
    out = []
    for budget in (float(1 << 40), 2.5 * engine._lib.query("sglm_lag_gram_w_work_bytes",
                                                             lg.n_raw, lg.K, 1, d.P)):
        monkeypatch.setattr(engine, "LAGW_WORK_BUDGET", budget)
        bf = SimpleNamespace(W=W, H=torch.zeros((10, d.P, d.P), device="cuda"))
        engine._lag_gram_w(d, lg, bf, fits, 0)
        torch.cuda.synchronize()
        out.append(bf.H.cpu().numpy())
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))
    for k in fits:
        assert np.array_equal(out[0][k][blk], out[1][k][blk]), k


def test_lag_gram_w_row_slab(engine, torch_mod):
    """A row slab of the design (one rank of a row-sharded solve, comm.py): the launch iterates
    only the occurrences whose lag window meets the slab's rows, and the slab's Gram is bitwise
    the dense bit-plane Gram of the same slab on integer weights."""
    from types import SimpleNamespace
    torch = torch_mod
    rng = np.random.default_rng(11)
    N, m, shifts, row0 = 9000, 24, list(range(-6, 6)), 6
    E = _events(rng, N, m, 0.03)
    n = N - row0 - 6
    d = engine.Design.from_events(E, shifts, row0, n, slab=(2000, 5000))
    lg = engine._lagw(d)
    assert lg is not None and d.n == 3000
    assert int(lg.w_occ.numel()) < int(lg.occ.numel())       # the other occurrences dropped
    fits = np.array([0, 2], dtype=np.int32)
    W = torch.zeros((3, d.ld), dtype=torch.float32, device="cuda")
    for k in fits:
        W[k, :d.n] = torch.from_numpy(rng.integers(0, 3, d.n).astype(np.float32))
    bf = SimpleNamespace(W=W, H=torch.full((3, d.P, d.P), float("nan"), device="cuda"))
    engine._lag_gram_w(d, lg, bf, fits, 0)
    Hd = _dense(engine, torch, d, W, list(fits))
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))
    for k in fits:
        a, b = Hd[k].cpu().numpy()[blk], bf.H[k].cpu().numpy()[blk]
        assert np.array_equal(a, b), (k, np.flatnonzero(a != b)[:5])
