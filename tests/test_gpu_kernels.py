"""HIP kernels vs the float64 oracle / numpy on the same seeded inputs (MI355X only)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import glm_ref, pp_ref

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


@pytest.fixture(scope="module")
def torch_mod(engine):
    import torch
    return torch


def test_timeshift_bit_exact_all_widths(engine, torch_mod):
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(1)
    for dt in (np.float64, np.float32, np.int64, np.int32, np.int16, np.uint8):
        X = (rng.random((37, 5)) * 100).astype(dt)
        shifts = [0, -3, -1, 1, 2, 5]
        fill = np.array(np.nan if np.issubdtype(dt, np.floating) else 0, dtype=dt)
        src = torch.from_numpy(X).cuda()
        cols, sh = np.tile(np.arange(5), len(shifts)), np.repeat(shifts, 5)
        out = torch.empty((37, cols.size), dtype=src.dtype, device="cuda")
        cols_d = torch.tensor(cols, dtype=torch.int32).cuda()    # keep alive across the launch
        sh_d = torch.tensor(sh, dtype=torch.int32).cuda()
        _lib.call("sglm_timeshift_expand", src.data_ptr(), 37, 5, 1,
                  cols_d.data_ptr(), sh_d.data_ptr(), cols.size,
                  out.data_ptr(), 37, cols.size, 1, 0, X.itemsize,
                  int(fill.view(np.uint64 if X.itemsize == 8 else
                                {4: np.uint32, 2: np.uint16, 1: np.uint8}[X.itemsize])), 0)
        ref = pp_ref.timeshift_multiple(X, [], shifts, fill_value=fill)
        got = out.cpu().numpy()
        assert got.dtype == X.dtype
        assert np.array_equal(got, ref.astype(X.dtype), equal_nan=True), dt


def test_known_answers_through_kernel(engine, torch_mod, golden):
    """backend/test/test_sglm_pp.py known answers, computed by the HIP kernel."""
    import sglm_pp
    g = golden("timeshift_known.npz")
    X = g["ts_X"]
    assert np.array_equal(sglm_pp.timeshift(X, shift_amt=1, fill_value=0), g["ts_fwd"])
    assert np.array_equal(sglm_pp.timeshift(X, shift_amt=-1, fill_value=0), g["ts_bwd"])
    assert np.array_equal(sglm_pp.timeshift(X, [0, 1], 1, keep_non_inx=True, fill_value=0),
                          g["ts_keep_fwd"])
    assert np.array_equal(sglm_pp.timeshift_multiple(X, shift_amt_list=[-1, 0, 1], fill_value=0),
                          g["ts_multi_all"])
    assert np.array_equal(sglm_pp.timeshift_multiple(X, [0, 3], [-1, 0, 1], fill_value=0),
                          g["ts_multi_03"])


def test_design_from_events_matches_dense(engine, torch_mod):
    from sglm_hip import synth
    s = synth.make(N=5000, m=7, L=6, rho=0.1, seed=3)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    X = d.xb[: s.p, : s.N].float().cpu().numpy().T
    assert np.array_equal(X, s.dense_X(np.float32))
    assert d.xf is None
    assert np.all(d.xb[s.p, : s.N].float().cpu().numpy() == 1.0)
    assert np.all(d.xb[:, s.N:].float().cpu().numpy() == 0.0)


def test_pack_and_gemv(engine, torch_mod, monkeypatch):
    torch = torch_mod
    monkeypatch.setattr(engine, "MIXED_MAX_K", 0)      # the all-f32 design path
    rng = np.random.default_rng(2)
    X = rng.normal(size=(3000, 77))
    d = engine.Design.from_host(X)
    assert d.xf is not None          # real-valued: not bf16-exact
    beta = rng.normal(size=(5, d.P)).astype(np.float32)
    beta[:, 78:] = 0
    eta = d.eta(torch.from_numpy(beta).cuda()).cpu().numpy()[:, :3000]
    ref = (np.hstack([X, np.ones((3000, 1))]) @ beta[:, :78].T.astype(np.float64)).T
    assert rel(eta, ref) < 1e-5


def test_xtr_and_syrk_match_numpy(engine, torch_mod):
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=6000, m=9, L=5, rho=0.2, seed=4)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    Xa = np.hstack([s.dense_X(), np.ones((s.N, 1))])
    rng = np.random.default_rng(5)
    B = 3
    W = np.zeros((B, d.ld), np.float32)
    R = np.zeros((B, d.ld), np.float32)
    W[:, : s.N] = rng.random((B, s.N))
    R[:, : s.N] = rng.normal(size=(B, s.N))
    Wd, Rd = torch.from_numpy(W).cuda(), torch.from_numpy(R).cuda()
    G = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
    work = torch.empty(_lib.query("sglm_xtr_work_bytes", d.P, B, d.n), dtype=torch.uint8, device="cuda")
    _lib.call("sglm_xtr", d.xg.data_ptr(), d.xtype, d.ld, d.P, d.n, Rd.data_ptr(), B,
              G.data_ptr(), work.data_ptr(), 0)
    Gref = (Xa.T @ R[:, : s.N].T.astype(np.float64)).T
    assert rel(G.cpu().numpy()[:, : Xa.shape[1]], Gref) < 1e-6
    for splits in (1, 3):
        H = torch.zeros((B, d.P, d.P), dtype=torch.float32, device="cuda")
        fits = torch.tensor([2, 0], dtype=torch.int32, device="cuda")
        wb = _lib.query("sglm_syrk_work_bytes", d.P, 2, splits)
        wk = torch.empty(max(wb, 16), dtype=torch.uint8, device="cuda")
        _lib.call("sglm_syrk", d.xb.data_ptr(), d.ld, d.P, d.n, Wd.data_ptr(), fits.data_ptr(), 2,
                  splits, H.data_ptr(), wk.data_ptr(), 0)
        Hc = H.cpu().numpy()
        pa = Xa.shape[1]
        for k in (2, 0):
            wb16 = torch.from_numpy(W[k, : s.N]).to(torch.bfloat16).float().numpy().astype(np.float64)
            Href = (Xa * wb16[:, None]).T @ Xa
            up = np.triu(np.ones((pa, pa), bool))
            assert rel(Hc[k][:pa, :pa][up], Href[up]) < 2e-6, (splits, k)
        assert np.all(Hc[1] == 0)       # fit 1 not requested


def test_chol_solve_matches_numpy(engine, torch_mod):
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(6)
    P, B, p = 512, 2, 300
    A = rng.normal(size=(B, 2000, p + 1))
    H = np.zeros((B, P, P), np.float32)
    g = np.zeros((B, P))
    for k in range(B):
        H[k, : p + 1, : p + 1] = A[k].T @ A[k]
        g[k, : p + 1] = rng.normal(size=p + 1)
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = 3.0
    dsh[:, p] = 0.0
    Hd = torch.from_numpy(H).cuda()
    gd = torch.from_numpy(g).cuda()
    out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
    fits = torch.tensor([0, 1], dtype=torch.int32, device="cuda")
    dshd = torch.from_numpy(dsh).cuda()
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8, device="cuda")
    _lib.call("sglm_chol_solve_ex", Hd.data_ptr(), P, fits.data_ptr(), 2, gd.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), 1, B,
              cw.data_ptr(), 0)
    x = out.cpu().numpy()
    for k in range(B):
        M = H[k, : p + 1, : p + 1].astype(np.float64) + np.diag(np.r_[np.full(p, 3.0), 0.0])
        ref = -np.linalg.solve(M, g[k, : p + 1])
        assert rel(x[k, : p + 1], ref) < 1e-3
        assert np.all(x[k, p + 1:] == 0)
    # re-use the factor (refactor = 0) with a new right-hand side
    g2 = rng.normal(size=(B, P))
    g2[:, p + 1:] = 0
    g2d = torch.from_numpy(g2).cuda()
    _lib.call("sglm_chol_solve_ex", Hd.data_ptr(), P, fits.data_ptr(), 2, g2d.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), 0, B,
              cw.data_ptr(), 0)
    x2 = out.cpu().numpy()
    for k in range(B):
        M = H[k, : p + 1, : p + 1].astype(np.float64) + np.diag(np.r_[np.full(p, 3.0), 0.0])
        assert rel(x2[k, : p + 1], -np.linalg.solve(M, g2[k, : p + 1])) < 1e-3
    # mixed chain: fit 1 gets a new matrix and is factored, fit 0 keeps its factor
    A1 = rng.normal(size=(2000, p + 1))
    H1 = np.zeros((P, P), np.float32)
    H1[: p + 1, : p + 1] = A1.T @ A1
    Hd[1].copy_(torch.from_numpy(H1))
    order = torch.tensor([1, 0], dtype=torch.int32, device="cuda")
    _lib.call("sglm_chol_solve_mixed", Hd.data_ptr(), P, order.data_ptr(), 2, 1, g2d.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), B,
              cw.data_ptr(), 0)
    x3 = out.cpu().numpy()
    for k, Hk in ((0, H[0]), (1, H1)):
        M = Hk[: p + 1, : p + 1].astype(np.float64) + np.diag(np.r_[np.full(p, 3.0), 0.0])
        assert rel(x3[k, : p + 1], -np.linalg.solve(M, g2[k, : p + 1])) < 1e-3, k


@pytest.mark.parametrize("P,p,B", [(192, 150, 40), (2048, 1990, 4), (64, 40, 3)])
def test_chol_solve_inv_vs_float64(engine, torch_mod, P, p, B):
    """sglm_chol_solve_inv: factor + explicit inverse by recursive doubling (ragged P = 3 x 64
    and the C4 P = 2048), solves on own, kept and aliased (rscale, frozen set of the source)
    inverses in tiles of <= 32 fits, against float64 solves."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P)
    H = np.zeros((B, P, P), np.float32)
    for k in range(2):
        A = rng.normal(size=(p + 400, p + 1))
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)          # frozen padding
    dsh[:, :p] = 0.5
    dsh[:, p] = 0.0                                  # intercept: unpenalised
    dsh[:, 7] = -1.0                                 # a frozen coordinate
    g = rng.normal(size=(B, P))
    Hd = torch.from_numpy(H).cuda()
    Md = torch.empty_like(Hd)
    gd = torch.from_numpy(g).cuda()
    out = torch.full((B, P), np.nan, dtype=torch.float32, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
    dshd = torch.from_numpy(dsh).cuda()
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8, device="cuda")

    def solve(lst, fsrc, rsc, nref, tiles):
        ints = torch.tensor(np.r_[lst, fsrc, np.asarray(tiles).reshape(-1)].astype(np.int32),
                            device="cuda")
        rs = torch.tensor(np.asarray(rsc, np.float32), device="cuda")
        n = len(lst)
        _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, ints.data_ptr(),
                  ints[n:].data_ptr(), rs.data_ptr(), n, nref, ints[2 * n:].data_ptr(),
                  len(tiles), gd.data_ptr(), dshd.data_ptr(), out.data_ptr(), info.data_ptr(),
                  frozen.data_ptr(), B, cw.data_ptr(), 0)
        return out.cpu().numpy()

    free = np.flatnonzero(dsh[0] >= 0)

    def want(src, q, scale):
        Mm = H[src].astype(np.float64)[np.ix_(free, free)] + np.diag(dsh[src, free])
        x = np.zeros(P)
        x[free] = -scale * np.linalg.solve(Mm, g[q, free])
        return x

    al = list(range(2, B))
    rsc_al = list(rng.uniform(0.7, 1.3, size=len(al)))
    lst = [0, 1] + al
    fsrc = [0, 1] + [0] * len(al)
    tiles = [(0, 1), (1, 1)] + [(2 + i, min(32, len(al) - i)) for i in range(0, len(al), 32)]
    x = solve(lst, fsrc, [1.0, 1.0] + rsc_al, 2, tiles)
    for q, src, sc in [(0, 0, 1.0), (1, 1, 1.0)] + list(zip(al, [0] * len(al), rsc_al)):
        ref = want(src, q, sc)
        assert rel(x[q], ref) < 1e-3, (q, rel(x[q], ref))
        assert np.all(x[q, dsh[0] < 0] == 0)
    # kept factors, new right-hand sides; an alias of slot 1
    g[:] = rng.normal(size=(B, P))
    gd.copy_(torch.from_numpy(g))
    x = solve([1, 0, 2], [1, 0, 1], [1.0, 1.0, 0.9], 0, [(0, 1), (1, 1), (2, 1)])
    for q, src, sc in ((1, 1, 1.0), (0, 0, 1.0), (2, 1, 0.9)):
        assert rel(x[q], want(src, q, sc)) < 1e-3, q


@pytest.mark.parametrize("P,p", [(256, 200), (2048, 1990)])
def test_chol_diag_four_pivots_equals_two(engine, torch_mod, P, p, monkeypatch):
    """The factor + inverse chain with four pivots per barrier in the diagonal step
    (chol_diag4q_kernel), and with look-ahead and packed FMAs (chol_diag4l_kernel), leaves the
    same factor, inverse, frozen set and drop count as two pivots per barrier
    (chol_diag4_kernel), bit for bit: a duplicated column (a dropped pivot), a frozen
    coordinate, three fits."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P)
    B = 3
    H = np.zeros((B, P, P), np.float32)
    for k in range(B):
        A = rng.normal(size=(p + 300, p + 1))
        A[:, 5] = A[:, 9]                                # dependent column
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = rng.uniform(0.0, 0.5, size=(B, 1))
    dsh[:, p] = 0.0
    dsh[:, [5, 9]] = 0.0                                 # unpenalised: pivot 9 drops
    dsh[:, 17] = -1.0                                    # frozen
    outs = {}
    for q in ("l", "1", "0"):
        monkeypatch.setenv("SGLM_DIAG4Q", "0" if q == "0" else "1")
        monkeypatch.setenv("SGLM_DIAG4L", "1" if q == "l" else "0")
        Hd = torch.from_numpy(H).cuda()
        Md = torch.zeros_like(Hd)
        out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
        info = torch.zeros(B, dtype=torch.int32, device="cuda")
        frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
        dshd = torch.from_numpy(dsh).cuda()
        cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8,
                         device="cuda")
        lst = torch.arange(B, dtype=torch.int32, device="cuda")
        rs = torch.ones(B, dtype=torch.float32, device="cuda")
        _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, lst.data_ptr(),
                  lst.data_ptr(), rs.data_ptr(), B, B, None, 0, None, dshd.data_ptr(),
                  out.data_ptr(), info.data_ptr(), frozen.data_ptr(), B, cw.data_ptr(), 0)
        torch.cuda.synchronize()
        outs[q] = [t.cpu().numpy() for t in (Hd, Md, info, frozen)]
    assert (outs["1"][2] >= 1).all()                     # the dependent column dropped
    for v in ("1", "l"):
        for a, b in zip(outs[v], outs["0"]):
            assert np.array_equal(a, b, equal_nan=True), v


@pytest.mark.parametrize("P,p,graph", [(192, 150, False), (2048, 1990, False), (2048, 1990, True)])
def test_chol_inv_columns_equal_levels(engine, torch_mod, P, p, graph, monkeypatch):
    """The inverse by left-looking block columns on a branch beside the factorisation
    (chol_inv_col_kernel, SGLM_INV_COL=1, the default) leaves the factor, frozen set and drop
    count bit for bit as the recursive-doubling levels after the chain (SGLM_INV_COL=0), and
    the same inverse to f32 rounding (zeros in the frozen and dropped columns): a dependent
    column, a frozen coordinate, three fits, on the null stream (direct launches) and on a
    stream (the cached chain graph with its two branches)."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P + 11)
    B = 3
    H = np.zeros((B, P, P), np.float32)
    for k in range(B):
        A = rng.normal(size=(p + 300, p + 1))
        A[:, 5] = A[:, 9]                                # dependent column
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = rng.uniform(0.0, 0.5, size=(B, 1))
    dsh[:, p] = 0.0
    dsh[:, [5, 9]] = 0.0                                 # unpenalised: pivot 9 drops
    dsh[:, 17] = -1.0                                    # frozen
    outs = {}
    st = torch.cuda.Stream() if graph else None
    monkeypatch.setenv("SGLM_INV_X3", "0")              # the levels in f32, as the columns
    for v in ("1", "0", "1"):
        monkeypatch.setenv("SGLM_INV_COL", v)
        Hd = torch.from_numpy(H).cuda()
        Md = torch.zeros_like(Hd)
        out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
        info = torch.zeros(B, dtype=torch.int32, device="cuda")
        frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
        dshd = torch.from_numpy(dsh).cuda()
        cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8,
                         device="cuda")
        lst = torch.arange(B, dtype=torch.int32, device="cuda")
        rs = torch.ones(B, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, lst.data_ptr(),
                  lst.data_ptr(), rs.data_ptr(), B, B, None, 0, None, dshd.data_ptr(),
                  out.data_ptr(), info.data_ptr(), frozen.data_ptr(), B, cw.data_ptr(),
                  st.cuda_stream if graph else 0)
        torch.cuda.synchronize()
        res = [t.cpu().numpy() for t in (Hd, Md, info, frozen)]
        if v in outs:                                    # a replay (graph) is deterministic
            for a, b in zip(res, outs[v]):
                assert np.array_equal(a, b, equal_nan=True)
        outs[v] = res
    (Hc, Mc, ic, fc), (Hl, Ml, il, fl) = outs["1"], outs["0"]
    assert (ic >= 1).all() and np.array_equal(ic, il) and np.array_equal(fc, fl)
    up = np.triu(np.ones((P, P), bool))
    assert np.array_equal(Hc[:, up], Hl[:, up])          # the factor is untouched
    for k in range(B):
        Uc, Ul = np.triu(Mc[k]).astype(np.float64), np.triu(Ml[k]).astype(np.float64)
        assert np.linalg.norm(Uc - Ul) <= 1e-5 * np.linalg.norm(Ul), k
        dead = fc[k].astype(bool)
        assert np.all(Mc[k][:, dead][up[:, dead]] == 0)  # frozen / dropped columns of M
        U = np.triu(Hc[k]).astype(np.float64)
        keep = np.flatnonzero(~dead)
        Iu = Uc[np.ix_(keep, keep)] @ U[np.ix_(keep, keep)]
        assert np.abs(Iu - np.eye(keep.size)).max() < 1e-3, k


@pytest.mark.parametrize("P,p,graph", [(192, 150, False), (2048, 1990, True)])
def test_chol_factor_then_invert(engine, torch_mod, P, p, graph):
    """sglm_chol_factor + sglm_chol_invert (the engine's deferred inversion) leave the factor,
    inverse, frozen set and drop count of sglm_chol_solve_inv bit for bit, and the substitution
    solve on the fresh factors (sglm_chol_solve_alias: own and aliased fits) matches the float64
    solve: a dependent column, a frozen coordinate, three fits."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P + 23)
    B = 3
    H = np.zeros((B, P, P), np.float32)
    for k in range(B):
        A = rng.normal(size=(p + 300, p + 1))
        A[:, 5] = A[:, 9]
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = rng.uniform(0.1, 0.5, size=(B, 1))
    dsh[:, p] = 0.0
    dsh[:, [5, 9]] = 0.0                                 # unpenalised: pivot 9 drops
    dsh[:, 17] = -1.0
    g = rng.normal(size=(B, P))
    st = torch.cuda.Stream() if graph else None
    sp = st.cuda_stream if graph else 0
    outs = []
    for mode in ("whole", "split"):
        Hd = torch.from_numpy(H).cuda()
        Md = torch.zeros_like(Hd)
        out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
        info = torch.zeros(B, dtype=torch.int32, device="cuda")
        frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
        dshd = torch.from_numpy(dsh).cuda()
        cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8,
                         device="cuda")
        lst = torch.arange(B, dtype=torch.int32, device="cuda")
        rs = torch.ones(B, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        if mode == "whole":
            _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, lst.data_ptr(),
                      lst.data_ptr(), rs.data_ptr(), B, B, None, 0, None, dshd.data_ptr(),
                      out.data_ptr(), info.data_ptr(), frozen.data_ptr(), B, cw.data_ptr(), sp)
        else:
            _lib.call("sglm_chol_factor", Hd.data_ptr(), Md.data_ptr(), P, lst.data_ptr(), B,
                      dshd.data_ptr(), info.data_ptr(), frozen.data_ptr(), B, cw.data_ptr(), sp)
            # substitution on the fresh factors: fits 0, 1 on their own, fit 2 aliased to 0
            gd = torch.from_numpy(g).cuda()
            fl = torch.tensor([0, 1, 2], dtype=torch.int32, device="cuda")
            fs = torch.tensor([0, 1, 0], dtype=torch.int32, device="cuda")
            rsc = torch.tensor([1.0, 1.0, 0.8], dtype=torch.float32, device="cuda")
            cw2 = torch.empty_like(cw)
            _lib.call("sglm_chol_solve_alias", Hd.data_ptr(), P, fl.data_ptr(), fs.data_ptr(), 3,
                      gd.data_ptr(), rsc.data_ptr(), out.data_ptr(), frozen.data_ptr(), B,
                      cw2.data_ptr(), sp)
            _lib.call("sglm_chol_invert", Hd.data_ptr(), Md.data_ptr(), P, lst.data_ptr(), B, B,
                      cw.data_ptr(), sp)
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy() for t in (Hd, Md, info, frozen, out)])
    (Hw, Mw, iw, fw, _), (Hs, Ms, is_, fs_, xs) = outs
    up = np.triu(np.ones((P, P), bool))
    assert np.array_equal(Hw[:, up], Hs[:, up]) and np.array_equal(Mw[:, up], Ms[:, up])
    assert np.array_equal(iw, is_) and np.array_equal(fw, fs_) and (iw >= 1).all()
    for q, src, sc in ((0, 0, 1.0), (1, 1, 1.0), (2, 0, 0.8)):
        keep = np.flatnonzero(~fs_[src].astype(bool))
        Mm = H[src].astype(np.float64)[np.ix_(keep, keep)] + np.diag(dsh[src, keep])
        ref = np.zeros(P)
        ref[keep] = -sc * np.linalg.solve(Mm, g[q, keep])
        assert rel(xs[q], ref) < 1e-3, (q, rel(xs[q], ref))
        assert np.all(xs[q, fs_[src].astype(bool)] == 0)


@pytest.mark.parametrize("P,p", [(192, 150), (2048, 1990)])
def test_chol_inv_split_precision_levels(engine, torch_mod, P, p, monkeypatch):
    """The inversion levels with split-precision products (SGLM_INV_X3, the default: three
    bf16 MFMAs per product, hi hi + hi lo + lo hi) leave the factor, frozen set and drop count
    of the f32 levels bit for bit and an inverse within 1e-4 of theirs (relative, Frobenius)
    whose solves match float64 at the other tests' 1e-3."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P + 31)
    B = 2
    H = np.zeros((B, P, P), np.float32)
    for k in range(B):
        A = rng.normal(size=(p + 300, p + 1))
        A[:, 5] = A[:, 9]
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = rng.uniform(0.05, 0.5, size=(B, 1))
    dsh[:, p] = 0.0
    dsh[:, [5, 9]] = 0.0
    dsh[:, 17] = -1.0
    g = rng.normal(size=(B, P))
    outs = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SGLM_INV_X3", v)
        Hd = torch.from_numpy(H).cuda()
        Md = torch.zeros_like(Hd)
        gd = torch.from_numpy(g).cuda()
        out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
        info = torch.zeros(B, dtype=torch.int32, device="cuda")
        frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
        dshd = torch.from_numpy(dsh).cuda()
        cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8,
                         device="cuda")
        ints = torch.tensor(np.r_[np.arange(B), np.arange(B), np.c_[np.arange(B), np.ones(B)]
                                  .reshape(-1)].astype(np.int32), device="cuda")
        rs = torch.ones(B, dtype=torch.float32, device="cuda")
        _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, ints.data_ptr(),
                  ints[B:].data_ptr(), rs.data_ptr(), B, B, ints[2 * B:].data_ptr(), B,
                  gd.data_ptr(), dshd.data_ptr(), out.data_ptr(), info.data_ptr(),
                  frozen.data_ptr(), B, cw.data_ptr(), 0)
        torch.cuda.synchronize()
        outs[v] = [t.cpu().numpy() for t in (Hd, Md, info, frozen, out)]
    (Hx, Mx, ix, fx, xx), (Hf, Mf, if_, ff, _) = outs["1"], outs["0"]
    up = np.triu(np.ones((P, P), bool))
    assert np.array_equal(Hx[:, up], Hf[:, up]) and np.array_equal(ix, if_)
    assert np.array_equal(fx, ff) and (ix >= 1).all()
    for k in range(B):
        Ux, Uf = np.triu(Mx[k]).astype(np.float64), np.triu(Mf[k]).astype(np.float64)
        assert np.linalg.norm(Ux - Uf) <= 1e-4 * np.linalg.norm(Uf), k
        keep = np.flatnonzero(~fx[k].astype(bool))
        Mm = H[k].astype(np.float64)[np.ix_(keep, keep)] + np.diag(dsh[k, keep])
        ref = np.zeros(P)
        ref[keep] = -np.linalg.solve(Mm, g[k, keep])
        assert rel(xx[k], ref) < 1e-3, (k, rel(xx[k], ref))


@pytest.mark.parametrize("P,p,B", [(768, 700, 6), (2048, 1990, 5)])
def test_chol_inv_many_fits_vs_float64(engine, torch_mod, P, p, B, monkeypatch):
    """Factor + inverse chain on several fits of their own with the 128 x 128 inversion tiles
    forced on every level s >= 128 (SGLM_INV128_WG=1: the ragged last level of P = 768, the
    four 128-tile levels of P = 2048), each solve against its float64 solve."""
    torch = torch_mod
    monkeypatch.setenv("SGLM_INV128_WG", "1")
    from sglm_hip import _lib
    rng = np.random.default_rng(P + B)
    H = np.zeros((B, P, P), np.float32)
    for k in range(B):
        A = rng.normal(size=(p + 300, p + 1))
        H[k, : p + 1, : p + 1] = A.T @ A / 100.0
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :p] = rng.uniform(0.2, 1.0, size=(B, 1))
    dsh[:, p] = 0.0
    g = rng.normal(size=(B, P))
    Hd = torch.from_numpy(H).cuda()
    Md = torch.empty_like(Hd)
    gd = torch.from_numpy(g).cuda()
    out = torch.full((B, P), np.nan, dtype=torch.float32, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
    dshd = torch.from_numpy(dsh).cuda()
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8, device="cuda")
    lst = list(range(B))
    tiles = [(q, 1) for q in range(B)]               # a tile shares one factor
    ints = torch.tensor(np.r_[lst, lst, np.asarray(tiles).reshape(-1)].astype(np.int32),
                        device="cuda")
    rs = torch.ones(B, dtype=torch.float32, device="cuda")
    _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, ints.data_ptr(),
              ints[B:].data_ptr(), rs.data_ptr(), B, B, ints[2 * B:].data_ptr(), B,
              gd.data_ptr(), dshd.data_ptr(), out.data_ptr(), info.data_ptr(),
              frozen.data_ptr(), B, cw.data_ptr(), 0)
    x = out.cpu().numpy()
    assert (info.cpu().numpy() == 0).all()
    free = np.arange(p + 1)
    for q in range(B):
        Mm = H[q].astype(np.float64)[np.ix_(free, free)] + np.diag(dsh[q, free])
        ref = np.zeros(P)
        ref[free] = -np.linalg.solve(Mm, g[q, free])
        assert rel(x[q], ref) < 1e-3, (q, rel(x[q], ref))
        assert np.all(x[q, p + 1:] == 0)


@pytest.mark.parametrize("P", [128, 2048])
def test_chol_inv_dropped_pivots(engine, torch_mod, P):
    """Factor + inverse chain (four-wave diagonal step) on a Gram with exactly duplicated and
    all-zero columns and no ridge: the dependent pivots fall below 1e-6 of their diagonal and
    are dropped (counted in info, frozen), and the solve on the explicit inverse equals the
    float64 solve restricted to the kept coordinates."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(P + 7)
    p = P - 9
    A = rng.normal(size=(p + 300, p))
    dup = [3, 70 % p, p - 2]                         # columns that copy their left neighbour
    for j in dup:
        A[:, j] = A[:, j - 1]
    A[:, 5] = 0.0                                    # an all-zero column (frozen at prep)
    H = np.zeros((1, P, P), np.float32)
    H[0, :p, :p] = A.T @ A / 100.0
    dsh = np.full((1, P), -1.0, np.float32)          # frozen padding
    dsh[0, :p] = 0.0                                 # no ridge: duplicates are singular
    g = rng.normal(size=(1, P))
    Hd = torch.from_numpy(H).cuda()
    Md = torch.empty_like(Hd)
    gd = torch.from_numpy(g).cuda()
    out = torch.full((1, P), np.nan, dtype=torch.float32, device="cuda")
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((1, P), dtype=torch.uint8, device="cuda")
    dshd = torch.from_numpy(dsh).cuda()
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, 1), dtype=torch.uint8, device="cuda")
    ints = torch.tensor(np.array([0, 0, 0, 1], np.int32), device="cuda")   # fits, fsrc, tile
    rs = torch.ones(1, dtype=torch.float32, device="cuda")
    _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, ints.data_ptr(),
              ints[1:].data_ptr(), rs.data_ptr(), 1, 1, ints[2:].data_ptr(), 1, gd.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), 1,
              cw.data_ptr(), 0)
    x = out.cpu().numpy()[0]
    frz = frozen.cpu().numpy()[0].astype(bool)
    assert int(info.item()) == len(dup)              # the duplicates' pivots were dropped
    assert frz[dup].all() and frz[5] and frz[p:].all()
    keep = np.flatnonzero(~frz)
    assert keep.size == p - len(dup) - 1
    Hk = (A.T @ A / 100.0)[np.ix_(keep, keep)]
    ref = np.zeros(P)
    ref[keep] = -np.linalg.solve(Hk, g[0, keep])
    assert np.all(x[frz] == 0)
    assert rel(x, ref) < 1e-2, rel(x, ref)


def _fit_one(engine, X, y, family, power, lam, fit_intercept=True):
    d = engine.Design.from_host(X)
    prob = engine.Problem(d, [y], [np.ones(len(y), np.uint8)])
    req = engine.FitReq(family=family, power=power, lam=lam, mask=0, resp=0,
                        fit_intercept=fit_intercept)
    (res,), _ = engine.irls(prob, [req])
    return res


def test_engine_poisson_vs_golden(engine, golden):
    g = golden("fits.npz")
    meta = json.load(open(os.path.join(GOLDEN, "fits_meta.json")))
    X, y = g["pois_X"], g["pois_y"]
    n = X.shape[0]
    for m in meta:
        r = _fit_one(engine, X, y, engine.FAM_TWEEDIE_LOG, 1.0, m["alpha"] * n, m["fit_intercept"])
        assert r.converged, m
        assert rel(r.coef, g[m["key"] + "_coef"]) < 1e-4, m           # north-star tolerance
        assert abs(r.intercept - float(g[m["key"] + "_b"])) < 1e-4 * max(1, abs(float(g[m["key"] + "_b"])))


def test_engine_gaussian_vs_golden(engine, golden):
    g = golden("fits.npz")
    X, y = g["gau_X"], g["gau_y"]
    r = _fit_one(engine, X, y, engine.FAM_SQUARED, 0.0, 0.0)
    assert rel(r.coef, g["ols_coef"]) < 1e-5
    for i, a in enumerate([0.1, 10.0, 1000.0]):
        r = _fit_one(engine, X, y, engine.FAM_SQUARED, 0.0, a)
        assert rel(r.coef, g[f"ridge_a{i}_coef"]) < 1e-5, a
        assert abs(r.intercept - float(g[f"ridge_a{i}_b"])) < 1e-5 * max(1, abs(float(g[f"ridge_a{i}_b"])))


def test_engine_gamma_vs_golden(engine, golden):
    g = golden("fits.npz")
    X, y = g["gam_X"], g["gam_y"]
    r = _fit_one(engine, X, y, engine.FAM_TWEEDIE_LOG, 2.0, 0.05 * X.shape[0])
    assert rel(r.coef, g["gam_coef"]) < 1e-4


def test_engine_batched_masks_match_oracle(engine):
    """Several (mask, lambda) fits in one batch == separate float64 fits on the row subsets."""
    from sglm_hip import synth
    s = synth.make(N=8000, m=5, L=4, rho=0.08, seed=9, beta_scale=0.3)
    X = s.dense_X()
    rng = np.random.default_rng(0)
    masks = [(rng.random(s.N) < 0.8).astype(np.uint8) for _ in range(3)]
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    prob = engine.Problem(d, [s.y], masks)
    reqs, refs = [], []
    for mi, m in enumerate(masks):
        for a in (1e-3, 1e-1):
            n_tr = int(m.sum())
            reqs.append(engine.FitReq(engine.FAM_TWEEDIE_LOG, 1.0, a * n_tr, mi, 0))
            refs.append(glm_ref.fit_tweedie_newton(X[m == 1], s.y[m == 1], a, 1.0))
    res, _ = engine.irls(prob, reqs)
    for r, (c, b) in zip(res, refs):
        assert r.converged
        assert rel(r.coef, c) < 1e-4


def test_syrk_f32_exact_gram(engine, torch_mod, monkeypatch):
    """Real-valued (not bf16-exact) design: the f32-MFMA Gram matches float64 to ~1e-6."""
    torch = torch_mod
    monkeypatch.setattr(engine, "MIXED_MAX_K", 0)      # the all-f32 design path
    from sglm_hip import _lib
    rng = np.random.default_rng(8)
    X = rng.normal(size=(5000, 140))
    d = engine.Design.from_host(X)
    assert d.xf is not None
    W = np.zeros((2, d.ld), np.float32)
    W[:, :5000] = rng.random((2, 5000))
    Wd = torch.from_numpy(W).cuda()
    Xa = np.hstack([X.astype(np.float32).astype(np.float64), np.ones((5000, 1))])
    for splits in (1, 4):
        H = torch.zeros((2, d.P, d.P), dtype=torch.float32, device="cuda")
        fits = torch.tensor([1], dtype=torch.int32, device="cuda")
        wk = torch.empty(max(_lib.query("sglm_syrk_work_bytes", d.P, 1, splits), 16),
                         dtype=torch.uint8, device="cuda")
        _lib.call("sglm_syrk_f32", d.xf.data_ptr(), d.ld, d.P, d.n, Wd.data_ptr(),
                  fits.data_ptr(), 1, splits, H.data_ptr(), wk.data_ptr(), 0)
        pa = Xa.shape[1]
        Href = (Xa * W[1, :5000, None].astype(np.float64)).T @ Xa
        up = np.triu(np.ones((pa, pa), bool))
        assert rel(H[1].cpu().numpy()[:pa, :pa][up], Href[up]) < 1e-5, splits   # f32 accumulation


def test_syrk_masked_row_groups(engine, torch_mod):
    """Row-group gathering (skipped test-trial blocks) == the dense masked Gram, bitwise."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=20000, m=9, L=5, rho=0.2, seed=12)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(13)
    trial_test = rng.random(200) < 0.3                # 100-row trials held out
    masks = [np.repeat(~trial_test, 100).astype(np.uint8), np.ones(s.N, np.uint8),
             np.zeros(s.N, np.uint8)]
    masks[2][:37] = 1                                  # a fit with a single partial group
    prob = engine.Problem(d, [s.y], masks)
    B = 3
    W = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    for k in range(B):
        W[k, : s.N] = torch.from_numpy(masks[k].astype(np.float32) * rng.random(s.N).astype(np.float32))
    fits = torch.tensor([0, 1, 2], dtype=torch.int32, device="cuda")
    goff = torch.from_numpy(prob.group_offset).cuda()
    gcnt = torch.from_numpy(prob.group_count).cuda()
    for splits in (1, 2):
        wk = torch.empty(max(_lib.query("sglm_syrk_work_bytes", d.P, B, splits), 16),
                         dtype=torch.uint8, device="cuda")
        H1 = torch.zeros((B, d.P, d.P), dtype=torch.float32, device="cuda")
        H2 = torch.zeros_like(H1)
        _lib.call("sglm_syrk", d.xb.data_ptr(), d.ld, d.P, d.n, W.data_ptr(), fits.data_ptr(), B,
                  splits, H1.data_ptr(), wk.data_ptr(), 0)
        _lib.call("sglm_syrk_masked", d.xb.data_ptr(), d.ld, d.P, d.n, W.data_ptr(),
                  fits.data_ptr(), B, splits, H2.data_ptr(), wk.data_ptr(),
                  prob.groups.data_ptr(), goff.data_ptr(), gcnt.data_ptr(), 0)
        up = torch.triu(torch.ones((d.P, d.P), dtype=torch.bool, device="cuda"))
        for k in range(B):
            a, b = H1[k][up], H2[k][up]
            assert torch.max(torch.abs(a - b)).item() <= 1e-6 * max(1.0, torch.max(torch.abs(a)).item()), (splits, k)


def _unpack_cbits(bits, P, nrows):
    """Host decode of the v6 compact layout -> (nrows, P) 0/1 matrix."""
    nblk = max(1, (nrows + 63) // 64)
    w = bits.reshape(nblk, P, 2).astype(np.uint32)
    rho = np.arange(32)
    pos = 4 * (rho // 8) + (rho % 8) // 2 + 16 * (rho % 2)
    out = np.zeros((nblk, 64, P), np.uint8)
    for half in range(2):
        out[:, 32 * half + rho, :] = ((w[:, :, half][:, None, :] >> pos[None, :, None]) & 1)
    return out.reshape(nblk * 64, P)[:nrows]


def test_pack_bits_rows_layout(engine, torch_mod):
    """Compacted bit-planes decode back to X[rows] (ragged row count, zero tail)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=5000, m=7, L=3, rho=0.2, seed=21)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    Xh = d.xb.float().cpu().numpy().T[: s.N]                 # (n, P)
    rng = np.random.default_rng(22)
    for rows in (np.sort(rng.choice(s.N, 1234, replace=False)).astype(np.int32), None):
        nr = 1234 if rows is not None else s.N
        rows_d = None if rows is None else torch.from_numpy(rows).cuda()
        bits = torch.zeros(((nr + 63) // 64) * d.P * 2, dtype=torch.int32, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        _lib.call("sglm_pack_bits_rows", d.xb.data_ptr(), d.ld, d.P,
                  None if rows_d is None else rows_d.data_ptr(), nr, bits.data_ptr(),
                  flag.data_ptr(), 0)
        torch.cuda.synchronize()
        assert int(flag.item()) == 0
        got = _unpack_cbits(bits.cpu().numpy().view(np.uint32), d.P, nr)
        ref = Xh if rows is None else Xh[rows]
        assert np.array_equal(got, ref.astype(np.uint8))
        tail = _unpack_cbits(bits.cpu().numpy().view(np.uint32), d.P, ((nr + 63) // 64) * 64)
        assert not tail[nr:].any()


def test_syrk_cbits_compacted_gram(engine, torch_mod):
    """Gram v6 (row-compacted bit-planes, register MFMA): bitwise equal to v2 on the full
    mask; within f32 summation-order noise of the float64 Gram on subsets (incl. empty)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=20000, m=13, L=6, rho=0.1, seed=31)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(32)
    masks = [np.ones(s.N, np.uint8), np.repeat(rng.random(200) >= 0.3, 100).astype(np.uint8),
             np.zeros(s.N, np.uint8), (rng.random(s.N) < 0.5).astype(np.uint8)]
    prob = engine.Problem(d, [s.y], masks)
    B = len(masks)
    W = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    for k in range(B):
        W[k, : s.N] = torch.from_numpy(masks[k] * (0.1 + rng.random(s.N)).astype(np.float32))
    fits = torch.arange(B, dtype=torch.int32, device="cuda")
    cbs = [prob.compact(k) for k in range(B)]
    nr_max = max(c[1] for c in cbs)
    stride = max(64, (nr_max + 63) // 64 * 64)
    wc = torch.zeros(B * stride, dtype=torch.bfloat16, device="cuda")
    desc = torch.tensor([[c[0].data_ptr(), c[1], wc.data_ptr() + 2 * k * stride,
                          0 if c[2] is None else c[2].data_ptr()] for k, c in enumerate(cbs)],
                        dtype=torch.int64).cuda()
    _lib.call("sglm_gather_w", W.data_ptr(), d.ld, fits.data_ptr(), B, desc.data_ptr(), nr_max, 0)
    Xh = d.xb.double().cpu().numpy()[:, : s.N]
    Wb = W.to(torch.bfloat16).double().cpu().numpy()[:, : s.N]
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))         # what the consumers read
    Href = torch.zeros((1, d.P, d.P), dtype=torch.float32, device="cuda")
    wk1 = torch.empty(16, dtype=torch.uint8, device="cuda")
    _lib.call("sglm_syrk", d.xb.data_ptr(), d.ld, d.P, d.n, W.data_ptr(),
              fits.data_ptr(), 1, 1, Href.data_ptr(), wk1.data_ptr(), 0)
    for splits in (1, 4):
        wk = torch.empty(max(_lib.query("sglm_syrk_work_bytes", d.P, B, splits), 16),
                         dtype=torch.uint8, device="cuda")
        H = torch.full((B, d.P, d.P), float("nan"), dtype=torch.float32, device="cuda")
        _lib.call("sglm_syrk_cbits", desc.data_ptr(), d.P, fits.data_ptr(), B, splits,
                  H.data_ptr(), wk.data_ptr(), 0)
        Hh = H.cpu().numpy()
        if splits == 1:
            assert np.array_equal(Hh[0][blk], Href[0].cpu().numpy()[blk])
        for k in range(B):
            ref = (Xh * Wb[k]) @ Xh.T
            got = Hh[k][blk]
            assert np.all(np.isfinite(got)), (splits, k)
            scale = max(np.max(np.abs(ref)), 1.0)
            assert np.max(np.abs(got - ref[blk])) <= 2e-6 * scale, (splits, k)


@pytest.mark.parametrize("L,splits", [(10, 1), (20, 3)])
def test_syrk_cbits_xcd_banded_placement(engine, torch_mod, monkeypatch, L, splits):
    """SGLM_SYRK_XCD=1 (128-blocks dealt to the XCDs by band pairs) computes every block with
    the same K slabs as the default placement: the Grams are equal bit for bit (P = 512 and
    1024, 1 and 3 row slabs, 3 fits)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=20000, m=50, L=L, rho=0.05, seed=L)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    assert (d.P // 128) % 4 == 0
    rng = np.random.default_rng(L)
    masks = [np.ones(s.N, np.uint8), (rng.random(s.N) < 0.5).astype(np.uint8),
             np.repeat(rng.random(200) >= 0.3, 100).astype(np.uint8)]
    prob = engine.Problem(d, [s.y], masks)
    B = len(masks)
    W = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    for k in range(B):
        W[k, : s.N] = torch.from_numpy(masks[k] * (0.1 + rng.random(s.N)).astype(np.float32))
    fits = torch.arange(B, dtype=torch.int32, device="cuda")
    cbs = [prob.compact(k) for k in range(B)]
    nr_max = max(c[1] for c in cbs)
    stride = max(64, (nr_max + 63) // 64 * 64)
    wc = torch.zeros(B * stride, dtype=torch.bfloat16, device="cuda")
    desc = torch.tensor([[c[0].data_ptr(), c[1], wc.data_ptr() + 2 * k * stride,
                          0 if c[2] is None else c[2].data_ptr()] for k, c in enumerate(cbs)],
                        dtype=torch.int64).cuda()
    _lib.call("sglm_gather_w", W.data_ptr(), d.ld, fits.data_ptr(), B, desc.data_ptr(), nr_max, 0)
    wk = torch.empty(max(_lib.query("sglm_syrk_work_bytes", d.P, B, splits), 16),
                     dtype=torch.uint8, device="cuda")
    blk = np.triu(np.ones((d.P, d.P), dtype=bool))
    out = {}
    for xm in ("0", "1"):
        monkeypatch.setenv("SGLM_SYRK_XCD", xm)
        H = torch.full((B, d.P, d.P), float("nan"), dtype=torch.float32, device="cuda")
        _lib.call("sglm_syrk_cbits", desc.data_ptr(), d.P, fits.data_ptr(), B, splits,
                  H.data_ptr(), wk.data_ptr(), 0)
        out[xm] = H.cpu().numpy()
    for k in range(B):
        assert np.all(np.isfinite(out["1"][k][blk])), k
        assert np.array_equal(out["0"][k][blk], out["1"][k][blk]), k


def test_eta_bits_matches_float64(engine, torch_mod):
    """MFMA eta over row-major bit-planes (beta split in 3 bf16 pieces) == X @ beta to f32
    accuracy, for every row incl. padding (0), with a ragged fit count (B = 37)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=7000, m=11, L=4, rho=0.1, seed=41)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    assert d.rbits is not None
    rng = np.random.default_rng(42)
    B = 37
    beta = (rng.standard_normal((B, d.P)) * np.exp(rng.uniform(-8, 3, (B, d.P)))).astype(np.float32)
    beta[:, d.p + 1:] = 0.0
    bd = torch.from_numpy(beta).cuda()
    out = torch.full((B, d.ld), float("nan"), dtype=torch.float32, device="cuda")
    work = torch.empty(_lib.query("sglm_eta_bits_work_bytes", d.P, B), dtype=torch.uint8,
                       device="cuda")
    _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, bd.data_ptr(), B, None, 1,
              out.data_ptr(), work.data_ptr(), 0)
    # a slot list computes exactly those rows (bitwise: each fit's column is independent) and
    # leaves the others untouched
    sl = torch.tensor([36, 0, 17, 5], dtype=torch.int32, device="cuda")
    out_s = torch.full_like(out, float("nan"))
    _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, bd.data_ptr(), 4,
              sl.data_ptr(), 1, out_s.data_ptr(), work.data_ptr(), 0)
    for k in (36, 0, 17, 5):
        assert torch.equal(out_s[k], out[k]), k
    assert torch.isnan(out_s[1]).all()
    ref_valu = torch.empty_like(out)
    _lib.call("sglm_gemv_eta", d.xb.data_ptr(), 0, d.ld, d.P, d.n, bd.data_ptr(), B,
              ref_valu.data_ptr(), 0)
    X = d.xb.double().cpu().numpy()                       # (P, ld)
    ref = beta.astype(np.float64) @ X                     # (B, ld)
    got = out.cpu().numpy()
    assert np.all(np.isfinite(got))
    scale = np.abs(beta.astype(np.float64)) @ np.abs(X)   # error bound scale per entry
    assert np.max(np.abs(got - ref) / np.maximum(scale, 1e-30)) < 2e-6
    assert not got[:, s.N + 1:].any()                     # padding rows are exactly 0
    assert np.max(np.abs(got - ref_valu.cpu().numpy()) / np.maximum(scale, 1e-30)) < 2e-6
    # direction mode: the selected rows of beta are rounded to bf16 in place and X times the
    # rounded rows is returned (one piece); other rows of beta are untouched
    bd2 = bd.clone()
    out_r = torch.full_like(out, float("nan"))
    _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, bd2.data_ptr(), 4,
              sl.data_ptr(), 0, out_r.data_ptr(), work.data_ptr(), 0)
    for k in (36, 0, 17, 5):
        assert torch.equal(bd2[k], bd[k].to(torch.bfloat16).float()), k
        rk = bd2[k].double().cpu().numpy() @ X
        sk = np.abs(bd2[k].double().cpu().numpy()) @ np.abs(X)
        assert np.max(np.abs(out_r[k].cpu().numpy() - rk) / np.maximum(sk, 1e-30)) < 2e-6, k
    assert torch.equal(bd2[1], bd[1]) and torch.isnan(out_r[1]).all()


@pytest.mark.parametrize("B", [200, 100, 70, 33, 7])
def test_eta_dir_kernel_equals_per_group_kernel(engine, torch_mod, B, monkeypatch):
    """Direction products through the pipelined kernel (eta_pipe_kernel<4, 4> / <2, 8> /
    <1, 8>: 512 / 1024 rows per workgroup, waves past the last row, ragged fit groups), the
    LDS-staged kernel (eta_dir_kernel: 128 fits x 256 rows per workgroup) and the per-group
    kernel agree bit for bit, and X d in float64 to f32 accuracy, through a slot list."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=20000, m=30, L=6, rho=0.05, seed=B)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(B)
    nb = B + 5
    beta = (rng.standard_normal((nb, d.P)) * np.exp(rng.uniform(-8, 3, (nb, d.P)))).astype(np.float32)
    beta[:, d.p + 1:] = 0.0
    slots = rng.permutation(nb)[:B].astype(np.int32)
    sl = torch.from_numpy(slots).cuda()
    work = torch.empty(_lib.query("sglm_eta_bits_work_bytes", d.P, B), dtype=torch.uint8,
                       device="cuda")
    outs = {}
    assert d.ld % 512 == 256                          # dead waves in the last workgroup
    variants = {"pipe": ("1", "0", "0"), "dir": ("0", "1", "0"), "group": ("0", "0", "0")}
    for c in "1234":
        variants["cfg" + c] = ("1", "0", c)
    for v, (pipe, dr, cfg) in variants.items():
        monkeypatch.setenv("SGLM_ETA_PIPE", pipe)
        monkeypatch.setenv("SGLM_ETA_DIR", dr)
        monkeypatch.setenv("SGLM_ETA_PIPE_CFG", cfg)
        bd = torch.from_numpy(beta).cuda()
        out = torch.full((nb, d.ld), float("nan"), dtype=torch.float32, device="cuda")
        _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, bd.data_ptr(), B,
                  sl.data_ptr(), 0, out.data_ptr(), work.data_ptr(), 0)
        outs[v] = (out.cpu().numpy(), bd.cpu().numpy())
    got, br = outs["pipe"]
    for v in variants:
        assert np.array_equal(outs[v][0], outs["group"][0], equal_nan=True), v
    monkeypatch.setenv("SGLM_ETA_PIPE_CFG", "0")
    # exact coefficients (three pieces): the pipelined kernel == the staged one, bit for bit
    ex = {}
    for v, (pipe, c3) in {"pipe": ("1", "0"), "pipe_w2": ("1", "1"), "staged": ("0", "0")}.items():
        monkeypatch.setenv("SGLM_ETA_PIPE", pipe)
        monkeypatch.setenv("SGLM_ETA3_CFG", c3)
        monkeypatch.setenv("SGLM_ETA_EXACT_STAGED", "1")
        bd = torch.from_numpy(beta).cuda()
        out = torch.full((nb, d.ld), float("nan"), dtype=torch.float32, device="cuda")
        _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, bd.data_ptr(), B,
                  sl.data_ptr(), 1, out.data_ptr(), work.data_ptr(), 0)
        ex[v] = out.cpu().numpy()
    assert np.array_equal(ex["pipe"], ex["staged"], equal_nan=True)
    assert np.array_equal(ex["pipe_w2"], ex["staged"], equal_nan=True)
    monkeypatch.setenv("SGLM_ETA3_CFG", "0")
    X64 = d.xb.double().cpu().numpy()
    for k in slots[:6]:
        ref = beta[k].astype(np.float64) @ X64
        sc = np.abs(beta[k].astype(np.float64)) @ np.abs(X64)
        assert np.max(np.abs(ex["pipe"][k] - ref) / np.maximum(sc, 1e-30)) < 1e-6, k
    X = d.xb.double().cpu().numpy()
    for k in slots[:12]:
        ref = br[k].astype(np.float64) @ X
        sc = np.abs(br[k].astype(np.float64)) @ np.abs(X)
        assert np.max(np.abs(got[k] - ref) / np.maximum(sc, 1e-30)) < 2e-6, k
    untouched = np.setdiff1d(np.arange(nb), slots)
    assert np.isnan(got[untouched]).all()


def test_compact_bits_equals_pack_bits_rows(engine, torch_mod):
    """Compaction from the 1-bit planes == compaction from the bf16 design, bit for bit."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=9000, m=9, L=3, rho=0.15, seed=51)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(52)
    for rows in (np.sort(rng.choice(s.N, 4321, replace=False)).astype(np.int32), None):
        nr = 4321 if rows is not None else s.N
        rows_d = None if rows is None else torch.from_numpy(rows).cuda()
        size = ((nr + 63) // 64) * d.P * 2
        a = torch.zeros(size, dtype=torch.int32, device="cuda")
        b = torch.ones(size, dtype=torch.int32, device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        rp = None if rows_d is None else rows_d.data_ptr()
        _lib.call("sglm_pack_bits_rows", d.xb.data_ptr(), d.ld, d.P, rp, nr, a.data_ptr(),
                  flag.data_ptr(), 0)
        _lib.call("sglm_compact_bits", d.xbits.data_ptr(), d.ld, d.P, rp, nr, b.data_ptr(), 0)
        c = torch.full((size,), 7, dtype=torch.int32, device="cuda")
        _lib.call("sglm_compact_rbits", d.rbits.data_ptr(), d.ld, d.P, rp, nr, c.data_ptr(), 0)
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        assert torch.equal(a, c)          # the ballot transpose of the row-major planes


def test_xtr_bits_matches_float64(engine, torch_mod):
    """MFMA gradient X^T R from compacted bit-planes (R split in 3 bf16 pieces) == float64
    X^T R to f32 accuracy, ragged B; also matches the f32-MFMA sglm_xtr."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=30000, m=11, L=4, rho=0.1, seed=61)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(62)
    B = 45
    R = np.zeros((B, d.ld), np.float32)
    R[:, : s.N] = (rng.standard_normal((B, s.N)) * np.exp(rng.uniform(-6, 3, (B, 1)))).astype(np.float32)
    Rd = torch.from_numpy(R).cuda()
    G = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
    w = torch.empty(_lib.query("sglm_xtr_bits_work_bytes", d.P, B, d.ld), dtype=torch.uint8,
                    device="cuda")
    _lib.call("sglm_xtr_bits", d.cbits_full().data_ptr(), d.ld, d.P, d.n, Rd.data_ptr(), B,
              G.data_ptr(), w.data_ptr(), 0)
    G2 = torch.zeros_like(G)
    w2 = torch.empty(_lib.query("sglm_xtr_work_bytes", d.P, B, d.n), dtype=torch.uint8,
                     device="cuda")
    _lib.call("sglm_xtr", d.xb.data_ptr(), 0, d.ld, d.P, d.n, Rd.data_ptr(), B, G2.data_ptr(),
              w2.data_ptr(), 0)
    X = d.xb.double().cpu().numpy()
    ref = R.astype(np.float64) @ X.T                      # (B, P)
    scale = np.abs(R.astype(np.float64)) @ np.abs(X.T)
    got = G.cpu().numpy()
    assert np.max(np.abs(got - ref) / np.maximum(scale, 1e-30)) < 2e-6
    assert np.max(np.abs(got - G2.cpu().numpy()) / np.maximum(scale, 1e-30)) < 4e-6


def test_fused_link_gradient_and_slot_lists(engine, torch_mod):
    """sglm_link_update writing R as packed bf16 pieces for a slot list, then
    sglm_xtr_bits_packed scattering G to those slots == the unfused path (f32 R, split, X^T R);
    the line-search sums over a slot list == the same rows of the all-slot call (bitwise)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=40000, m=12, L=4, rho=0.08, seed=71)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(72)
    masks = [(rng.random(s.N) < 0.8).astype(np.uint8), np.ones(s.N, np.uint8)]
    prob = engine.Problem(d, [s.y, np.roll(s.y, 7)], masks)
    B = 40
    fr = torch.from_numpy(rng.integers(0, 2, B).astype(np.int32)).cuda()
    fm = torch.from_numpy(rng.integers(0, 2, B).astype(np.int32)).cuda()
    eta = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    eta[:, : s.N] = torch.from_numpy(rng.normal(-1.0, 0.5, (B, s.N)).astype(np.float32))
    W = torch.zeros_like(eta)
    R = torch.zeros_like(eta)
    _lib.call("sglm_link_update", 1, 1.0, d.n, d.ld, B, None, eta.data_ptr(), prob.Y.data_ptr(),
              prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(), W.data_ptr(), R.data_ptr(), None, None,
              None, 0)
    G = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
    w = torch.empty(_lib.query("sglm_xtr_bits_work_bytes", d.P, B, d.ld), dtype=torch.uint8,
                    device="cuda")
    _lib.call("sglm_xtr_bits", d.cbits_full().data_ptr(), d.ld, d.P, d.n, R.data_ptr(), B,
              G.data_ptr(), w.data_ptr(), 0)
    slots = np.array([3, 39, 0, 21, 22, 8, 30], dtype=np.int32)
    sl = torch.from_numpy(slots).cuda()
    ns = len(slots)
    W2 = torch.full_like(W, float("nan"))
    Rp = torch.empty(3 * 32 * d.ld, dtype=torch.bfloat16, device="cuda")
    _lib.call("sglm_link_update", 1, 1.0, d.n, d.ld, ns, sl.data_ptr(), eta.data_ptr(),
              prob.Y.data_ptr(), prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(), W2.data_ptr(),
              None, Rp.data_ptr(), None, None, 0)
    G2 = torch.full_like(G, float("nan"))
    w2 = torch.empty(_lib.query("sglm_xtr_bits_packed_work_bytes", d.P, ns, d.ld),
                     dtype=torch.uint8, device="cuda")
    _lib.call("sglm_xtr_bits_packed", d.cbits_full().data_ptr(), d.ld, d.P, d.n, Rp.data_ptr(),
              ns, sl.data_ptr(), G2.data_ptr(), w2.data_ptr(), 0)
    X = d.xb.double().cpu().numpy()
    scale = np.abs(R.double().cpu().numpy()) @ np.abs(X.T)
    for k in slots:
        assert torch.equal(W2[k], W[k]), k
        err = np.abs(G2[k].cpu().numpy() - G[k].cpu().numpy()) / np.maximum(scale[k], 1e-30)
        assert np.max(err) < 4e-6, k
    assert torch.isnan(G2[1]).all() and torch.isnan(W2[1]).all()
    # line-search sums and drift over a slot list
    deta = torch.zeros_like(eta)
    deta[:, : s.N] = torch.from_numpy(rng.normal(0, 0.1, (B, s.N)).astype(np.float32))
    tv = torch.tensor([0.0, 1.0, 0.5, 0.25, 0.125], dtype=torch.float32, device="cuda")
    wk = torch.empty(_lib.query("sglm_rowsum_work_bytes", B, 8, d.n), dtype=torch.uint8,
                     device="cuda")
    L = torch.zeros(B * 5, dtype=torch.float64, device="cuda")
    dm = torch.zeros(B, dtype=torch.float32, device="cuda")
    _lib.call("sglm_loss_trials_max", 1, 1.0, d.n, d.ld, B, None, eta.data_ptr(), deta.data_ptr(),
              prob.Y.data_ptr(), prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(), tv.data_ptr(), 5,
              L.data_ptr(), dm.data_ptr(), wk.data_ptr(), 0)
    L2 = torch.zeros(ns * 5, dtype=torch.float64, device="cuda")
    dm2 = torch.zeros(ns, dtype=torch.float32, device="cuda")
    _lib.call("sglm_loss_trials_max", 1, 1.0, d.n, d.ld, ns, sl.data_ptr(), eta.data_ptr(),
              deta.data_ptr(), prob.Y.data_ptr(), prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(),
              tv.data_ptr(), 5, L2.data_ptr(), dm2.data_ptr(), wk.data_ptr(), 0)
    Lh, L2h = L.view(B, 5).cpu().numpy(), L2.view(ns, 5).cpu().numpy()
    assert np.array_equal(L2h, Lh[slots]) and np.array_equal(dm2.cpu().numpy(), dm.cpu().numpy()[slots])
    # eta axpy over the slot list
    st = torch.from_numpy(rng.random(ns).astype(np.float32)).cuda()
    e2 = eta.clone()
    _lib.call("sglm_eta_axpy", d.n, d.ld, ns, sl.data_ptr(), st.data_ptr(), deta.data_ptr(),
              e2.data_ptr(), 0)
    for q, k in enumerate(slots):
        # (the kernel may contract to one FMA: compare to f32 rounding)
        assert torch.allclose(e2[k, : s.N], eta[k, : s.N] + st[q] * deta[k, : s.N],
                              rtol=1e-6, atol=1e-7), k
    assert torch.equal(e2[1], eta[1])
    # link with the fused predictor update == axpy, then link
    e3 = eta.clone()
    W3 = torch.zeros_like(W)
    Rp3 = torch.empty_like(Rp)
    _lib.call("sglm_link_update", 1, 1.0, d.n, d.ld, ns, sl.data_ptr(), e3.data_ptr(),
              prob.Y.data_ptr(), prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(), W3.data_ptr(),
              None, Rp3.data_ptr(), st.data_ptr(), deta.data_ptr(), 0)
    W4 = torch.zeros_like(W)
    Rp4 = torch.empty_like(Rp)
    _lib.call("sglm_link_update", 1, 1.0, d.n, d.ld, ns, sl.data_ptr(), e2.data_ptr(),
              prob.Y.data_ptr(), prob.M.data_ptr(), fr.data_ptr(), fm.data_ptr(), W4.data_ptr(),
              None, Rp4.data_ptr(), None, None, 0)
    for k in slots:
        assert torch.equal(e3[k], e2[k]) and torch.equal(W3[k], W4[k]), k
    nb = 3 * 32 * d.ld
    assert torch.equal(Rp3.view(3, 32, d.ld)[:, :ns], Rp4.view(3, 32, d.ld)[:, :ns])


def test_step_scalars_and_update_vs_float64(engine, torch_mod):
    """sglm_step_scalars (g.d, penalty terms, max|d|, max|w + t d| per trial step) and
    sglm_step_update over a slot list vs float64 torch on the same inputs."""
    torch = torch_mod
    from sglm_hip import _lib
    rng = np.random.default_rng(81)
    B, P = 9, 512
    g = torch.from_numpy(rng.normal(size=(B, P))).cuda()
    w = torch.from_numpy(rng.normal(size=(B, P))).cuda()
    d = torch.from_numpy(rng.normal(size=(B, P)).astype(np.float32)).cuda()
    lp = torch.from_numpy(np.abs(rng.normal(size=(B, P)))).cuda()
    t = torch.tensor([0.0, 1.0, 0.5, 0.25, 0.125, 0.0625, 2.0 ** -10], dtype=torch.float64,
                     device="cuda")
    slots = torch.tensor([7, 0, 3, 8], dtype=torch.int32, device="cuda")
    T = t.numel()
    out = torch.empty(4 * (6 + T), dtype=torch.float64, device="cuda")
    _lib.call("sglm_step_scalars", P, P, 4, slots.data_ptr(), g.data_ptr(), w.data_ptr(),
              d.data_ptr(), lp.data_ptr(), t.data_ptr(), T, out.data_ptr(), 0)
    o = out.view(4, 6 + T).cpu().numpy()
    nc = 300                                   # max|w + t d| over the first ncoef only
    out2 = torch.empty_like(out)
    _lib.call("sglm_step_scalars", P, nc, 4, slots.data_ptr(), g.data_ptr(), w.data_ptr(),
              d.data_ptr(), lp.data_ptr(), t.data_ptr(), T, out2.data_ptr(), 0)
    o2 = out2.view(4, 6 + T).cpu().numpy()
    for q, k in enumerate((7, 0, 3, 8)):
        dk = d[k, :nc].double()
        assert np.allclose(o2[q, 5:5 + T], [float((w[k, :nc] + tj * dk).abs().max())
                                            for tj in t.tolist()], rtol=1e-12, atol=1e-12)
        assert np.array_equal(o2[q, :4], o[q, :4])
        assert o2[q, 4] == float(dk.abs().max())
        assert o2[q, 5 + T] == float(d[k, nc:].double().abs().max())
    for q, k in enumerate((7, 0, 3, 8)):
        dk = d[k].double()
        ref = [float((g[k] * dk).sum()), float((lp[k] * w[k] * w[k]).sum()),
               float((lp[k] * w[k] * dk).sum()), float((lp[k] * dk * dk).sum()),
               float(dk.abs().max())] + [float((w[k] + tj * dk).abs().max()) for tj in t.tolist()] \
            + [0.0]
        assert np.allclose(o[q], ref, rtol=1e-12, atol=1e-12), (k, o[q], ref)
    step = torch.tensor([0.5, 0.0, 1.0, 0.25], dtype=torch.float64, device="cuda")
    w2 = w.clone()
    _lib.call("sglm_step_update", P, 4, slots.data_ptr(), step.data_ptr(), d.data_ptr(),
              w2.data_ptr(), 0)
    for q, k in enumerate((7, 0, 3, 8)):
        assert torch.allclose(w2[k], w[k] + step[q] * d[k].double(), rtol=0, atol=1e-15)
    assert torch.equal(w2[1], w[1])


@pytest.mark.parametrize("m,L,event_major,N", [(50, 20, False, 200_001), (7, 3, True, 13_000),
                                               (17, 9, False, 6_144), (3, 1, False, 100)])
def test_lag_xtr_vs_float64(engine, m, L, event_major, N):
    """sglm_lag_xtr (X^T R from the event occurrences of a time-shifted design) against
    float64 torch on the dense expansion: both layouts, m over and under 16 events (the two
    register-accumulator variants), sizes off and on the tile boundary, a slot subset."""
    import torch
    from sglm_hip import _lib, engine as E, synth
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.05, seed=m + N)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, event_major=event_major)
    assert d.lag is not None
    Xd = d.xb[: d.p + 1, : d.n].double().t().contiguous()           # dense (n, p + 1)
    B = 9
    rng = np.random.default_rng(3)
    R = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    R[:, : d.n] = torch.from_numpy(rng.normal(size=(B, d.n)).astype(np.float32)).cuda()
    slots = torch.tensor([8, 0, 5, 3], dtype=torch.int32, device="cuda")
    g = torch.full((B, d.P), 7.0, dtype=torch.float64, device="cuda")
    lg = d.lag
    work = torch.empty(_lib.query("sglm_lag_xtr_work_bytes", d.P, lg.K, B, d.n),
                       dtype=torch.uint8, device="cuda")
    _lib.call("sglm_lag_xtr", lg.occ.data_ptr(), lg.tbeg.data_ptr(), lg.tend.data_ptr(),
              lg.shifts.data_ptr(), lg.m, lg.K, lg.layout, lg.row0, d.n, d.P, R.data_ptr(),
              d.ld, slots.data_ptr(), 4, g.data_ptr(), work.data_ptr(), 0)
    got = g.cpu().numpy()
    for k in (8, 0, 5, 3):
        ref = (Xd.t() @ R[k, : d.n].double()).cpu().numpy()
        np.testing.assert_allclose(got[k, : d.p + 1], ref, rtol=1e-12, atol=1e-9)
        assert np.all(got[k, d.p + 1:] == 0)
    for k in (1, 2, 4, 6, 7):
        assert np.all(got[k] == 7.0)                                   # untouched slots


@pytest.mark.parametrize("B,ngw", [(45, "2"), (7, "1"), (120, "2"), (70, "1"), (70, "2"),
                                   (120, "1")])
def test_xtr_bits_four_panel_kernel_vs_float64(engine, torch_mod, B, ngw, monkeypatch):
    """The four-panel gradient kernel (xtr_bits4_kernel, R staged in LDS for 512 predictors,
    one or two 32-fit groups per workgroup, forced by SGLM_XTR_NGW; P % 512 == 0) against
    float64 X^T R, ragged fit counts and a half-empty last workgroup (70 fits, two groups)."""
    torch = torch_mod
    monkeypatch.setenv("SGLM_XTR_NGW", ngw)
    monkeypatch.setenv("SGLM_XTR_PIPE", "0")        # xtr_bits4_kernel first (the reference)
    from sglm_hip import _lib, synth
    s = synth.make(N=40_000, m=50, L=5, rho=0.05, seed=B)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    assert d.P % 512 == 0
    rng = np.random.default_rng(B)
    R = np.zeros((B, d.ld), np.float32)
    R[:, : s.N] = (rng.standard_normal((B, s.N)) * np.exp(rng.uniform(-6, 3, (B, 1)))).astype(np.float32)
    Rd = torch.from_numpy(R).cuda()
    G = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
    w = torch.empty(_lib.query("sglm_xtr_bits_work_bytes", d.P, B, d.ld), dtype=torch.uint8,
                    device="cuda")
    _lib.call("sglm_xtr_bits", d.cbits_full().data_ptr(), d.ld, d.P, d.n, Rd.data_ptr(), B,
              G.data_ptr(), w.data_ptr(), 0)
    X = d.xb.double()
    ref = (Rd.double() @ X.t()).cpu().numpy()
    scale = (Rd.double().abs() @ X.abs().t()).cpu().numpy()
    assert np.max(np.abs(G.cpu().numpy() - ref) / np.maximum(scale, 1e-30)) < 2e-6
    # the software-pipelined kernel (xtr_bits5_kernel): the same MFMA sequence per wave, so
    # the same partial sums bit for bit; also on the two-wave one-group variant
    for pipe_env in ({"SGLM_XTR_PIPE": "1"}, {"SGLM_XTR_PIPE": "1", "SGLM_XTR_NGW": "3"},
                     {"SGLM_XTR_PIPE": "1", "SGLM_XTR_NGW": "1"}):
        for k, v in pipe_env.items():
            monkeypatch.setenv(k, v)
        G2 = torch.zeros_like(G)
        _lib.call("sglm_xtr_bits", d.cbits_full().data_ptr(), d.ld, d.P, d.n, Rd.data_ptr(), B,
                  G2.data_ptr(), w.data_ptr(), 0)
        if pipe_env.get("SGLM_XTR_NGW", ngw) != ngw:
            assert np.max(np.abs(G2.cpu().numpy() - ref) / np.maximum(scale, 1e-30)) < 2e-6
        else:
            assert torch.equal(G2, G), pipe_env


@pytest.mark.parametrize("shifts,event_major,row0,slab", [
    (list(range(-5, 10)), False, 9, None),          # contiguous lags, shift-major
    ([0, 2, 3, 7, -4], True, 7, None),              # scattered lags, event-major
    (list(range(0, 40)), False, 0, None),           # rows past the start of E (zero)
    (list(range(-3, 12)), False, 11, (3000, 11000)),  # a row slab of a row-sharded solve
])
def test_lag_gram_equals_the_dense_gram(engine, torch_mod, shifts, event_major, row0, slab):
    """sglm_lag_gram (event cross-correlations) against the float64 X^T X of the expanded
    design: bf16(w) * count exactly on the 128-blocks I <= J of every listed fit, other fits and
    the lower blocks untouched."""
    torch = torch_mod
    from sglm_hip import _lib
    E_ = engine
    rng = np.random.default_rng(len(shifts) + row0)
    n_raw, m = 12_000, 7
    Ev = (rng.random((n_raw, m)) < 0.05).astype(np.float32)
    Ev[:40, 2] = 1.0                                 # occurrences at both ends of the window
    Ev[-40:, 5] = 1.0
    n = n_raw - (max(shifts) - min(shifts)) - 3
    d = E_.Design.from_events(Ev, shifts, row0, n, event_major=event_major, slab=slab)
    assert d.lag is not None and d.lag.ebits is not None
    nloc = d.n
    X = d.xb[:, :nloc].double()
    G = (X @ X.t()).cpu().numpy()
    B, P = 3, d.P
    W = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    W[:, 0] = torch.tensor([0.7318, 1.0, 2.5e-3])
    H = torch.full((B, P, P), float("nan"), dtype=torch.float32, device="cuda")
    fits = torch.tensor([0, 2], dtype=torch.int32, device="cuda")
    lg = d.lag
    work = torch.empty(_lib.query("sglm_lag_gram_work_bytes", lg.m, lg.smin, lg.smax),
                       dtype=torch.uint8, device="cuda")
    _lib.call("sglm_lag_gram", lg.occ.data_ptr(), lg.ev_off.data_ptr(), lg.ebits.data_ptr(),
              lg.nwords, lg.shifts.data_ptr(), lg.m, lg.K, lg.layout, lg.smin, lg.smax, lg.row0,
              lg.n, lg.n_raw, P, W.data_ptr(), d.ld, fits.data_ptr(), 2, H.data_ptr(),
              work.data_ptr(), 0)
    torch.cuda.synchronize()
    Hh = H.cpu().numpy()
    blk = np.arange(P) // 128
    upper = blk[:, None] <= blk[None, :]
    for k in (0, 2):
        w = np.float32(torch.tensor(float(W[k, 0])).to(torch.bfloat16).float().item())
        want = (w * G.astype(np.float32)).astype(np.float32)
        assert np.array_equal(Hh[k][upper], want[upper]), k
        assert np.isnan(Hh[k][~upper]).all()
    assert np.isnan(Hh[1]).all()


def test_grid_first_gram_from_event_correlations(engine):
    """The C3-shape grid takes its first (constant-weight) Gram from sglm_lag_gram and reaches
    the same fits as with the MFMA Gram (the first Hessian differs only by f32 rounding; the
    fixed point is the exact gradient's)."""
    import pandas as pd
    from sglm_hip import folds, grid, synth
    from sglm_hip.estimators import Objective
    E_ = engine
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    d = E_.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    objs = [Objective("irls", E_.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100)
            for a in np.logspace(-4, 1, 6)]
    st = E_.IrlsStats()
    a = grid.run(d, s.y, cv_idx, objs, [0] * 6, stats=st)
    assert st.lag_grams >= 1
    old = E_.LAG_GRAM
    try:
        E_.LAG_GRAM = False
        st2 = E_.IrlsStats()
        b = grid.run(d, s.y, cv_idx, objs, [0] * 6, stats=st2)
        assert st2.lag_grams == 0
    finally:
        E_.LAG_GRAM = old
    for x, y in zip(a, b):
        assert x["converged"] and y["converged"]
        assert rel(x["cv_coefs"], y["cv_coefs"]) < 1e-5
        assert rel(x["refit_coef"], y["refit_coef"]) < 1e-5


def test_lag_gram_only_for_constant_weights(engine):
    """Gamma / Tweedie weights carry y on every row (h = y e^-eta for power 2) even at a
    constant eta: their first Gram must stay the MFMA Gram over the rows."""
    import pandas as pd
    from sglm_hip import folds, grid, synth
    from sglm_hip.estimators import Objective
    E_ = engine
    s = synth.make(N=50_000, m=10, L=8, family="poisson", rho=0.05, seed=4)
    y = s.y + 0.5                                        # strictly positive (Gamma's range)
    d = E_.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(5)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=3)
    for power in (2.0, 1.5):
        objs = [Objective("irls", E_.FAM_TWEEDIE_LOG, power, float(a), "n", True, 100)
                for a in (1e-3, 1e-1)]
        st = E_.IrlsStats()
        a = grid.run(d, y, cv_idx, objs, [0, 0], stats=st)
        assert st.lag_grams == 0, power
        assert all(r["converged"] for r in a)


def test_grid_bad_fold_index_raises_index_error(engine):
    """A fold list naming a row outside [-n, n) raises IndexError, as the reference's
    X[idx_train] does (the mask builder checks it when the grid is one process)."""
    from sglm_hip import grid, synth
    from sglm_hip.estimators import Objective
    E_ = engine
    s = synth.make(N=5_000, m=4, L=3, family="poisson", rho=0.05, seed=2)
    d = E_.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    tr = np.arange(0, 4000)
    te = np.arange(4000, s.N + 1)                       # one past the last row
    objs = [Objective("irls", E_.FAM_TWEEDIE_LOG, 1.0, 1e-2, "n", True, 100)]
    with pytest.raises(IndexError):
        grid.run(d, s.y, [(tr, te)], objs, [0])


@pytest.mark.parametrize("B,lim", [(45, 128), (130, 256), (7, 128)])
def test_xtr_bits_int_exact(engine, torch_mod, B, lim):
    """sglm_xtr_bits_int (one bf16 piece, the digit planes of an exact X^T y) equals the float64
    X^T D exactly for integer columns |d| <= lim (one, two and four 32-column groups per
    workgroup), and sglm_digit_planes writes the balanced base-256 digits of rint(m y s)."""
    torch = torch_mod
    from sglm_hip import _lib, synth
    s = synth.make(N=70_000, m=50, L=10, rho=0.05, seed=B)
    d = engine.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    assert d.P % 512 == 0 and d.xtr_int_ok()
    rng = np.random.default_rng(B)
    Bp = (B + 31) // 32 * 32
    D = np.zeros((Bp, d.ld), np.float32)
    D[:B, : s.N] = rng.integers(-lim, lim + 1, (B, s.N))
    Dd = torch.from_numpy(D).cuda().to(torch.bfloat16)
    G = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
    d.xtr_int(Dd, B, G)
    X = d.xb.double()
    ref = (torch.from_numpy(D[:B]).cuda().double() @ X.t()).cpu().numpy()
    assert np.array_equal(G.cpu().numpy(), ref)
    # digit planes: 3 pairs (response, mask) with a multiplicity mask
    R, F = 2, 2
    Y = rng.normal(size=(R, s.N)) * np.array([[1.0], [1e3]])
    M = np.zeros((F, d.ld), np.uint8)
    M[0, : s.N] = rng.integers(0, 2, s.N)
    M[1, : s.N] = rng.integers(0, 3, s.N)
    Yd, Md = torch.from_numpy(Y).cuda(), torch.from_numpy(M).cuda()
    pr = torch.tensor([0, 1, 1], dtype=torch.int32, device="cuda")
    pm = torch.tensor([1, 0, 1], dtype=torch.int32, device="cuda")
    sc = torch.tensor([2.0 ** 30, 2.0 ** 20, 2.0 ** 21], dtype=torch.float64, device="cuda")
    nd = 5
    Dp = torch.zeros((32, d.ld), dtype=torch.bfloat16, device="cuda")
    _lib.call("sglm_digit_planes", Md.data_ptr(), d.ld, Yd.data_ptr(), s.N, s.N, pr.data_ptr(),
              pm.data_ptr(), sc.data_ptr(), 3, nd, Dp.data_ptr(), d.ld, 0)
    got = Dp.float().cpu().numpy()
    for i, (r, m) in enumerate(((0, 1), (1, 0), (1, 1))):
        v = np.rint(M[m, : s.N].astype(np.float64) * Y[r] * float(sc[i])).astype(np.int64)
        for q in range(nd):
            dq = np.mod(v + 128, 256) - 128
            assert np.array_equal(got[q * 3 + i, : s.N], dq.astype(np.float32)), (i, q)
            v = (v - dq) // 256
        assert np.all(v == 0)
        assert np.all(got[:, s.N:] == 0)


@pytest.mark.parametrize("m,L,event_major,N,row0_off", [(50, 20, False, 200_003, 0),
                                                       (7, 3, True, 13_000, 2),
                                                       (70, 4, False, 9_000, 0)])
def test_lag_bits_equal_packed_dense_design(engine, monkeypatch, m, L, event_major, N, row0_off):
    """The bit-planes built straight from the events (sglm_event_bits + sglm_lag_bits) equal the
    ones packed from the dense bf16 design (sglm_pack_bits / _pack_bits_t), the occurrence
    bitmaps equal LagStructure's, and the lazily built dense design equals the eager one; also
    a design whose row window reaches past the events' first rows (zero fill) and m > 64 (no
    LagStructure)."""
    import torch
    from sglm_hip import synth
    E_ = engine
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.05, seed=m + N)
    row0 = s.L - 1 - row0_off
    n = s.N - 1
    designs = {}
    for lb in (False, True):
        monkeypatch.setattr(E_, "LAG_BITS", lb)
        designs[lb] = E_.Design.from_events(s.E, s.shifts, row0, n, event_major=event_major)
    a, b = designs[False], designs[True]
    assert b._xb is None                               # no dense copy built yet
    assert torch.equal(a.xbits, b.xbits)
    assert torch.equal(a.rbits, b.rbits)
    if a.lag is not None:
        assert b.lag is not None and torch.equal(a.lag.ebits, b.lag.ebits)
        # the occurrence bitmaps against numpy: bit u & 31 of word u >> 5 = (E[u, a] != 0)
        nw = a.lag.nwords
        nz = np.zeros((m, nw * 32), dtype=np.uint8)
        nz[:, : s.E.shape[0]] = (np.asarray(s.E) != 0).T
        ref = np.packbits(nz, axis=1, bitorder="little").view("<u4").view(np.int32)
        assert np.array_equal(b.lag.ebits.cpu().numpy(), ref)
    else:
        assert b.lag is None
    assert torch.equal(a.xb, b.xb)                     # built on first use
    assert torch.equal(a.cbits_full(), b.cbits_full())
