"""Rank-deficient and ill-conditioned unpenalised fits on the MI355X (round 4).

The reference's OLS is LinearRegression -> scipy lstsq (backend/sglm.py:96-101 -> sklearn
_base.py:701): float64, minimum-norm coefficients on a rank-deficient design.  Its unpenalised
Poisson is TweedieRegressor(alpha=0) lbfgs from w = 0 (backend/sglm.py:112-115), which stays in
the row space of X (duplicated columns share the weight).  The engine decides dependence on the
float64 factor of the exact mask Gram (sglm_chol64_factor), solves squared-loss fits on float64
factors, and projects unpenalised fits onto the minimum-norm point (sglm_chol64_minnorm).

Bars: coefficients 1e-5 relative (Gaussian) / 1e-4 (Poisson) of the sklearn goldens in
tests/golden/rank.npz and fits.npz (made by tests/golden/make_golden.py).
"""
import numpy as np
import pytest

from test_oracle_golden import rank_design
from oracle import glm_ref

pytestmark = pytest.mark.gpu
TOL_POIS, TOL_GAUSS = 1e-4, 1e-5


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _chol64(H32, dshift, lamp, tol):
    """Run sglm_chol64_factor on host matrices (f32 upper triangles) -> (U, state, nulls,
    counts) as numpy."""
    import torch
    from sglm_hip import _lib
    nf, P, _ = H32.shape
    dev = "cuda"
    H = torch.from_numpy(np.ascontiguousarray(H32, dtype=np.float32)).to(dev)
    ds = torch.from_numpy(np.ascontiguousarray(dshift, dtype=np.float32)).to(dev)
    lp = torch.from_numpy(np.ascontiguousarray(lamp, dtype=np.float64)).to(dev)
    idx = torch.arange(nf, dtype=torch.int32, device=dev)
    U = torch.empty((nf, P, P), dtype=torch.float64, device=dev)
    st = torch.empty((nf, P), dtype=torch.uint8, device=dev)
    nulls = torch.empty((nf, P), dtype=torch.int32, device=dev)
    counts = torch.empty((nf, 2), dtype=torch.int32, device=dev)
    work = torch.empty(_lib.query("sglm_chol64_work_bytes", P, nf), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("sglm_chol64_factor", H.data_ptr(), P, idx.data_ptr(), ds.data_ptr(),
              lp.data_ptr(), idx.data_ptr(), nf, tol, U.data_ptr(), st.data_ptr(),
              nulls.data_ptr(), counts.data_ptr(), work.data_ptr(), s)
    return H, ds, U, st, nulls, counts, idx


@pytest.mark.parametrize("P", [128, 2048])
def test_chol64_kernels_vs_numpy(engine, P):
    """Dependent, zero and excluded coordinates (one duplicate pair straddling a 64-block edge,
    one combination of three columns, one all-zero column, an excluded coordinate), and a
    ridge-shifted full-rank factor: the dependent set is found exactly, the float64 solve equals
    numpy's on the kept coordinates, and the min-norm projection equals the pseudo-inverse
    solution."""
    import torch
    from sglm_hip import _lib
    rng = np.random.default_rng(P)
    p = P - 7                                  # pad coordinates p+1 .. P-1 are excluded
    n = 3 * P
    X = (rng.random((n, p)) < 0.2).astype(np.float64)
    X[:, 63] = X[:, 70]                        # 70 depends on 63 (later pivot is dropped)
    X[:, 100] = X[:, 3] + X[:, 5]          # 100 = 3 + 5 (integer combination)
    X[:, 40] = 0.0
    Xa = np.hstack([X, np.ones((n, 1))])
    G = Xa.T @ Xa
    H = np.zeros((2, P, P), np.float32)
    for f in range(2):
        H[f, :p + 1, :p + 1] = G
    dshift = np.full((2, P), -1.0, np.float32)
    dshift[:, :p + 1] = 0.0
    dshift[0, 20] = -1.0                       # excluded coordinate in factor 0
    lamp = np.zeros((2, P))
    lamp[1, :p] = 2.5                          # factor 1: ridge, full rank
    H_d, ds, U, st, nulls, counts, idx = _chol64(H, dshift, lamp, 1e-9)
    st_h, cnt = st.cpu().numpy(), counts.cpu().numpy()
    dep = np.flatnonzero(st_h[0] == 1)
    assert list(dep) == [70, 100], dep
    assert st_h[0, 40] == 3 and st_h[0, 20] == 2 and np.all(st_h[0, p + 1:] == 2)
    assert cnt[0].tolist() == [2, 3] and cnt[1].tolist() == [0, 0]
    assert np.all(st_h[1, :p + 1] == 0)
    # solve: both factors, two right-hand sides each
    g = np.zeros((4, P))
    g[:, :p + 1] = rng.normal(size=(4, p + 1))
    gd = torch.from_numpy(g).cuda()
    delta = torch.zeros((4, P), dtype=torch.float32, device="cuda")
    fits = torch.arange(4, dtype=torch.int32, device="cuda")
    fsrc = torch.tensor([0, 0, 1, 1], dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.call("sglm_chol64_solve", U.data_ptr(), P, st.data_ptr(), fits.data_ptr(),
              fsrc.data_ptr(), 4, gd.data_ptr(), delta.data_ptr(), s)
    dl = delta.cpu().numpy().astype(np.float64)
    keep = np.flatnonzero(st_h[0] == 0)
    A = G[np.ix_(keep, keep)]
    for q in range(2):
        ref = -np.linalg.solve(A, g[q, keep])
        assert rel(dl[q, keep], ref) < 1e-6
        assert np.all(dl[q, np.setdiff1d(np.arange(P), keep)] == 0.0)
    A1 = G + np.diag(np.r_[np.full(p, 2.5), 0.0])
    for q in (2, 3):
        ref = -np.linalg.solve(A1, g[q, :p + 1])
        assert rel(dl[q, :p + 1], ref) < 1e-6
    # min-norm projection of a kept-coordinate solution of factor 0 (w_dep = 0)
    y = Xa[:, keep] @ rng.normal(size=keep.size) + rng.normal(size=n)
    sol = np.zeros(P)
    sol[keep] = np.linalg.lstsq(Xa[:, keep], y, rcond=None)[0]
    beta = torch.from_numpy(sol[None, :].copy()).cuda()
    work = torch.empty(_lib.query("sglm_chol64_minnorm_work_bytes", P, 2), dtype=torch.uint8,
                       device="cuda")
    f0 = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.call("sglm_chol64_minnorm", U.data_ptr(), P, p, st.data_ptr(), nulls.data_ptr(),
              counts.data_ptr(), 2, f0.data_ptr(), f0.data_ptr(), 1, beta.data_ptr(),
              work.data_ptr(), s)
    got = beta.cpu().numpy()[0]
    # reference: lstsq (min-norm over the coefficients, intercept free) without column 20
    cols = np.array([j for j in range(p + 1) if j != 20])
    Xr = Xa[:, cols]
    c_ref, _ = glm_ref.fit_ols(Xr[:, :-1], y)
    b_ref = float(np.mean(y - Xr[:, :-1] @ c_ref))
    assert rel(got[cols[:-1]], c_ref) < 1e-8
    assert abs(got[p] - b_ref) < 1e-8 * max(1.0, abs(b_ref))
    assert abs(got[63] - got[70]) < 1e-10 and got[40] == 0.0 and got[20] == 0.0


def test_duplicated_event_lag_design_ols(engine, golden):
    """C1 shape (10k x 100 lag design): event 9 duplicates event 2 (ten dependent lag columns),
    event 5 never occurs (ten zero columns) -> sklearn LinearRegression, coefficients and
    intercept at 1e-5, duplicated lags split equally."""
    import sglm
    g = golden("rank.npz")
    X, y = rank_design(g, "dup"), g["dup_y"]
    glm = sglm.GLM("Normal", alpha=0, l1_ratio=0)
    glm.fit(X, y)
    assert rel(glm.coef_, g["dup_coef"]) < TOL_GAUSS
    assert abs(glm.intercept_ - float(g["dup_b"])) < TOL_GAUSS * max(1, abs(float(g["dup_b"])))
    for bi in range(10):
        assert abs(glm.coef_[bi * 10 + 2] - glm.coef_[bi * 10 + 9]) < 1e-9
        assert glm.coef_[bi * 10 + 5] == 0.0


def test_ill_conditioned_full_rank_ols(engine, golden):
    """A full-rank 0/1 lag design with cond(X~^T X~) ~ 7e6 (two state indicators differing on
    one row, lags -15..14, 100k rows): no coefficient is dropped and the fit equals sklearn
    LinearRegression at 1e-5."""
    import sglm
    g = golden("rank.npz")
    X, y = rank_design(g, "ill"), g["ill_y"]
    assert 1e6 < float(g["ill_cond"]) < 1e8
    glm = sglm.GLM("Normal", alpha=0)
    glm.fit(X, y)
    assert rel(glm.coef_, g["ill_coef"]) < TOL_GAUSS
    assert abs(glm.intercept_ - float(g["ill_b"])) < TOL_GAUSS * max(1, abs(float(g["ill_b"])))


def test_poisson_alpha0_duplicate_column(engine, golden):
    """Unpenalised Poisson with a duplicated column: sklearn lbfgs from 0 (tol 1e-12) keeps the
    pair equal; the engine's minimum-norm point matches at 1e-4."""
    import sglm
    g = golden("rank.npz")
    X, y = rank_design(g, "pdup"), g["pdup_y"]
    glm = sglm.GLM("Poisson", alpha=0.0)
    glm.fit(X, y)
    assert rel(glm.coef_, g["pdup_coef"]) < TOL_POIS
    assert abs(glm.intercept_ - float(g["pdup_b"])) < TOL_POIS * max(1, abs(float(g["pdup_b"])))
    assert abs(glm.coef_[5] - glm.coef_[-1]) < 1e-8


def test_ols_grid_rank_deficient_folds_vs_oracle(engine, golden):
    """The CV grid with alpha = 0 on the duplicated-event design: every split fit and refit
    is the minimum-norm lstsq solution of its own rows (oracle glm_ref.fit_ols on X[train])."""
    import sglm_cv
    from oracle import folds_ref
    g = golden("rank.npz")
    X, y = rank_design(g, "dup"), g["dup_y"]
    trial = np.arange(X.shape[0]) // 100
    np.random.seed(3)
    cv_idx = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([trial]), num_folds=3)
    kws = [{"alpha": 0.0, "l1_ratio": 0.0}, {"alpha": 0.0, "l1_ratio": 0.0, "roll": 2}]
    out = sglm_cv.cv_glm_mult_params(X, y, cv_idx, "Normal", kws, score_method="r2")
    for j, r in enumerate(out["full_cv_results"]):
        yy = np.roll(y, 2) if j == 1 else y
        for k, (tr, te) in enumerate(cv_idx):
            c, b = glm_ref.fit_ols(X[tr], yy[tr])
            assert rel(r["cv_coefs"][:, k], c) < TOL_GAUSS, (j, k)
            assert abs(r["cv_intercepts"][k] - b) < TOL_GAUSS * max(1.0, abs(b))
        c, b = glm_ref.fit_ols(X, y)
        assert rel(r["model"].coef_, c) < TOL_GAUSS
