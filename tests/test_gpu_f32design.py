"""All-real designs beyond the mixed budget on the MI355X (round 6).

A design whose non-binary columns are too many for the float64 continuous block
(n k(k+1)/2 > MIXED_BUDGET products per Gram -- z-scored or differenced columns,
backend/sglm_pp.py:105-190, at session scale) is kept as ONE f32 matrix: the Gram on f32 MFMA
(syrk_f32_kernel), gradient and eta on f32 MFMA, rank decisions on the f32 factor at
RANK_TOL_F32.  The budget is lowered here so that a 200k-row design takes that path, and the
fits through the drop-in API are held to the float64 oracle at the north star's bars (1e-5
Gaussian, 1e-4 Poisson, relative) on the f32-rounded design -- the data that path fits.
"""
import numpy as np
import pytest

from oracle import glm_ref

pytestmark = pytest.mark.gpu
TOL_POIS, TOL_GAUSS = 1e-4, 1e-5


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _design(n=200_000, k=80, seed=21):
    """k z-scored continuous columns (a smooth signal and its lagged differences, as
    sglm_pp.zscore / diff make them) beside ten 0/1 event columns."""
    rng = np.random.default_rng(seed)
    sig = np.cumsum(rng.normal(size=(n, k // 2)), axis=0)
    dif = np.vstack([np.zeros((1, k // 2)), np.diff(sig, axis=0)])
    C = np.hstack([sig, dif])
    C = (C - C.mean(0)) / C.std(0)
    E = (rng.random((n, 10)) < 0.05).astype(np.float64)
    X = np.hstack([C, E]).astype(np.float32).astype(np.float64)     # the f32-exact data
    beta = rng.normal(0, 0.05, X.shape[1])
    return X, beta, rng


def test_f32_design_path_taken(engine, monkeypatch):
    monkeypatch.setattr(engine, "MIXED_BUDGET", 1e6)
    X, _, _ = _design(n=20_000)
    d = engine.Design.from_host(X)
    assert d.xf is not None and d.cont is None          # one f32 matrix, no float64 block
    monkeypatch.setattr(engine, "MIXED_BUDGET", 1e12)
    d2 = engine.Design.from_host(X)
    assert d2.xf is None and d2.cont is not None         # within budget: the mixed design


def test_f32_design_ols_and_poisson_vs_oracle(engine, monkeypatch):
    import sglm
    monkeypatch.setattr(engine, "MIXED_BUDGET", 1e6)
    X, beta, rng = _design()
    y = X @ beta + 0.3 + rng.normal(0, 0.5, X.shape[0])
    glm = sglm.GLM("Normal", alpha=0)
    glm.fit(X, y)
    c, b = glm_ref.fit_ols(X, y)
    assert rel(np.r_[glm.coef_, glm.intercept_], np.r_[c, b]) < TOL_GAUSS
    yp = rng.poisson(np.exp(X @ (0.3 * beta) - 0.5)).astype(np.float64)
    for alpha in (1e-3, 0.1):
        glm = sglm.GLM("Poisson", alpha=alpha)
        glm.fit(X, yp)
        c, b = glm_ref.fit_tweedie_newton(X, yp, alpha, 1.0)
        assert rel(np.r_[glm.coef_, glm.intercept_], np.r_[c, b]) < TOL_POIS, alpha


def test_f32_design_cv_grid_vs_oracle(engine, monkeypatch):
    """A 3-split Poisson grid through sglm_cv.cv_glm_mult_params on the f32 design: every
    split fit, the refit and the fold scores against the oracle's grid (cv_ref.cv_mult)."""
    import sglm_cv
    from oracle import cv_ref
    monkeypatch.setattr(engine, "MIXED_BUDGET", 1e6)
    X, beta, rng = _design(n=60_000, k=40)
    y = rng.poisson(np.exp(X @ (0.3 * beta) - 0.5)).astype(np.float64)
    idx = np.arange(X.shape[0])
    cv_idx = []
    for s in range(3):
        test = (idx // 100) % 3 == s
        cv_idx.append((idx[~test], idx[test]))
    kws = sglm_cv.generate_mult_params({"alpha": [0.01, 0.3]}, {"model_name": "Poisson"})
    ref_kws = [dict(k) for k in kws]
    out = sglm_cv.cv_glm_mult_params(X, y, cv_idx, "Normal", kws)
    ref = cv_ref.cv_mult(X, y, cv_idx, ref_kws)
    for r, q in zip(out["full_cv_results"], ref["full_cv_results"]):
        assert rel(r["cv_coefs"], q["cv_coefs"]) < TOL_POIS, r["glm_kwargs"]
        assert rel(r["cv_intercepts"], q["cv_intercepts"]) < TOL_POIS
        assert rel(r["model"].coef_, q["coef"]) < TOL_POIS
        assert np.max(np.abs(r["cv_scores_test"] - q["cv_scores_test"])) < 1e-6
