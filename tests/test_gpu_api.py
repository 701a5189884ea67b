"""Drop-in API (sglm / sglm_cv / sglm_ez / sglm_pp) on the MI355X vs golden fixtures & oracle.

Tolerances (BASELINE.json north star): coefficients within 1e-4 relative (Poisson / Gamma)
and 1e-5 relative (Gaussian) of the tight-tolerance sklearn minimiser; fold indices and
timeshift outputs bit-exact.  Relative error = max|a - b| / max|b| over the vector.
"""
import json
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN
from oracle import cv_ref, folds_ref, glm_ref, pp_ref

pytestmark = pytest.mark.gpu
TOL_POIS, TOL_GAUSS = 1e-4, 1e-5


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_glm_all_families_vs_golden(engine, golden):
    import sglm
    g = golden("fits.npz")
    meta = json.load(open(os.path.join(GOLDEN, "fits_meta.json")))
    for m in meta:
        glm = sglm.GLM("Poisson", alpha=m["alpha"], fit_intercept=m["fit_intercept"])
        glm.fit(g["pois_X"], g["pois_y"])
        assert rel(glm.coef_, g[m["key"] + "_coef"]) < TOL_POIS, m
        assert glm.beta_ is glm.coef_ and glm.beta0_ == glm.intercept_
    glm = sglm.GLM("Gamma", alpha=0.05)
    glm.fit(g["gam_X"], g["gam_y"])
    assert rel(glm.coef_, g["gam_coef"]) < TOL_POIS
    X, y = g["gau_X"], g["gau_y"]
    glm = sglm.GLM("Normal", alpha=0, l1_ratio=0, max_iter=1000)
    glm.fit(X, y)
    assert rel(glm.coef_, g["ols_coef"]) < TOL_GAUSS
    for i, a in enumerate([0.1, 10.0, 1000.0]):
        glm = sglm.GLM("Gaussian", alpha=a, l1_ratio=0)
        glm.fit(X, y)
        assert rel(glm.coef_, g[f"ridge_a{i}_coef"]) < TOL_GAUSS
    for i, a in enumerate([1e-3, 1e-2]):
        glm = sglm.GLM("Gaussian", alpha=a, l1_ratio=1)
        glm.fit(X, y)
        assert rel(glm.coef_, g[f"lasso_a{i}_coef"]) < TOL_GAUSS, a
        glm = sglm.GLM("Gaussian", alpha=a, l1_ratio=0.5)
        glm.fit(X, y)
        assert rel(glm.coef_, g[f"enet_a{i}_coef"]) < TOL_GAUSS, a
        assert abs(glm.intercept_ - float(g[f"enet_a{i}_b"])) < 1e-5 * max(1, abs(float(g[f"enet_a{i}_b"])))


def test_glm_rank_deficient_ols(engine, golden):
    """Duplicate + all-zero column, alpha = 0: the COEFFICIENTS equal lstsq's minimum-norm
    solution (sklearn _base.py:701; the duplicated pair splits the weight equally), the zero
    column's coefficient is 0, and the fitted values match."""
    import sglm
    g = golden("fits.npz")
    X, y = g["olsr_X"], g["gau_y"]
    glm = sglm.GLM("Normal", alpha=0)
    glm.fit(X, y)
    assert rel(glm.coef_, g["olsr_coef"]) < TOL_GAUSS
    assert abs(glm.intercept_ - float(g["olsr_b"])) < TOL_GAUSS * max(1, abs(float(g["olsr_b"])))
    assert glm.coef_[7] == 0.0
    assert abs(glm.coef_[2] - glm.coef_[6]) < 1e-9
    pred_ref = X @ g["olsr_coef"] + float(g["olsr_b"])
    assert rel(glm.predict(X), pred_ref) < 1e-5


def test_glm_scores_and_residuals(engine, golden):
    import sglm
    g = golden("fits.npz")
    X, y = g["pois_X"], g["pois_y"]
    glm = sglm.GLM("Poisson", alpha=0.1, score_method="r2")
    glm.fit(X, y)
    spec = glm_ref.FitSpec("tweedie", alpha=0.1, power=1.0)
    c, b = glm_ref.fit_tweedie_newton(X, y, 0.1, 1.0)
    assert abs(glm.score(X, y) - glm_ref.r2_score(spec, c, b, X, y)) < 1e-6
    assert abs(glm.neg_mse_score(X, y) - glm_ref.neg_mse_score(spec, c, b, X, y)) < 1e-6 * max(1, abs(glm_ref.neg_mse_score(spec, c, b, X, y)))
    r, mr = glm.get_residuals(X, y)
    assert rel(r, y - glm_ref.predict(spec, c, b, X)) < 1e-5
    assert rel(mr, y - y.mean()) == 0


def test_poisson_y_range_error(engine):
    import sglm
    X = np.random.default_rng(0).random((50, 3))
    with pytest.raises(ValueError, match="out of the valid range"):
        sglm.GLM("Poisson").fit(X, -np.ones(50))
    # through the CV grid: one negative response on a training row of some split
    import sglm_cv
    y = np.ones(50)
    y[7] = -1.0
    cv_idx = [(np.setdiff1d(np.arange(50), np.arange(k, 50, 5)), np.arange(k, 50, 5))
              for k in range(5)]
    kws = sglm_cv.generate_mult_params({"alpha": [1.0]}, {"model_name": "Poisson"})
    with pytest.raises(ValueError, match="out of the valid range"):
        sglm_cv.cv_glm_mult_params(X, y, cv_idx, "Normal", kws)


def test_cv_grid_vs_golden(engine, golden):
    import sglm_cv
    g = golden("cv_grid.npz")
    X, y = g["cvg_X"], g["cvg_y"]
    cv_idx = [(g[f"cvg_k{k}_train"], g[f"cvg_k{k}_test"]) for k in range(3)]
    kws = sglm_cv.generate_mult_params({"alpha": list(g["cvg_alphas"])}, {"model_name": "Poisson"})
    out = sglm_cv.cv_glm_mult_params(X, y, cv_idx, "Normal", kws)
    assert all("model_name" not in k for k in kws)          # popped from the caller's dicts
    for j, r in enumerate(out["full_cv_results"]):
        assert rel(r["cv_coefs"], g[f"cvg_a{j}_cv_coefs"]) < TOL_POIS
        assert rel(r["cv_intercepts"], g[f"cvg_a{j}_cv_intercepts"]) < TOL_POIS
        assert rel(r["cv_scores_test"], g[f"cvg_a{j}_scores_test"]) < 1e-6
        assert rel(r["cv_scores_train"], g[f"cvg_a{j}_scores_train"]) < 1e-6
        assert abs(r["cv_R2_score"] - float(g[f"cvg_a{j}_R2"])) < 1e-6
        assert abs(r["cv_mse_score"] - float(g[f"cvg_a{j}_mse"])) < 1e-6 * float(g[f"cvg_a{j}_mse"])
        assert rel(r["model"].coef_, g[f"cvg_a{j}_full_coef"]) < TOL_POIS
        assert set(r) == {"cv_coefs", "cv_intercepts", "cv_scores_train", "cv_scores_test",
                          "cv_mean_score_train", "cv_mean_score", "cv_std_score", "cv_R2_score",
                          "cv_mse_score", "glm_kwargs", "model"}
    best = int(np.argmax([float(g[f"cvg_a{j}_scores_test"].mean()) for j in range(3)]))
    assert out["best_params"] == out["full_cv_results"][best]["glm_kwargs"]


def test_simple_cv_fit_gaussian_grid_vs_oracle(engine):
    """Ridge/Lasso/OLS grid with rolls, r2 scoring, trial-id folds — against the oracle."""
    import sglm_ez
    import sglm_cv
    from sglm_hip import synth
    s = synth.make(N=6000, m=4, L=3, family="gaussian", rho=0.1, seed=21, beta_scale=0.5)
    X = pd.DataFrame(s.dense_X(), columns=[f"c{i}" for i in range(s.p)])
    X["nTrial"] = s.trial
    y = pd.Series(s.y)
    np.random.seed(3)
    cv_idx = sglm_ez.cv_idx_by_trial_id(X, trial_id_columns=["nTrial"], num_folds=4)
    np.random.seed(3)
    ref_idx = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]), num_folds=4)
    for (a, b), (c, d) in zip(cv_idx, ref_idx):
        assert np.array_equal(a, c) and np.array_equal(b, d)
    Xf = X.drop(columns="nTrial")
    kws = sglm_cv.generate_mult_params({"alpha": [0, 0.5, 50.0], "l1_ratio": [0, 1]},
                                       {"max_iter": 1000})
    kws[1]["roll"] = 3
    ref_kws = [dict(k) for k in kws]
    out = sglm_ez.simple_cv_fit(Xf, y, cv_idx, kws, model_type="Normal", score_method="r2")
    ref = cv_ref.cv_mult(Xf.values, y.values, cv_idx, ref_kws, score_method="r2")
    for r, q in zip(out[4]["full_cv_results"], ref["full_cv_results"]):
        assert rel(r["cv_coefs"], q["cv_coefs"]) < TOL_GAUSS, r["glm_kwargs"]
        # R^2 is dimensionless and near 0 here: absolute tolerance
        assert np.max(np.abs(r["cv_scores_test"] - q["cv_scores_test"])) < 1e-6
        assert abs(r["cv_R2_score"] - q["cv_R2_score"]) < 1e-6
        assert rel(r["model"].coef_, q["coef"]) < TOL_GAUSS
    assert out[2] == ref["best_params"]


def test_timeshift_cols_dataframe(engine):
    import sglm_ez
    X = pd.DataFrame(np.arange(200).reshape((100, 2)), columns=["A", "B"])
    X["B"] = (X["B"] - 1) * 2 + 1
    out = sglm_ez.timeshift_cols(X, ["A"], neg_order=-2, pos_order=2)
    assert list(out.columns) == ["A", "B", "A_-2", "A_-1", "A_1", "A_2"]
    ref = pp_ref.timeshift_multiple(X.values, [0], [0, -2, -1, 1, 2])
    assert np.array_equal(out.values.astype(float), ref.astype(float), equal_nan=True)


def test_c2_scale_poisson_parity(engine):
    """C2 shape (Poisson 100k x 500, alpha = 1.0) against the float64 oracle."""
    from sglm_hip import synth
    import sglm
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    X = s.dense_X()
    glm = sglm.GLM("Poisson", alpha=1.0)
    glm.fit(X, s.y)
    c, b = glm_ref.fit_tweedie_newton(X, s.y, 1.0, 1.0)
    assert rel(glm.coef_, c) < TOL_POIS
    glm = sglm.GLM("Poisson", alpha=1e-4)
    glm.fit(X, s.y)
    c, b = glm_ref.fit_tweedie_newton(X, s.y, 1e-4, 1.0)
    assert rel(glm.coef_, c) < TOL_POIS


def test_c3_shape_poisson_grid_vs_oracle(engine):
    """C3 shape: Poisson 100k x 500 timeshifted design, 5 GroupShuffleSplit splits on trial
    ids (seed 3), 3 lambdas of the logspace(-4, 1, 20) grid, r2 (D^2) scoring — every fold
    fit, refit, score and the pooled R^2 against the float64 oracle; folds bit-exact."""
    import sglm_cv
    import sglm_ez
    from sglm_hip import synth
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    X = s.dense_X()
    np.random.seed(3)
    df = pd.DataFrame({"nTrial": s.trial})
    cv_idx = sglm_ez.cv_idx_by_trial_id(df, trial_id_columns=["nTrial"], num_folds=5)
    np.random.seed(3)
    ref_idx = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]), num_folds=5)
    for (a, b), (c, d) in zip(cv_idx, ref_idx):
        assert np.array_equal(a, c) and np.array_equal(b, d)
    alphas = [float(v) for v in np.logspace(-4, 1, 20)[[0, 10, 19]]]
    kws = sglm_cv.generate_mult_params({"alpha": alphas}, {"model_name": "Poisson"})
    ref_kws = [dict(k) for k in kws]
    out = sglm_cv.cv_glm_mult_params(X, s.y, cv_idx, "Normal", kws, score_method="r2")
    ref = cv_ref.cv_mult(X, s.y, cv_idx, ref_kws, score_method="r2")
    for r, q in zip(out["full_cv_results"], ref["full_cv_results"]):
        assert rel(r["cv_coefs"], q["cv_coefs"]) < TOL_POIS, r["glm_kwargs"]
        assert rel(r["cv_intercepts"], q["cv_intercepts"]) < TOL_POIS
        assert np.max(np.abs(r["cv_scores_test"] - q["cv_scores_test"])) < 1e-6
        assert np.max(np.abs(r["cv_scores_train"] - q["cv_scores_train"])) < 1e-6
        assert abs(r["cv_R2_score"] - q["cv_R2_score"]) < 1e-6
        assert rel(r["model"].coef_, q["coef"]) < TOL_POIS
    assert out["best_params"] == ref["best_params"]


def test_setup_model_fit_timeshift_vals_by_dict(engine):
    """Package event-major expansion (setup_model_fit.timeshift_vals_by_dict): lag 0
    duplicated, int columns promoted to float64, NaN drop on the LAST entry's extreme lags —
    against the oracle restatement and plain pandas shift()."""
    from sglm.features import setup_model_fit as smf
    rng = np.random.default_rng(31)
    n = 500
    df = pd.DataFrame({"ev_a": (rng.random(n) < 0.1).astype(np.int64),
                       "ev_b": (rng.random(n) < 0.2).astype(np.float32),
                       "sig": rng.standard_normal(n),
                       "nTrial": np.arange(n) // 50})
    orders = {"ev_a": (-3, 2), "ev_b": (-1, 4), "sig": (-2, 2)}
    for keep in (True, False):
        out, names = smf.timeshift_vals_by_dict(df, orders, keep_nans=keep)
        assert names == [f"{c}_{s}" for c, (lo, hi) in orders.items() for s in range(lo, hi + 1)]
        assert list(out.columns) == list(df.columns) + names
        for c, (lo, hi) in orders.items():
            for s in range(lo, hi + 1):
                exp = df[[c]].shift(s)[c]
                if not keep:
                    exp = exp.loc[out.index]
                assert out[f"{c}_{s}"].dtype == exp.dtype, (c, s)
                assert np.array_equal(out[f"{c}_{s}"].values, exp.values, equal_nan=True), (c, s)
        idx = {c: i for i, c in enumerate(df.columns)}
        ref = pp_ref.timeshift_by_dict(df.values.astype(np.float64),
                                       {idx[c]: o for c, o in orders.items()}, keep_nans=keep)
        assert ref.shape == out.shape
        assert np.array_equal(out.values.astype(np.float64), ref, equal_nan=True)


def test_multi_response_enet_path_vs_oracle(engine):
    """C5 path (small): 3 responses x 3 alphas elastic net (l1_ratio 0.5), 3 trial-id splits +
    refits in ONE call with shared per-mask Grams and Gram-algebra scores — against the oracle
    run per response (what the reference's per-response loop computes)."""
    from sglm_hip import enet, synth
    s = synth.make(N=6000, m=5, L=3, family="gaussian", rho=0.15, seed=41, beta_scale=0.5)
    X = s.dense_X()
    rng = np.random.default_rng(42)
    B = rng.normal(0, 0.5, (s.p, 3))
    Y = X @ B + 0.3 + rng.normal(0, 1.0, (s.N, 3))
    np.random.seed(3)
    cv_idx = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]), num_folds=3)
    alphas = [1e-3, 1e-2, 1e-1]
    for method in ("r2", "mse"):
        st = {}
        out = enet.cv_enet_path(X, Y, cv_idx, alphas, l1_ratio=0.5, max_iter=1000,
                                score_method=method, stats=st)
        assert st["grams"] == 7 and st["fits"] == 3 * 3 * 4
        for r in range(3):
            kws = [{"alpha": a, "l1_ratio": 0.5, "max_iter": 1000} for a in alphas]
            ref = cv_ref.cv_mult(X, Y[:, r], cv_idx, kws, score_method=method)
            for j, q in enumerate(ref["full_cv_results"]):
                g = out[r][j]
                assert rel(g["cv_coefs"], q["cv_coefs"]) < TOL_GAUSS, (r, j)
                assert rel(g["cv_intercepts"], q["cv_intercepts"]) < TOL_GAUSS
                tol = 1e-6 if method == "r2" else 1e-6 * np.max(np.abs(q["cv_scores_test"]))
                assert np.max(np.abs(g["cv_scores_test"] - q["cv_scores_test"])) < tol
                assert np.max(np.abs(g["cv_scores_train"] - q["cv_scores_train"])) < tol
                assert abs(g["cv_R2_score"] - q["cv_R2_score"]) < 1e-6
                assert rel(g["refit_coef"], q["coef"]) < TOL_GAUSS
                assert abs(g["refit_intercept"] - q["intercept"]) < 1e-5 * max(1, abs(q["intercept"]))
                assert g["converged"]


def test_c1_shape_ols_vs_oracle(engine):
    """C1 shape (Gaussian OLS 10k x 100, one trial-id split): the drop-in GLM on the MI355X
    against the oracle's lstsq (1e-5 relative) and its train/test scores."""
    import sglm
    from sglm_hip import synth
    s = synth.make(N=10_000, m=10, L=5, family="gaussian", rho=0.05, seed=7)
    X = s.dense_X()
    np.random.seed(3)
    tr, te = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]),
                                              num_folds=1, test_size=0.2)[0]
    glm = sglm.GLM("Normal", alpha=0)
    glm.fit(X[tr], s.y[tr])
    c, b = glm_ref.fit_ols(X[tr], s.y[tr])
    assert rel(glm.coef_, c) < TOL_GAUSS
    assert abs(glm.intercept_ - b) < TOL_GAUSS * max(1.0, abs(b))
    pred = X[te] @ c + b
    assert abs(glm.neg_mse_score(X[te], s.y[te]) + np.mean((s.y[te] - pred) ** 2)) < 1e-6


def test_holdout_resplit_cv_vs_sequential_oracle(engine):
    """3 holdout resplits x (4 folds x 3 ridge/lasso params + refits) as ONE batched solve,
    against the sequential loop restated with the oracle on the same RNG stream: splits
    bit-exact, fold coefficients / scores and the best refit's holdout scores to tolerance."""
    import sglm_ez
    from sglm_hip import synth
    s = synth.make(N=8000, m=5, L=3, family="gaussian", rho=0.12, seed=61, beta_scale=0.5)
    X = s.dense_X()
    ids = pd.DataFrame({"nTrial": s.trial})
    kws = [{"alpha": 0.5, "l1_ratio": 0}, {"alpha": 5.0, "l1_ratio": 0},
           {"alpha": 0.01, "l1_ratio": 1, "max_iter": 1000}]
    np.random.seed(9)
    out = sglm_ez.holdout_resplit_cv(X, s.y, ids, kws, num_runs=3, id_cols=["nTrial"],
                                     perc_holdout=0.25, num_folds=4, score_method="r2")
    np.random.seed(9)
    codes = folds_ref.trial_bucket_codes([s.trial])
    G = int(codes.max() + 1)
    for run in out:
        test_ids = np.random.choice(G, size=int(G * 0.25))          # backend: with replacement
        hold = np.isin(codes, test_ids)
        assert np.array_equal(run["holdout"], hold)
        setup = np.flatnonzero(~hold)
        sc = folds_ref.trial_bucket_codes([s.trial[setup]])
        ref_idx = folds_ref.cv_idx_from_bucket_ids(sc, num_folds=4)
        for (a, b), (c, d) in zip(run["cv_idx"], ref_idx):
            assert np.array_equal(a, c) and np.array_equal(b, d)
        ref = cv_ref.cv_mult(X[setup], s.y[setup], ref_idx, [dict(k) for k in kws],
                             score_method="r2")
        for g, q in zip(run["full_cv_results"], ref["full_cv_results"]):
            assert rel(g["cv_coefs"], q["cv_coefs"]) < TOL_GAUSS
            assert np.max(np.abs(g["cv_scores_test"] - q["cv_scores_test"])) < 1e-6
        assert run["best_params"] == ref["best_params"]
        qb = ref["full_cv_results"][ref["best_index"]]
        pred = X[hold] @ qb["coef"] + qb["intercept"]
        yh = s.y[hold]
        r2 = 1 - np.sum((yh - pred) ** 2) / np.sum((yh - yh.mean()) ** 2)
        assert abs(run["holdout_score"] - r2) < 1e-6
        assert abs(run["holdout_neg_mse_score"] + np.mean((yh - pred) ** 2)) < 1e-6 * max(1, np.mean(yh ** 2))


@pytest.mark.parametrize("n,p", [(7, 1), (63, 3), (65, 255), (1000, 256), (1000, 257),
                                 (3000, 40)])
def test_odd_shapes_vs_oracle(engine, n, p):
    """Padding boundaries (P = 256, 512), rows below one 64-row K-step, ragged n, with and
    without intercept, binary and real-valued designs: Poisson and ridge vs the oracle."""
    import sglm
    rng = np.random.default_rng(n * 1000 + p)
    for binary in (True, False):
        X = (rng.random((n, p)) < 0.3).astype(np.float64) if binary else rng.normal(0, 1, (n, p))
        w = rng.normal(0, 0.3 / np.sqrt(p), p)
        y = rng.poisson(np.exp(X @ w + 0.2)).astype(np.float64)
        if y.sum() == 0:
            y[0] = 1.0
        for fi in (True, False):
            a = 1.0
            glm = sglm.GLM("Poisson", alpha=a, fit_intercept=fi)
            glm.fit(X, y)
            c, b = glm_ref.fit_tweedie_newton(X, y, a, 1.0, fit_intercept=fi)
            assert rel(glm.coef_, c) < TOL_POIS, (n, p, binary, fi)
            assert abs(glm.intercept_ - b) < TOL_POIS * max(1.0, abs(b)), (n, p, binary, fi)
            yg = X @ w + rng.normal(0, 1, n)
            glm = sglm.GLM("Normal", alpha=2.0, l1_ratio=0, fit_intercept=fi)
            glm.fit(X, yg)
            c, b = glm_ref.fit_ridge(X, yg, 2.0, fit_intercept=fi)
            assert rel(glm.coef_, c) < TOL_GAUSS, (n, p, binary, fi, "ridge")
            assert abs(glm.intercept_ - b) < TOL_GAUSS * max(1.0, abs(b))


def test_hessian_reuse_keeps_the_fixed_point(engine, monkeypatch):
    """Hessian reuse, lambda-neighbour sharing and cross-mask sharing (engine.HESS_REUSE_TOL,
    HESS_SHARE_TOL, HESS_XMASK_TOL) only change the inexact-Newton contraction, not the
    minimiser: a C3-shape 5-split x 20-lambda Poisson grid with the defaults matches the same
    grid with a fresh own Hessian every iteration (1e-5 relative), converges everywhere, and
    actually kept and aliased factors; two lambdas are also held to the float64 oracle."""
    import pandas as pd
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    lams = np.logspace(-4, 1, 20)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100) for a in lams]
    st = E.IrlsStats()
    fast = grid.run(d, s.y, cv_idx, objs, [0] * len(objs), stats=st)
    assert st.reused > 0 and st.aliased > 0 and st.gram_fits < st.fit_iters
    monkeypatch.setattr(E, "HESS_REUSE_TOL", 0.0)
    monkeypatch.setattr(E, "HESS_SHARE_TOL", 0.0)
    monkeypatch.setattr(E, "HESS_XMASK_TOL", 0.0)
    st0 = E.IrlsStats()
    exact = grid.run(d, s.y, cv_idx, objs, [0] * len(objs), stats=st0)
    assert st0.reused == 0 and st0.aliased == 0
    for a, b in zip(fast, exact):
        assert rel(a["cv_coefs"], b["cv_coefs"]) < 1e-5
        assert rel(a["cv_intercepts"], b["cv_intercepts"]) < 1e-5
        assert rel(a["refit_coef"], b["refit_coef"]) < 1e-5
        assert a["converged"] and b["converged"]
    X = s.dense_X()
    for j in (0, 12):
        c, b0 = glm_ref.fit_tweedie_newton(X, s.y, float(lams[j]), 1.0)
        assert rel(fast[j]["refit_coef"], c) < TOL_POIS


def test_first_iteration_gradient_dedup(engine, monkeypatch):
    """GRAD_DEDUP (round 6): in the first iteration the link and the gradient run once per
    (mask, response, intercept) start key and the other fits' gradient rows are copies.  A
    C3-shape 5-split x 20-lambda Poisson grid plus a no-intercept and a rolled-response group
    (distinct keys of one mask) matches the same grid with every fit's own link and gradient
    (1e-6 relative: the gradient's split-K slabs follow the batch size) and converges
    everywhere."""
    import pandas as pd
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=2)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(5)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    lams = np.logspace(-4, 1, 20)
    objs = ([Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100) for a in lams]
            + [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", False, 100)
               for a in lams[:3]])
    rolls = [0] * len(lams) + [7] * 3
    st = E.IrlsStats()
    on = grid.run(d, s.y, cv_idx, objs, rolls, stats=st)
    assert st.grad_dedup > 0
    monkeypatch.setattr(E, "GRAD_DEDUP", False)
    st0 = E.IrlsStats()
    off = grid.run(d, s.y, cv_idx, objs, rolls, stats=st0)
    assert st0.grad_dedup == 0
    for a, b in zip(on, off):
        assert rel(a["cv_coefs"], b["cv_coefs"]) < 1e-6
        assert rel(a["cv_intercepts"], b["cv_intercepts"]) < 1e-6
        assert rel(a["refit_coef"], b["refit_coef"]) < 1e-6
        assert a["converged"] and b["converged"]


def test_concurrent_chains_equal_one_chain(engine, monkeypatch):
    """A batch of new factorisations split over two concurrent chains (CHOL_SPLIT = 2, the
    default for >= CHOL_SPLIT_MIN) does per fit the arithmetic of one chain: a C3-shape
    5-split x 20-lambda Poisson grid (20 new factors in its first iteration) gives the same
    coefficients bit for bit with one chain."""
    import pandas as pd
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=4)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(6)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100)
            for a in np.logspace(-4, 1, 20)]
    monkeypatch.setattr(E, "CHOL_SPLIT", 2)
    monkeypatch.setattr(E, "CHOL_SPLIT_MIN", 12)
    two = grid.run(d, s.y, cv_idx, objs, [0] * len(objs))
    monkeypatch.setattr(E, "CHOL_SPLIT", 1)
    one = grid.run(d, s.y, cv_idx, objs, [0] * len(objs))
    for a, b in zip(two, one):
        assert np.array_equal(a["cv_coefs"], b["cv_coefs"])
        assert np.array_equal(a["refit_coef"], b["refit_coef"])
        assert a["converged"] and b["converged"]


def test_enet_cd_lane_kernel_equals_reg_kernel(engine, monkeypatch):
    """The lane-decision CD kernel (eight fits per 512-thread workgroup, SGLM_CD_FPW=8, the
    default) and the four-fit register kernel (SGLM_CD_FPW=4) perform the same arithmetic per
    coordinate in the same order: the coefficients agree bit for bit (p = 500, 4 responses x 5
    alphas x 3 splits + refit = 80 fits, a ragged last workgroup)."""
    from sglm_hip import enet, synth
    s = synth.make(N=20_000, m=50, L=5, family="gaussian", rho=0.05, seed=8, beta_scale=0.3)
    X = s.dense_X()
    rng = np.random.default_rng(9)
    Y = np.stack([s.y + rng.normal(0, 1, s.N) for _ in range(4)], 1)
    np.random.seed(4)
    cv_idx = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]), num_folds=3)
    alphas = [1e-4, 1e-3, 1e-2, 1e-1, 1.0]
    outs = {}
    for fpw in ("4", "8"):
        monkeypatch.setenv("SGLM_CD_FPW", fpw)
        st = {}
        outs[fpw] = enet.cv_enet_path(X, Y, cv_idx, alphas, l1_ratio=0.5, stats=st)
    for r in range(4):
        for j in range(len(alphas)):
            a, b = outs["4"][r][j], outs["8"][r][j]
            assert np.array_equal(a["cv_coefs"], b["cv_coefs"]), (r, j)
            assert np.array_equal(a["refit_coef"], b["refit_coef"]), (r, j)
            assert a["n_iter"] == b["n_iter"] and a["converged"] and b["converged"]
