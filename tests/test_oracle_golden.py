"""Pin the CPU oracle against the committed golden fixtures (no GPU)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from oracle import cv_ref, folds_ref, glm_ref, pp_ref

from conftest import GOLDEN


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


# ------------------------------------------------------------------ timeshift known answers
def test_timeshift_known_answers(golden):
    g = golden("timeshift_known.npz")
    X = g["ts_X"]
    assert np.array_equal(pp_ref.timeshift(X, shift_amt=0), X)
    assert np.array_equal(pp_ref.timeshift(X, [0, 3], 0), X[:, [0, 3]])
    assert np.array_equal(pp_ref.timeshift(X, shift_amt=1, fill_value=0), g["ts_fwd"])
    assert np.array_equal(pp_ref.timeshift(X, [0, 3], 1, fill_value=0), g["ts_fwd"][:, [0, 3]])
    assert np.array_equal(pp_ref.timeshift(X, shift_amt=-1, fill_value=0), g["ts_bwd"])
    assert np.array_equal(pp_ref.timeshift(X, [0, 1], 1, keep_non_inx=True, fill_value=0),
                          g["ts_keep_fwd"])
    assert np.array_equal(pp_ref.timeshift(X, [0, 1], -1, keep_non_inx=True, fill_value=0),
                          g["ts_keep_bwd"])
    assert np.array_equal(pp_ref.timeshift_multiple(X, shift_amt_list=[-1, 0, 1], fill_value=0),
                          g["ts_multi_all"])
    assert np.array_equal(pp_ref.timeshift_multiple(X, [0, 3], [-1, 0, 1], fill_value=0),
                          g["ts_multi_03"])


def test_timeshift_by_dict_matches_pandas_shift():
    rng = np.random.default_rng(0)
    X = (rng.random((50, 3)) < 0.3).astype(float)
    df = pd.DataFrame(X, columns=list("abc"))
    orders = {0: (-2, 3), 2: (-1, 1)}
    out = pp_ref.timeshift_by_dict(X, orders)
    cols = [df]
    for c, (ng, ps) in orders.items():
        name = df.columns[c]
        for s in range(ng, ps + 1):
            cols.append(df[[name]].shift(s).rename({name: f"{name}_{s}"}, axis=1))
    ref = pd.concat(cols, axis=1)
    # setup_model_fit.py:88-94 uses the last entry's (neg, pos) = (-1, 1) for every column
    ref = ref.dropna(subset=["a_-1", "c_-1", "a_1", "c_1"])
    assert np.array_equal(out, ref.values, equal_nan=True)


# ------------------------------------------------------------------ fits
def test_poisson_fits(golden):
    g = golden("fits.npz")
    meta = json.load(open(os.path.join(GOLDEN, "fits_meta.json")))
    X, y = g["pois_X"], g["pois_y"]
    for m in meta:
        coef, b = glm_ref.fit_tweedie_newton(X, y, m["alpha"], 1.0,
                                             fit_intercept=m["fit_intercept"])
        assert rel(coef, g[m["key"] + "_coef"]) < 1e-9, m
        assert abs(b - float(g[m["key"] + "_b"])) < 1e-9


def test_poisson_zero_column(golden):
    g = golden("fits.npz")
    coef, b = glm_ref.fit_tweedie_newton(g["pois_zero_X"], g["pois_y"], 0.0, 1.0)
    # sklearn's newton-cholesky leaves lbfgs-level error on this singular Hessian
    assert rel(coef, g["pois_zero_coef"]) < 1e-6
    assert coef[3] == 0.0


def test_gamma_fit(golden):
    g = golden("fits.npz")
    coef, b = glm_ref.fit_tweedie_newton(g["gam_X"], g["gam_y"], 0.05, 2.0)
    assert rel(coef, g["gam_coef"]) < 1e-9
    assert abs(b - float(g["gam_b"])) < 1e-9


def test_gaussian_fits(golden):
    g = golden("fits.npz")
    X, y = g["gau_X"], g["gau_y"]
    c, b = glm_ref.fit_ols(X, y)
    assert rel(c, g["ols_coef"]) < 1e-10
    for i, a in enumerate([0.1, 10.0, 1000.0]):
        c, b = glm_ref.fit_ridge(X, y, a)
        assert rel(c, g[f"ridge_a{i}_coef"]) < 1e-10
        assert abs(b - float(g[f"ridge_a{i}_b"])) < 1e-10
    for i, a in enumerate([1e-3, 1e-2]):
        c, b = glm_ref.fit_enet_cd(X, y, a, 1.0)
        assert rel(c, g[f"lasso_a{i}_coef"]) < 1e-7
        c, b = glm_ref.fit_enet_cd(X, y, a, 0.5)
        assert rel(c, g[f"enet_a{i}_coef"]) < 1e-7
    c, b = glm_ref.fit_ols(g["olsr_X"], y)
    assert rel(c, g["olsr_coef"]) < 1e-8


def test_tweedie_via_spec_matches_ridge_scaling(golden):
    """Tweedie(power=0) objective uses mean + alpha/2 (not Ridge's sum + alpha)."""
    g = golden("fits.npz")
    X, y = g["gau_X"], g["gau_y"]
    n = X.shape[0]
    c1, b1 = glm_ref.fit_tweedie_newton(X, y, 0.01, 0.0)
    c2, b2 = glm_ref.fit_ridge(X, y, 0.01 * n)
    assert rel(c1, c2) < 1e-9


# ------------------------------------------------------------------ folds
def test_group_shuffle_split_bit_exact(golden):
    g = golden("folds.npz")
    trial = np.arange(5000) // 100
    for seed in (0, 3, 17):
        codes = folds_ref.trial_bucket_codes([trial])
        assert np.array_equal(codes, g[f"f{seed}_codes"])
        np.random.seed(seed)
        splits = folds_ref.cv_idx_from_bucket_ids(codes, num_folds=5)
        for k, (tr, te) in enumerate(splits):
            assert np.array_equal(tr, g[f"f{seed}_k{k}_train"])
            assert np.array_equal(te, g[f"f{seed}_k{k}_test"])
    assert np.array_equal(folds_ref.trial_bucket_codes([trial, trial // 7]),
                          g["codes_two_backend"])
    assert np.array_equal(folds_ref.trial_bucket_codes([trial, trial // 7], package_style=True),
                          g["codes_two_package"])
    bid = folds_ref.bucket_ids_by_timeframe(437, 20)
    np.random.seed(5)
    splits = folds_ref.cv_idx_from_bucket_ids(bid)
    assert len(splits) == int(g["tf_nsplits"])
    for k, (tr, te) in enumerate(splits):
        assert np.array_equal(tr, g[f"tf_k{k}_train"])
        assert np.array_equal(te, g[f"tf_k{k}_test"])


# ------------------------------------------------------------------ CV grid
def test_cv_grid_aggregation(golden):
    g = golden("cv_grid.npz")
    X, y = g["cvg_X"], g["cvg_y"]
    cv_idx = [(g[f"cvg_k{k}_train"], g[f"cvg_k{k}_test"]) for k in range(3)]
    kws = cv_ref.generate_mult_params({"alpha": list(g["cvg_alphas"])},
                                      {"model_name": "Poisson"})
    res = cv_ref.cv_mult(X, y, cv_idx, kws)
    for j, r in enumerate(res["full_cv_results"]):
        assert rel(r["cv_coefs"], g[f"cvg_a{j}_cv_coefs"]) < 1e-8
        assert rel(r["cv_scores_test"], g[f"cvg_a{j}_scores_test"]) < 1e-9
        assert abs(r["cv_R2_score"] - float(g[f"cvg_a{j}_R2"])) < 1e-9
        assert abs(r["cv_mse_score"] - float(g[f"cvg_a{j}_mse"])) < 1e-9
        assert rel(r["coef"], g[f"cvg_a{j}_full_coef"]) < 1e-8
    best = int(np.argmax([float(g[f"cvg_a{j}_scores_test"].mean()) for j in range(3)]))
    assert res["best_index"] == best


def test_generate_mult_params_order():
    out = cv_ref.generate_mult_params({"alpha": [1, 2], "l1_ratio": [0, 1]}, {"max_iter": 5})
    assert out == [{"max_iter": 5, "alpha": 1, "l1_ratio": 0},
                   {"max_iter": 5, "alpha": 1, "l1_ratio": 1},
                   {"max_iter": 5, "alpha": 2, "l1_ratio": 0},
                   {"max_iter": 5, "alpha": 2, "l1_ratio": 1}]


def test_c1_ols_oracle_vs_sklearn():
    """C1 shape (Gaussian OLS, 10k x 100 timeshifted design, 1 split): the oracle's lstsq
    restatement against scikit-learn LinearRegression called directly (plumbing only)."""
    import sys
    from sklearn.linear_model import LinearRegression
    sys.path.insert(0, __import__("conftest").PKG)
    from sglm_hip import synth
    s = synth.make(N=10_000, m=10, L=5, family="gaussian", rho=0.05, seed=7)
    X = s.dense_X()
    np.random.seed(3)
    cv = folds_ref.cv_idx_from_bucket_ids(folds_ref.trial_bucket_codes([s.trial]), num_folds=1,
                                          test_size=0.2)
    tr, te = cv[0]
    c, b = glm_ref.fit_ols(X[tr], s.y[tr])
    sk = LinearRegression().fit(X[tr], s.y[tr])
    assert np.max(np.abs(c - sk.coef_)) <= 1e-9 * max(1.0, np.max(np.abs(sk.coef_)))
    assert abs(b - sk.intercept_) <= 1e-9 * max(1.0, abs(sk.intercept_))


def test_d2_score_and_tweedie_power_pinned_to_sklearn(golden):
    """glm_ref.r2_score's D^2 (GLM.r2_score for Tweedie, backend/sglm.py:184 -> sklearn
    TweedieRegressor.score) and the explicit-power Tweedie fit (backend/sglm.py:116-117)
    against sklearn 1.7.2 (tests/golden/make_golden.py::api_extras)."""
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    tr, te = np.arange(0, 2400), np.arange(2400, 3000)
    for key in ("tw15", "pois", "tw12"):
        power, a = float(g[f"{key}_power"]), float(g[f"{key}_alpha"])
        c, b = glm_ref.fit_tweedie_newton(X[tr], y[tr], a, power)
        assert np.max(np.abs(c - g[f"{key}_coef"])) < 1e-8 * max(1, np.max(np.abs(c))), key
        assert abs(b - float(g[f"{key}_b"])) < 1e-8
        spec = glm_ref.FitSpec("tweedie", alpha=a, power=power)
        for rows, tag in ((tr, "train"), (te, "test")):
            d2 = glm_ref.r2_score(spec, g[f"{key}_coef"], float(g[f"{key}_b"]), X[rows], y[rows])
            assert abs(d2 - float(g[f"{key}_d2_{tag}"])) < 1e-12, (key, tag)
    spec = glm_ref.FitSpec("tweedie", alpha=0.05, power=2.0)
    d2 = glm_ref.r2_score(spec, g["gam_coef"], float(g["gam_b"]), g["gam_X"], g["gam_y"])
    assert abs(d2 - float(g["gam_d2"])) < 1e-12


def test_warm_start_oracle_reaches_the_same_minimiser(golden):
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    tr = np.arange(0, 2400)
    c, b = glm_ref.fit_tweedie_newton(X[tr], y[tr], 0.01, 1.0,
                                      coef0=np.r_[g["warm_w0"], float(g["warm_b0"])])
    assert np.max(np.abs(c - g["warm_coef"])) < 1e-8
    assert abs(b - float(g["warm_b"])) < 1e-8


# ------------------------------------------------------------------ rank deficiency (round 4)
def rank_design(g, key):
    """X of a rank.npz case, rebuilt from its bit-packed events with the fixture's expansion."""
    from sglm_hip import synth
    if key == "pdup":
        sh = tuple(g["pdup_shape"])
        return np.unpackbits(g["pdup_X"], axis=0)[: sh[0]].astype(np.float64)
    sh = tuple(g[f"{key}_shape"])
    E = np.unpackbits(g[f"{key}_E"], axis=0)[: sh[0]].astype(np.float32)
    L, N = int(g[f"{key}_L"]), int(g[f"{key}_N"])
    return synth.Synthetic(E=E, L=L, shifts=synth.shift_list(L), N=N, beta=None, intercept=0.0,
                           y=None, trial=None, family="gaussian").dense_X()


def test_rank_fixtures_pin_the_oracle(golden):
    """lstsq's minimum-norm OLS on a duplicated-event lag design and on a cond ~7e6 full-rank
    0/1 design, and unpenalised Poisson lbfgs from 0 with a duplicated column: the oracle
    (glm_ref.fit_ols / fit_tweedie_newton) reproduces sklearn's answers."""
    g = golden("rank.npz")
    X = rank_design(g, "dup")
    c, b = glm_ref.fit_ols(X, g["dup_y"])
    assert rel(c, g["dup_coef"]) < 1e-9 and abs(b - float(g["dup_b"])) < 1e-9
    for bi in range(10):                       # event 9 duplicates event 2: equal split
        assert abs(c[bi * 10 + 2] - c[bi * 10 + 9]) < 1e-12
        assert abs(c[bi * 10 + 5]) < 1e-12     # event 5 never occurs
    X = rank_design(g, "ill")
    assert 1e6 < float(g["ill_cond"]) < 1e8
    c, b = glm_ref.fit_ols(X, g["ill_y"])
    assert rel(c, g["ill_coef"]) < 1e-8
    X = rank_design(g, "pdup")
    c, b = glm_ref.fit_tweedie_newton(X, g["pdup_y"], 0.0, 1.0)
    assert rel(c, g["pdup_coef"]) < 1e-6 and abs(c[5] - c[-1]) < 1e-12


# ------------------------------------------------------------------ mixed designs (round 5)
def mixed_design(g, key="mx"):
    """X of a mixed.npz case: the bit-packed 0/1 columns and the float64 continuous columns
    (``key`` 'mxill' takes the near-collinear counter pair) at their positions."""
    N, p = (int(v) for v in g["mx_shape"])
    X = np.zeros((N, p))
    X[:, g["mx_binc"]] = np.unpackbits(g["mx_bits"], axis=0)[:N].astype(np.float64)
    X[:, g["mx_cpos"]] = g["mxill_cont"] if key == "mxill" else g["mx_cont"]
    return X


def test_mixed_fixtures_pin_the_oracle(golden):
    """The production layout (0/1 lags + two cumcount^2/5000 counters + session dummies,
    fit_intercept=False; sglm_cb_concat_make_design_mat.py:211-216, 224-244, 266): the oracle's
    float64 lstsq / damped Newton reproduce sklearn's LinearRegression and TweedieRegressor
    answers, including the near-collinear counter pair (cond ~7e9)."""
    g = golden("mixed.npz")
    X = mixed_design(g)
    c, b = glm_ref.fit_ols(X, g["mx_y"], fit_intercept=False)
    assert rel(c, g["mx_coef"]) < 1e-10 and b == 0.0
    c, b = glm_ref.fit_ols(X[:, :-1], g["mx_y"])
    assert rel(c, g["mxfi_coef"]) < 1e-10 and abs(b - float(g["mxfi_b"])) < 1e-10
    Xi = mixed_design(g, "mxill")
    assert 1e9 < float(g["mxill_cond"]) < 1e11
    c, _ = glm_ref.fit_ols(Xi, g["mxill_y"], fit_intercept=False)
    assert rel(c, g["mxill_coef"]) < 1e-7
    c, _ = glm_ref.fit_tweedie_newton(X, g["mxpois_y"], 1e-4, 1.0, fit_intercept=False)
    assert rel(c, g["mxpois_coef"]) < 1e-7
    # the counters: cumcount^2 / 5000 over runs of consecutive integers
    cont = g["mx_cont"]
    for j in range(2):
        v = np.round(np.sqrt(cont[:, j] * 5000)).astype(np.int64)
        assert np.allclose(v.astype(float) ** 2 / 5000, cont[:, j], rtol=0, atol=1e-15)


def test_ols_chunks_matches_dense_lstsq(golden):
    """The chunked normal-equations OLS oracle (full-size grids) equals the dense lstsq oracle
    and sklearn's LinearRegression golden."""
    g = golden("fits.npz")
    X, y = g["gau_X"], g["gau_y"]
    ch = [(X[a:a + 700], y[a:a + 700]) for a in range(0, X.shape[0], 700)]
    c, b = glm_ref.fit_ols_chunks(ch)
    assert rel(c, g["ols_coef"]) < 1e-9 and abs(b - float(g["ols_b"])) < 1e-9
    gm = golden("mixed.npz")
    Xm = mixed_design(gm)
    c, b = glm_ref.fit_ols_chunks([(Xm, gm["mx_y"])], fit_intercept=False)
    assert rel(c, gm["mx_coef"]) < 1e-9 and b == 0.0
