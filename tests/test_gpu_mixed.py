"""Mixed 0/1 + continuous designs on the MI355X (round 5).

The reference's production design (sglm_cb_concat_make_design_mat.py:224-244, 266, 310) puts two
unshifted continuous counters -- cumcount^2 / (50*100) over the ENL / ENLP rows of each trial,
pp_design_mat.py:167-172 -- and one 0/1 dummy per session beside the 0/1 event lags, converts the
frame with ``convert_dtypes()`` and fits OLS (alpha = 0, fit_intercept=False) through
``simple_cv_fit`` (:356-363) in float64.  The engine keeps the 0/1 columns as bit-planes and
the continuous ones as a float64 block (csrc/mixed.hip); squared-loss fits are solved in Gram
space in float64 (engine._gram_ls).

Bars: coefficients 1e-5 relative (Gaussian) / 1e-4 (Poisson) of the sklearn goldens in
tests/golden/mixed.npz (tests/golden/make_golden.py mixed); kernel products against float64
numpy at their arithmetic's rounding.
"""
import numpy as np
import pandas as pd
import pytest

from oracle import glm_ref
from test_oracle_golden import mixed_design

pytestmark = pytest.mark.gpu
TOL_POIS, TOL_GAUSS = 1e-4, 1e-5


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_mixed_split_and_products(engine, golden):
    """from_host splits the design (0/1 columns as bit-planes, the two counters float64 at their
    positions); X beta, X^T R and the Gram rows of the counters (weighted and exact) against
    float64 numpy."""
    import torch
    g = golden("mixed.npz")
    X = mixed_design(g)
    N, p = X.shape
    d = engine.Design.from_host(X)
    assert d.k == 2 and list(d.cpos) == list(g["mx_cpos"]) and d.xbits is not None
    assert np.array_equal(d.cont[:, :N].cpu().numpy(), X[:, g["mx_cpos"]].T)
    rng = np.random.default_rng(3)
    beta = np.zeros((3, d.P), np.float32)
    beta[:, :p + 1] = rng.normal(0, 1, (3, p + 1))
    eta = d.eta(torch.from_numpy(beta).cuda())[:, :N].double().cpu().numpy()
    ref = beta[:, :p].astype(np.float64) @ X.T + beta[:, p:p + 1]
    assert np.max(np.abs(eta - ref)) < 1e-6 * np.max(np.abs(ref))
    R = rng.normal(0, 1, (4, d.ld)).astype(np.float32)
    R[:, N:] = 0
    G = torch.empty((4, d.P), dtype=torch.float64, device="cuda")
    d.xtr(torch.from_numpy(R).cuda(), 4, G)
    Gh = G.cpu().numpy()
    ref = R[:, :N].astype(np.float64) @ np.hstack([X, np.ones((N, 1))])
    cp = list(g["mx_cpos"])
    # 0/1 columns: exact products, f32 slab sums (float64 across slabs); the continuous
    # columns: float64 throughout
    assert np.max(np.abs(Gh[:, :p + 1] - ref)) < 1e-6 * np.max(np.abs(ref))
    assert np.max(np.abs(Gh[:, cp] - ref[:, cp])) < 1e-12 * np.max(np.abs(ref[:, cp]))
    # Gram rows of the counters: exact (mask multiplicities) and weighted (f32 IRLS weights)
    M = np.zeros((2, d.ld), np.uint8)
    M[0, :N] = 1
    M[1, :N] = rng.integers(0, 3, N)
    Md = torch.from_numpy(M).cuda()
    S = d.mix_gram_rows(M=Md, mrows=[0, 1]).cpu().numpy()
    Xa = np.hstack([X, np.ones((N, 1))])
    for s in range(2):
        ref = (Xa * M[s, :N, None]).T @ X[:, g["mx_cpos"]]
        # digit planes: 2^-38 of max |m c| per element, float64 sums
        assert np.max(np.abs(S[s][:, :p + 1] - ref.T)) < 1e-11 * np.max(np.abs(ref))
    W = np.zeros((3, d.ld), np.float32)
    W[:, :N] = rng.random((3, N))
    S = d.mix_gram_rows(W=torch.from_numpy(W).cuda(), wslots=[2, 0]).cpu().numpy()
    for s, slot in enumerate((2, 0)):
        ref = (Xa * W[slot, :N, None].astype(np.float64)).T @ X[:, g["mx_cpos"]]
        assert np.max(np.abs(S[s][:, :p + 1] - ref.T)) < 1e-6 * np.max(np.abs(ref))


@pytest.mark.parametrize("key", ["mx", "mxfi", "mxill"])
def test_mixed_ols_goldens(engine, golden, key):
    """LinearRegression on the production layout (fit_intercept=False, the session dummies as
    intercepts), with an intercept (one dummy dropped), and with a near-collinear counter pair
    (cond(X^T X) ~ 7e9: a float32 Gram cannot resolve it) -- sklearn's float64 lstsq answers at
    1e-5 through the drop-in GLM."""
    import sglm
    g = golden("mixed.npz")
    X = mixed_design(g, "mxill" if key == "mxill" else "mx")
    y = g["mxill_y"] if key == "mxill" else g["mx_y"]
    if key == "mxfi":
        glm = sglm.GLM("Normal", alpha=0.0)
        glm.fit(X[:, :-1], y)
        assert rel(glm.model.coef_, g["mxfi_coef"]) < TOL_GAUSS
        assert abs(glm.model.intercept_ - float(g["mxfi_b"])) < TOL_GAUSS
        return
    glm = sglm.GLM("Normal", alpha=0.0, fit_intercept=False)
    glm.fit(X, y)
    assert rel(glm.model.coef_, g[f"{key}_coef"]) < TOL_GAUSS
    assert glm.model.intercept_ == 0.0


def test_mixed_ridge_and_poisson(engine, golden):
    """Ridge (closed form vs the float64 normal equations) and the Poisson fit of the same
    design (TweedieRegressor alpha 1e-4, fit_intercept=False) against sklearn at 1e-4."""
    import sglm
    g = golden("mixed.npz")
    X = mixed_design(g)
    glm = sglm.GLM("Poisson", alpha=1e-4, fit_intercept=False)
    glm.fit(X, g["mxpois_y"])
    assert rel(glm.model.coef_, g["mxpois_coef"]) < TOL_POIS
    for a in (0.5, 50.0):
        glm = sglm.GLM("Normal", alpha=a, l1_ratio=0.0, fit_intercept=False)
        glm.fit(X, g["mx_y"])
        c = np.linalg.solve(X.T @ X + a * np.eye(X.shape[1]), X.T @ g["mx_y"])
        assert rel(glm.model.coef_, c) < TOL_GAUSS


def _prod_frame(g, key="mx"):
    """The golden design as the production driver hands it to simple_cv_fit: named columns,
    session dummies from pd.get_dummies (bool), nTrial, then convert_dtypes()
    (sglm_cb_concat_make_design_mat.py:244, 266)."""
    X = mixed_design(g, key)
    N, p = X.shape
    cpos = list(g["mx_cpos"])
    cols = {}
    for j in range(p - 3):
        cols[f"time_from_enl_onset" if j == cpos[0] else
             "time_from_enlp_onset" if j == cpos[1] else f"ev{j}"] = X[:, j]
    df = pd.DataFrame(cols)
    sess = np.argmax(X[:, -3:], axis=1)
    df["session"] = np.array(["s0", "s1", "s2"])[sess]
    df["nTrial"] = g["mx_trial"]
    df = pd.get_dummies(df, columns=["session"])
    df = df.convert_dtypes()
    return df


@pytest.mark.parametrize("family", ["Normal", "Poisson"])
def test_mixed_simple_cv_fit_convert_dtypes(engine, golden, family):
    """The production flow on a convert_dtypes() frame (Int64 / Float64 / boolean columns):
    cv_idx_by_trial_id -> drop nTrial -> simple_cv_fit.  Every fold's coefficients against the
    float64 oracle on the fold's rows and the refit against the sklearn golden (1e-5 OLS,
    1e-4 Poisson)."""
    import sglm_ez
    g = golden("mixed.npz")
    df = _prod_frame(g)
    assert any(str(dt) in ("Int64", "Float64", "boolean") for dt in df.dtypes)
    y = pd.Series(g["mx_y"] if family == "Normal" else g["mxpois_y"]).convert_dtypes()
    np.random.seed(30186)
    folds = sglm_ez.cv_idx_by_trial_id(df, y=y, trial_id_columns=["nTrial"], num_folds=3,
                                       test_size=0.2)
    Xs = df.drop(columns=["nTrial"])
    if family == "Normal":
        params = [{"alpha": 0.0, "l1_ratio": 0.0, "max_iter": 1000, "fit_intercept": False}]
    else:
        # the family comes from each dict's 'model_name' (popped with default 'Gaussian',
        # backend/sglm_cv.py:288); model_type only picks the discarded PCA warm-up (:275)
        params = [{"model_name": "Poisson", "alpha": 1e-4, "fit_intercept": False}]
    best_score, _, best_params, best_model, cvr = sglm_ez.simple_cv_fit(
        Xs, y, folds, params, model_type=family, verbose=0, score_method="r2")
    X = mixed_design(g)
    yv = np.asarray(y, dtype=np.float64)
    full = cvr["full_cv_results"][0]
    for k, (tr, te) in enumerate(folds):
        if family == "Normal":
            c, _ = glm_ref.fit_ols(X[tr], yv[tr], fit_intercept=False)
            assert rel(full["cv_coefs"][:, k], c) < TOL_GAUSS
        else:
            c, _ = glm_ref.fit_tweedie_newton(X[tr], yv[tr], 1e-4, 1.0, fit_intercept=False)
            assert rel(full["cv_coefs"][:, k], c) < TOL_POIS
    ref = g["mx_coef"] if family == "Normal" else g["mxpois_coef"]
    assert rel(best_model.model.coef_, ref) < (TOL_GAUSS if family == "Normal" else TOL_POIS)
    assert np.isfinite(best_score)
