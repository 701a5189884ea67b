"""Generate the committed golden fixtures (run once in the build container).

Sources — never the reference code itself (its import/execution was denied):
* scikit-learn 1.7.2 estimators called DIRECTLY with the kwargs ``backend/sglm.py:95-130``
  would select, at tight tolerance (the minimiser the reference's solver approaches), plus
  the default-tolerance lbfgs output (what the reference literally prints) for the record;
* sklearn ``GroupShuffleSplit`` on seeded global RNG for the fold indices
  (backend/sglm_pp.py:262-263, backend/sglm_ez.py:334-342 key scheme);
* the known answers of ``backend/test/test_sglm_pp.py`` (inputs ``arange(20).reshape(5,4)``
  and the 4x3 matrix), rebuilt here from the same tiny numpy expressions.

Usage: ``python tests/golden/make_golden.py`` -> tests/golden/*.npz / *.json
       ``python tests/golden/make_golden.py api`` -> tests/golden/api.npz only
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import pandas as pd
from sklearn.linear_model import (ElasticNet, Lasso, LinearRegression, Ridge,
                                  TweedieRegressor)
from sklearn.model_selection import GroupShuffleSplit

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "sabatinilab-glm_amd"))
from sglm_hip import synth  # noqa: E402  (synthetic data generator only)

warnings.filterwarnings("ignore")


def timeshift_known_answers():
    X = np.arange(20).reshape(5, 4)
    z = np.zeros((1, 4))
    fwd = np.concatenate([z, X], axis=0)[:-1]
    bwd = np.concatenate([X, z], axis=0)[1:]
    keep_fwd = X.copy().astype(float)
    keep_fwd[:, [0, 1]] = np.concatenate([z[:, [0, 1]], X[:, [0, 1]]], axis=0)[:-1]
    keep_bwd = X.copy().astype(float)
    keep_bwd[:, [0, 1]] = np.concatenate([X[:, [0, 1]], z[:, [0, 1]]], axis=0)[1:]
    multi_all = np.concatenate([bwd, X, fwd], axis=1)
    multi_03 = np.concatenate([bwd[:, [0, 3]], X, fwd[:, [0, 3]]], axis=1)
    Z = np.array([[0, -1, 0], [1, 1, 0], [0, 1, 0], [2, 3, 4]])
    return dict(ts_X=X, ts_fwd=fwd, ts_bwd=bwd, ts_keep_fwd=keep_fwd, ts_keep_bwd=keep_bwd,
                ts_multi_all=multi_all, ts_multi_03=multi_03,
                z_X=Z, z_expected=(Z - Z.mean(0)) / Z.std(0),
                diff_expected=np.array([[1, 2, 0], [-1, 0, 0], [2, 2, 4]]))


def fits():
    out = {}
    meta = []
    # Poisson on a synthetic timeshift design (0/1 events, lags -5..4 -> p = 40)
    sp = synth.make(N=3000, m=4, L=5, family="poisson", rho=0.05, seed=10, beta_scale=0.3)
    Xp = sp.dense_X()
    out["pois_X"] = Xp
    out["pois_y"] = sp.y
    for i, a in enumerate([1e-3, 0.1, 1.0]):
        for fi in (True, False):
            tight = TweedieRegressor(power=1, alpha=a, fit_intercept=fi, solver="newton-cholesky",
                                     tol=1e-12, max_iter=1000).fit(Xp, sp.y)
            ref = TweedieRegressor(power=1, alpha=a, fit_intercept=fi).fit(Xp, sp.y)
            key = f"pois_a{i}_fi{int(fi)}"
            out[key + "_coef"] = tight.coef_
            out[key + "_b"] = np.array(tight.intercept_)
            out[key + "_lbfgs_coef"] = ref.coef_
            out[key + "_niter"] = np.array(tight.n_iter_)
            meta.append(dict(key=key, alpha=a, fit_intercept=fi, family="Poisson"))
    # Poisson with an all-zero column and alpha = 0 (rank-deficient Hessian)
    Xz = Xp[:, :12].copy()
    Xz[:, 3] = 0.0
    tz = TweedieRegressor(power=1, alpha=0.0, solver="newton-cholesky", tol=1e-12,
                          max_iter=1000).fit(Xz, sp.y)
    out["pois_zero_X"] = Xz
    out["pois_zero_coef"] = tz.coef_
    out["pois_zero_b"] = np.array(tz.intercept_)
    # Gamma (power 2, log link)
    sg = synth.make(N=2000, m=3, L=3, family="gamma", rho=0.1, seed=20, beta_scale=0.2)
    Xg = sg.dense_X()
    tg = TweedieRegressor(power=2, alpha=0.05, solver="newton-cholesky", tol=1e-12,
                          max_iter=1000).fit(Xg, sg.y)
    out.update(gam_X=Xg, gam_y=sg.y, gam_coef=tg.coef_, gam_b=np.array(tg.intercept_))
    # Gaussian: OLS / Ridge / Lasso / ElasticNet on a real-valued + event design
    sn = synth.make(N=2500, m=5, L=3, family="gaussian", rho=0.1, seed=30, beta_scale=0.5)
    Xn = sn.dense_X()
    Xn = np.hstack([Xn, np.random.default_rng(31).normal(size=(Xn.shape[0], 2))])
    yn = sn.y + Xn[:, -2:] @ np.array([0.3, -0.2])
    out.update(gau_X=Xn, gau_y=yn)
    ols = LinearRegression().fit(Xn, yn)
    out.update(ols_coef=ols.coef_, ols_b=np.array(ols.intercept_))
    for i, a in enumerate([0.1, 10.0, 1000.0]):
        r = Ridge(alpha=a).fit(Xn, yn)
        out[f"ridge_a{i}_coef"] = r.coef_
        out[f"ridge_a{i}_b"] = np.array(r.intercept_)
    for i, a in enumerate([1e-3, 1e-2]):
        las = Lasso(alpha=a, tol=1e-14, max_iter=1000000).fit(Xn, yn)
        out[f"lasso_a{i}_coef"] = las.coef_
        out[f"lasso_a{i}_b"] = np.array(las.intercept_)
        en = ElasticNet(alpha=a, l1_ratio=0.5, tol=1e-14, max_iter=1000000).fit(Xn, yn)
        out[f"enet_a{i}_coef"] = en.coef_
        out[f"enet_a{i}_b"] = np.array(en.intercept_)
    # OLS, rank deficient (duplicate + zero column): min-norm solution
    Xr = np.hstack([Xn[:, :6], Xn[:, [2]], np.zeros((Xn.shape[0], 1))])
    olr = LinearRegression().fit(Xr, yn)
    out.update(olsr_X=Xr, olsr_coef=olr.coef_, olsr_b=np.array(olr.intercept_))
    return out, meta


def folds():
    out = {}
    trial = np.arange(5000) // 100
    X = pd.DataFrame({"nTrial": trial, "iBlock": trial // 7})
    for seed in (0, 3, 17):
        # single id column, backend key scheme (sglm_ez.py:334-340)
        key = X["nTrial"].astype(str).str.len().astype(str) + ":" + X["nTrial"].astype(str)
        codes = key.astype("category").cat.codes.values
        np.random.seed(seed)
        splits = list(GroupShuffleSplit(n_splits=5, test_size=0.2).split(X, None, codes))
        for k, (tr, te) in enumerate(splits):
            out[f"f{seed}_k{k}_train"] = tr
            out[f"f{seed}_k{k}_test"] = te
        out[f"f{seed}_codes"] = codes
    # two id columns (backend '_' join) and the package '__len:' join
    k1 = (X["nTrial"].astype(str).str.len().astype(str) + ":" + X["nTrial"].astype(str)
          + "_" + X["iBlock"].astype(str))
    out["codes_two_backend"] = k1.astype("category").cat.codes.values
    s0, s1 = X["nTrial"].apply(str), X["iBlock"].apply(str)
    k2 = (s0.str.len().apply(str) + ":" + s0 + "__" + s1.str.len().apply(str) + ":" + s1)
    out["codes_two_package"] = k2.astype("category").cat.codes.values
    # timeframe buckets (sglm_pp.py:218-234) with LOO default num_folds
    N = 437
    bid = np.arange(N) // (N // 20)
    np.random.seed(5)
    splits = list(GroupShuffleSplit(n_splits=int(bid.max() + 1),
                                    test_size=1 / (bid.max() + 1)).split(np.zeros(N), None, bid))
    for k, (tr, te) in enumerate(splits):
        out[f"tf_k{k}_train"] = tr
        out[f"tf_k{k}_test"] = te
    out["tf_nsplits"] = np.array(len(splits))
    return out


def cv_grid():
    """3-split x 3-lambda Poisson grid, computed with sklearn in the reference's loop order."""
    sp = synth.make(N=4000, m=3, L=3, family="poisson", rho=0.08, seed=40, beta_scale=0.3)
    X = sp.dense_X()
    y = sp.y
    codes = (pd.Series(sp.trial).astype(str).str.len().astype(str) + ":"
             + pd.Series(sp.trial).astype(str)).astype("category").cat.codes.values
    np.random.seed(7)
    cv_idx = list(GroupShuffleSplit(n_splits=3, test_size=1 / 3).split(X, None, codes))
    out = {"cvg_X": X, "cvg_y": y}
    for k, (tr, te) in enumerate(cv_idx):
        out[f"cvg_k{k}_train"] = tr
        out[f"cvg_k{k}_test"] = te
    alphas = [0.01, 0.1, 1.0]
    for j, a in enumerate(alphas):
        def mk():
            return TweedieRegressor(power=1, alpha=a, solver="newton-cholesky", tol=1e-12,
                                    max_iter=1000)
        coefs, bs, s_tr, s_te, res, mres = [], [], [], [], [], []
        for tr, te in cv_idx:
            m = mk().fit(X[tr], y[tr])
            coefs.append(m.coef_)
            bs.append(m.intercept_)
            s_tr.append(-np.mean((y[tr] - m.predict(X[tr])) ** 2))
            s_te.append(-np.mean((y[te] - m.predict(X[te])) ** 2))
            res.append(y[te] - m.predict(X[te]))
            mres.append(y[te] - y[te].mean())
        full = mk().fit(X, y)
        R, MR = np.concatenate(res), np.concatenate(mres)
        out[f"cvg_a{j}_cv_coefs"] = np.array(coefs).T
        out[f"cvg_a{j}_cv_intercepts"] = np.array(bs)
        out[f"cvg_a{j}_scores_train"] = np.array(s_tr)
        out[f"cvg_a{j}_scores_test"] = np.array(s_te)
        out[f"cvg_a{j}_R2"] = np.array(1 - np.sum(R ** 2) / np.sum(MR ** 2))
        out[f"cvg_a{j}_mse"] = np.array(np.mean(R ** 2))
        out[f"cvg_a{j}_full_coef"] = full.coef_
        out[f"cvg_a{j}_full_b"] = np.array(full.intercept_)
    out["cvg_alphas"] = np.array(alphas)
    return out


def api_extras():
    """Round-2 pins: Tweedie with an explicit power (GLM('Tweedie', power=1.5),
    backend/sglm.py:116-117), sklearn's D^2 ``TweedieRegressor.score`` (what GLM.r2_score
    returns for the Tweedie family, backend/sglm.py:184) on train and held-out rows, and a
    warm-started fit (backend/sglm.py:91-92,134-140: coef_/intercept_ preset, warm_start)."""
    out = {}
    sp = synth.make(N=3000, m=4, L=5, family="poisson", rho=0.05, seed=10, beta_scale=0.3)
    X, y = sp.dense_X(), sp.y
    tr, te = np.arange(0, 2400), np.arange(2400, 3000)
    out.update(api_X=X, api_y=y)
    for key, power, a in (("tw15", 1.5, 0.05), ("pois", 1.0, 0.01), ("tw12", 1.2, 0.1)):
        m = TweedieRegressor(power=power, alpha=a, solver="newton-cholesky", tol=1e-12,
                             max_iter=1000).fit(X[tr], y[tr])
        out[f"{key}_coef"] = m.coef_
        out[f"{key}_b"] = np.array(m.intercept_)
        out[f"{key}_d2_train"] = np.array(m.score(X[tr], y[tr]))
        out[f"{key}_d2_test"] = np.array(m.score(X[te], y[te]))
        out[f"{key}_alpha"] = np.array(a)
        out[f"{key}_power"] = np.array(power)
    # Gamma D^2 (power 2) on the gamma design
    sg = synth.make(N=2000, m=3, L=3, family="gamma", rho=0.1, seed=20, beta_scale=0.2)
    Xg = sg.dense_X()
    mg = TweedieRegressor(power=2, alpha=0.05, solver="newton-cholesky", tol=1e-12,
                          max_iter=1000).fit(Xg, sg.y)
    out.update(gam_X=Xg, gam_y=sg.y, gam_coef=mg.coef_, gam_b=np.array(mg.intercept_),
               gam_d2=np.array(mg.score(Xg, sg.y)))
    # warm start: lbfgs from a preset (coef_, intercept_) reaches the same minimiser
    w0 = np.full(X.shape[1], 0.05)
    mw = TweedieRegressor(power=1, alpha=0.01, warm_start=True, solver="newton-cholesky",
                          tol=1e-12, max_iter=1000)
    mw.coef_, mw.intercept_ = w0.copy(), -0.5
    mw.fit(X[tr], y[tr])
    out.update(warm_w0=w0, warm_b0=np.array(-0.5), warm_coef=mw.coef_,
               warm_b=np.array(mw.intercept_))
    return out


def main():
    if sys.argv[1:] == ["api"]:            # round-2 fixture only (others unchanged)
        np.savez_compressed(os.path.join(HERE, "api.npz"), **api_extras())
        print("api fixture written")
        return
    np.savez_compressed(os.path.join(HERE, "api.npz"), **api_extras())
    np.savez_compressed(os.path.join(HERE, "timeshift_known.npz"), **timeshift_known_answers())
    f, meta = fits()
    np.savez_compressed(os.path.join(HERE, "fits.npz"), **f)
    with open(os.path.join(HERE, "fits_meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    np.savez_compressed(os.path.join(HERE, "folds.npz"), **folds())
    np.savez_compressed(os.path.join(HERE, "cv_grid.npz"), **cv_grid())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
