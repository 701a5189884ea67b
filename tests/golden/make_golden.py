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
       ``python tests/golden/make_golden.py rank`` -> tests/golden/rank.npz only
       ``python tests/golden/make_golden.py mixed`` -> tests/golden/mixed.npz only
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


def _lag_X(E, L, N):
    """Shift-major lag expansion of synth.Synthetic.dense_X (shifts [0] + [-L..-1] + [1..L-1])."""
    return synth.Synthetic(E=E, L=L, shifts=synth.shift_list(L), N=N, beta=None, intercept=0.0,
                           y=None, trial=None, family="gaussian").dense_X()


def rank_cases():
    """Round-4 pins of lstsq's minimum-norm answer (backend/sglm.py:96-101 -> sklearn
    _base.py:701) and of unpenalised Poisson lbfgs from w = 0 (backend/sglm.py:112-115):
    * dup: C1 shape (10k x 100, 10 events x lags -5..4) with event 9 a copy of event 2 (ten
      duplicated lag columns) and event 5 never occurring (ten zero columns) -> LinearRegression;
    * ill: a full-rank 0/1 lag design with cond(X~^T X~) ~ 7e6: two slow state indicators
      (runs of 2000-5000 rows) that differ on one row, plus a sparse event, lags -15..14 ->
      LinearRegression (a float32 factor cannot resolve it);
    * pdup: Poisson 3000 x 41 with a duplicated column, alpha = 0, lbfgs at tol 1e-12.
    Events are stored bit-packed; the tests rebuild X with the same expansion."""
    out = {}
    s = synth.make(N=10000, m=10, L=5, family="gaussian", rho=0.05, seed=7)
    E = s.E.copy()
    E[:, 9] = E[:, 2]
    E[:, 5] = 0.0
    X = _lag_X(E, 5, 10000)
    rng = np.random.default_rng(71)
    y = X @ rng.normal(0, 0.3, X.shape[1]) + 0.5 + rng.normal(0, 1, X.shape[0])
    ols = LinearRegression().fit(X, y)
    out.update(dup_E=np.packbits(E.astype(np.uint8), axis=0), dup_shape=np.array(E.shape),
               dup_L=np.array(5), dup_N=np.array(10000), dup_y=y, dup_coef=ols.coef_,
               dup_b=np.array(ols.intercept_))
    # ill-conditioned, full rank
    rng = np.random.default_rng(5)
    L, N = 15, 100000
    Nr = N + 2 * L - 1

    def runs(lo, hi):
        x = np.zeros(Nr)
        t, v = 0, int(rng.integers(0, 2))
        while t < Nr:
            n_ = int(rng.integers(lo, hi))
            x[t:t + n_] = v
            v, t = 1 - v, t + n_
        return x
    e1 = runs(2000, 5000)
    e2 = e1.copy()
    e2[Nr // 3] = 1 - e2[Nr // 3]
    E = np.stack([e1, e2, (rng.random(Nr) < 0.05).astype(float)], 1).astype(np.float32)
    X = _lag_X(E, L, N)
    beta = rng.normal(0, 0.5, X.shape[1])
    y = np.round((X @ beta + 0.3 + rng.normal(0, 1, N)) * 4096) / 4096
    Xt = np.hstack([X, np.ones((N, 1))])
    ev = np.linalg.eigvalsh(Xt.T @ Xt)
    ols = LinearRegression().fit(X, y)
    out.update(ill_E=np.packbits(E.astype(np.uint8), axis=0), ill_shape=np.array(E.shape),
               ill_L=np.array(L), ill_N=np.array(N), ill_y=y, ill_coef=ols.coef_,
               ill_b=np.array(ols.intercept_), ill_cond=np.array(ev[-1] / ev[0]))
    # Poisson, duplicated column, alpha = 0: lbfgs from 0 keeps the duplicates equal
    sp = synth.make(N=3000, m=4, L=5, family="poisson", rho=0.05, seed=10, beta_scale=0.3)
    Xp = np.hstack([sp.dense_X(), sp.dense_X()[:, [5]]])
    tp = TweedieRegressor(power=1, alpha=0.0, tol=1e-12, max_iter=100000).fit(Xp, sp.y)
    out.update(pdup_X=np.packbits(Xp.astype(np.uint8), axis=0), pdup_shape=np.array(Xp.shape),
               pdup_y=sp.y, pdup_coef=tp.coef_, pdup_b=np.array(tp.intercept_),
               pdup_niter=np.array(tp.n_iter_))
    return out


def _prod_columns(N, seed):
    """A production-like design in the layout of sglm_cb_concat_make_design_mat.py (:224-244,
    :266, :310): 0/1 event lags (8 events x shifts 0, -5..-1, 1..4, shift-major), the two
    unshifted counters of pp_design_mat.py:167-172 -- (ENL | Cue) rows' cumcount within the
    trial, squared / (50*100), and the state_ENLP rows' cumcount within (trial, nENL), squared /
    (50*100), 0 elsewhere -- and one 0/1 dummy per session (pd.get_dummies(session)).  Returns
    (X, continuous column positions, trial ids)."""
    rng = np.random.default_rng(seed)
    lens = []
    while sum(lens) < N:
        lens.append(int(rng.integers(80, 160)))
    nTrial = np.repeat(np.arange(1, len(lens) + 1), lens)[:N]
    Cue, ENL, ENLP, nENL = (np.zeros(N) for _ in range(4))
    t0 = 0
    for ln in lens:
        if t0 >= N:
            break
        Cue[t0] = 1
        le = int(rng.integers(20, 60))
        ENL[t0 + 1:min(N, t0 + 1 + le)] = 1
        s0 = t0 + 1 + le
        for q in range(int(rng.integers(0, 3))):       # 0-2 penalty periods (nENL = 1, 2)
            lp = int(rng.integers(8, 20))
            ENLP[s0:min(N, s0 + lp, t0 + ln)] = 1
            nENL[s0:min(N, s0 + lp, t0 + ln)] = q + 1
            s0 += lp + int(rng.integers(2, 6))
        t0 += ln
    df = pd.DataFrame({"nTrial": nTrial, "Cue": Cue, "ENL": ENL, "ENLP": ENLP, "nENL": nENL})
    sel = (df.ENL == 1) | (df.Cue == 1)
    t_enl = np.zeros(N)
    t_enl[sel.values] = df.loc[sel].groupby("nTrial").cumcount().values ** 2 / (50 * 100)
    selp = df.ENLP == 1
    t_enlp = np.zeros(N)
    t_enlp[selp.values] = (df.loc[selp].groupby(["nTrial", "nENL"]).cumcount().values ** 2
                           / (50 * 100))
    L = 5
    E = (rng.random((N + 2 * L, 8)) < 0.04).astype(np.float32)
    Xl = _lag_X(E, L, N)
    ntr = int(nTrial.max())
    session = np.minimum((nTrial - 1) * 3 // ntr, 2)
    S = np.stack([(session == j).astype(float) for j in range(3)], 1)
    X = np.hstack([Xl, t_enl[:, None], t_enlp[:, None], S])
    cpos = np.array([Xl.shape[1], Xl.shape[1] + 1])
    return X, cpos, nTrial


def mixed_cases():
    """Round-5 pins of the production design (mixed 0/1 + continuous, fit_intercept=False,
    alpha = 0; sglm_cb_concat_make_design_mat.py:211-216, 356-363 -> LinearRegression, lstsq in
    float64, sklearn _base.py:701):
    * mx: LinearRegression(fit_intercept=False) on the design of _prod_columns (12,000 x 85);
    * mxfi: LinearRegression() (intercept) on it minus the last session dummy;
    * mxill: the second counter replaced by the first times (1 + 1e-4 w), w = +-1 per row (a
      near-collinear pair: cond(X^T X) ~ 1e10, beyond any float32 Gram);
    * mxpois: TweedieRegressor(power=1, alpha=1e-4, fit_intercept=False), newton-cholesky at tol
      1e-12, on Poisson counts from the same design.
    0/1 columns are stored bit-packed, the continuous ones as float64."""
    X, cpos, trial = _prod_columns(12000, 51)
    N, p = X.shape
    rng = np.random.default_rng(52)
    binc = np.setdiff1d(np.arange(p), cpos)
    beta = rng.normal(0, 0.4, p)
    beta[cpos] = [0.8, -0.6]
    y = X @ beta + rng.normal(0, 1.0, N)
    out = dict(mx_bits=np.packbits(X[:, binc].astype(np.uint8), axis=0), mx_binc=binc,
               mx_cpos=cpos, mx_cont=X[:, cpos].copy(), mx_shape=np.array(X.shape),
               mx_trial=trial, mx_y=y)
    out["mx_coef"] = LinearRegression(fit_intercept=False).fit(X, y).coef_
    fi = LinearRegression().fit(X[:, :-1], y)
    out.update(mxfi_coef=fi.coef_, mxfi_b=np.array(fi.intercept_))
    w = np.where(rng.random(N) < 0.5, -1.0, 1.0)
    Xi = X.copy()
    Xi[:, cpos[1]] = X[:, cpos[0]] * (1 + 1e-4 * w)
    yi = Xi @ beta + rng.normal(0, 1.0, N)
    ev = np.linalg.eigvalsh(Xi.T @ Xi)
    out.update(mxill_cont=Xi[:, cpos].copy(), mxill_y=yi,
               mxill_coef=LinearRegression(fit_intercept=False).fit(Xi, yi).coef_,
               mxill_cond=np.array(ev[-1] / ev[0]))
    bp = rng.normal(0, 0.15, p)
    bp[-3:] = [0.5, 0.7, 0.3]
    bp[cpos] = [0.05, -0.08]
    yp = rng.poisson(np.exp(X @ bp)).astype(float)
    tp = TweedieRegressor(power=1, alpha=1e-4, fit_intercept=False, solver="newton-cholesky",
                          tol=1e-12, max_iter=1000).fit(X, yp)
    out.update(mxpois_y=yp, mxpois_coef=tp.coef_)
    return out


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
    if sys.argv[1:] == ["mixed"]:          # round-5 fixture only (others unchanged)
        np.savez_compressed(os.path.join(HERE, "mixed.npz"), **mixed_cases())
        print("mixed fixture written")
        return
    if sys.argv[1:] == ["rank"]:           # round-4 fixture only (others unchanged)
        np.savez_compressed(os.path.join(HERE, "rank.npz"), **rank_cases())
        print("rank fixture written")
        return
    np.savez_compressed(os.path.join(HERE, "api.npz"), **api_extras())
    np.savez_compressed(os.path.join(HERE, "rank.npz"), **rank_cases())
    np.savez_compressed(os.path.join(HERE, "mixed.npz"), **mixed_cases())
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
