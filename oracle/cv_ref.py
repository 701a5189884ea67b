"""CPU restatement of the reference CV grid — TEST INFRASTRUCTURE.

* ``generate_mult_params`` — backend/sglm_cv.py:476-496 (fixed kwargs first, then
                             itertools.product over keys, last key fastest).
* ``cv_single``            — backend/sglm_cv.py:42-206 with GLM.fit_set (backend/sglm.py:
                             254-312): roll (:95-96), per-split fit on X[idx_train] /
                             y_rolled[idx_train], train/test scores, residual pooling, full refit on
                             UN-rolled y (:180-181, score_method not forwarded -> 'mse').
* ``cv_mult``              — backend/sglm_cv.py:210-428: model_name popped per kwargs
                             (default 'Gaussian', :288), best = first strict max (:402-415).
                             The discarded PCA warm-up (:273-282) has no observable output
                             and is skipped.

Serial, deterministic, float64; uses oracle.glm_ref for every fit.
"""
from __future__ import annotations

import itertools

import numpy as np

from . import glm_ref


def generate_mult_params(kwarg_lists, kwargs=None):
    base_list = [[kwargs]] if kwargs else []
    flipped = base_list + [[{key: v} for v in kwarg_lists[key]] for key in kwarg_lists]
    prod = list(itertools.product(*flipped))
    return [{k: d[k] for d in combo for k in d} for combo in prod]


def _score(spec, coef, b, X, y, method):
    if method == "r2":
        return glm_ref.r2_score(spec, coef, b, X, y)
    return glm_ref.neg_mse_score(spec, coef, b, X, y)


def cv_single(X, y, cv_idx, model_name, glm_kwargs, score_method="mse", tight=True):
    glm_kwargs = dict(glm_kwargs)
    roll = glm_kwargs.pop("roll", 0)
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    y_rolled = np.roll(y, roll)
    spec = glm_ref.spec_from_glm_kwargs(model_name, glm_kwargs)
    K = len(cv_idx)
    cv_coefs = np.zeros((X.shape[1], K))
    cv_b = np.zeros(K)
    s_tr = np.zeros(K)
    s_te = np.zeros(K)
    resids, mresids = [], []
    for k, (tr, te) in enumerate(cv_idx):
        coef, b = glm_ref.fit(spec, X[tr], y_rolled[tr], tight=tight)
        cv_coefs[:, k] = coef
        cv_b[k] = b
        s_tr[k] = _score(spec, coef, b, X[tr], y_rolled[tr], score_method)
        s_te[k] = _score(spec, coef, b, X[te], y_rolled[te], score_method)
        yt = y_rolled[te]
        resids.append(yt - glm_ref.predict(spec, coef, b, X[te]))
        mresids.append(yt - np.mean(yt))
    coef, b = glm_ref.fit(spec, X, y, tight=tight)
    R = np.concatenate(resids)
    return {
        "cv_coefs": cv_coefs,
        "cv_intercepts": cv_b,
        "cv_scores_train": s_tr,
        "cv_scores_test": s_te,
        "cv_mean_score_train": np.mean(s_tr),
        "cv_mean_score": np.mean(s_te),
        "cv_std_score": np.std(s_te),
        "cv_R2_score": glm_ref.calc_R2(R, np.concatenate(mresids)),
        "cv_mse_score": np.mean(np.square(R)),
        "glm_kwargs": glm_kwargs,
        "coef": coef,
        "intercept": b,
    }


def cv_mult(X, y, cv_idx, glm_kwarg_lst, score_method="mse", tight=True):
    resp = []
    for kw in glm_kwarg_lst:
        kw = dict(kw)
        model_name = kw.pop("model_name", "Gaussian")
        resp.append(cv_single(X, y, cv_idx, model_name, kw, score_method, tight))
    best, best_std, best_params, best_i = -np.inf, None, None, None
    for i, r in enumerate(resp):
        s = r["cv_R2_score"] if score_method == "r2" else r["cv_mean_score"]
        if s > best:
            best, best_std, best_params, best_i = s, r["cv_std_score"], r["glm_kwargs"], i
    return {"best_score": best, "best_score_std": best_std, "best_params": best_params,
            "best_index": best_i, "full_cv_results": resp}
