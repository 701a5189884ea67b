"""Drop-in for ``backend/sglm_cv.py`` (import as ``import sglm_cv``).

Same functions, arguments, printed summaries and return dicts as the reference
(backend/sglm_cv.py:15-496).  Instead of a thread pool that fits ``X[idx_train, :]``
copies one at a time with sklearn, every (split, hyper-parameter) fit of the grid — plus
the per-parameter full refits — is solved in one batched IRLS on the MI355X
(sglm_hip.grid).  Differences on purpose:
  * the discarded PCA warm-up (:273-282) is skipped (no observable output);
  * results are assembled in grid order, so ``full_cv_results`` order and the pooled
    residual sums are deterministic (the reference's order depends on thread timing);
  * no worker threads, hence no queue deadlock (:26, :36).
"""
from __future__ import annotations

import itertools
import queue
import threading  # noqa: F401  (API parity)

import numpy as np

import sglm_
from sglm_hip import grid as _grid


class SGLM_worker():
    """backend/sglm_cv.py:15-40, kept for API compatibility (bounded queue waits)."""

    def __init__(self, queue, verbose=0):
        self.queue = queue
        self.verbose = verbose

    def run_single(self):
        while True:
            try:
                glm, args, kwargs = self.queue.get(timeout=3)
            except queue.Empty:
                return
            glm.fit_set(*args, **kwargs)
            self.queue.task_done()

    def run_multi(self):
        while True:
            try:
                args, kwargs = self.queue.get(timeout=3)
            except queue.Empty:
                return
            cv_glm_single_params(*args, **kwargs)
            self.queue.task_done()


def _values(a):
    from sglm_hip.lagframe import LagFrame
    if isinstance(a, LagFrame):
        return a.design()                      # resident lagged frame: its device design
    if hasattr(a, "values") and not isinstance(a, np.ndarray) and getattr(a, "ndim", 1) == 2:
        from sglm_hip.estimators import host_matrix
        return host_matrix(a)                  # nullable (convert_dtypes) frames per block
    return a.values if hasattr(a, "values") and not isinstance(a, np.ndarray) else a


def _run(X, y, cv_idx, params, score_method, beta_=None, beta0_=None, verbose=0):
    """params: list of (model_name, glm_kwargs, roll) -> list of reference ret_dicts."""
    objectives, models = [], []
    for model_name, glm_kwargs, roll in params:
        # constructing the GLM validates kwargs exactly like the reference's per-fold GLM()
        g = sglm_.GLM(model_name, beta0_=beta0_, beta_=beta_, **glm_kwargs,
                      score_method=score_method)
        objectives.append(g.model.objective())
        models.append(sglm_.GLM(model_name, beta0_=beta0_, beta_=beta_, **glm_kwargs))
    X = _values(X)
    y = np.asarray(_values(y))
    res = _grid.run(X, y.reshape(-1), cv_idx, objectives, [p[2] for p in params],
                    score_method=score_method,
                    coef0=beta_ if isinstance(beta_, np.ndarray) else None,
                    intercept0=beta0_)
    out = []
    for (model_name, glm_kwargs, roll), r, glm in zip(params, res, models):
        glm._set_fitted(r["refit_coef"], r["refit_intercept"], max(r["n_iter"]))
        d = {k: r[k] for k in ("cv_coefs", "cv_intercepts", "cv_scores_train", "cv_scores_test",
                               "cv_mean_score_train", "cv_mean_score", "cv_std_score",
                               "cv_R2_score", "cv_mse_score")}
        d["glm_kwargs"] = glm_kwargs
        d["model"] = glm
        if verbose > 0:
            print('Completing arguments:', glm_kwargs)
        print(f"{glm_kwargs}\n> cv_mean_score_train: {d['cv_mean_score_train']}\n"
              f"> cv_R2_score: {d['cv_R2_score']}\n> cv_mean_score: {d['cv_mean_score']}")
        out.append(d)
    return out


def cv_glm_single_params(X, y, cv_idx, model_name, glm_kwargs, verbose=0, resp_list=[],
                         beta_=None, beta0_=None, score_method='mse'):
    """backend/sglm_cv.py:42-206 — one hyper-parameter set over all splits + refit."""
    roll = glm_kwargs.pop('roll', 0)
    ret_dict = _run(X, y, cv_idx, [(model_name, glm_kwargs, roll)], score_method, beta_,
                    beta0_, verbose)[0]
    resp_list.append(ret_dict)
    return ret_dict


def cv_glm_mult_params(X, y, cv_idx, model_name, glm_kwarg_lst, verbose=0, score_method='mse'):
    """backend/sglm_cv.py:210-428 — the whole grid as one batched device solve."""
    params = []
    for glm_kwargs in glm_kwarg_lst:
        print(glm_kwargs)
        mn = glm_kwargs.pop('model_name', 'Gaussian')     # mutates the caller's dict (:288)
        roll = glm_kwargs.pop('roll', 0)                   # (:95)
        params.append((mn, glm_kwargs, roll))
    resp = _run(X, y, cv_idx, params, score_method, verbose=verbose)

    best_score = -np.inf
    best_score_std = best_params = best_model = None
    for cv_result in resp:
        if score_method == 'r2' and cv_result['cv_R2_score'] > best_score:
            best_score = cv_result['cv_R2_score']
            best_score_std = cv_result['cv_std_score']
            best_params = cv_result['glm_kwargs']
            best_model = cv_result['model']
        elif score_method == 'mse' and cv_result['cv_mean_score'] > best_score:
            best_score = cv_result['cv_mean_score']
            best_score_std = cv_result['cv_std_score']
            best_params = cv_result['glm_kwargs']
            best_model = cv_result['model']
    return {
        'best_score': best_score,
        'best_score_std': best_score_std,
        'best_params': best_params,
        'best_model': best_model,
        'full_cv_results': resp,
    }


def generate_mult_params(kwarg_lists, kwargs=None):
    """backend/sglm_cv.py:476-496."""
    base_list = [[kwargs]] if kwargs else []
    flipped_dict_list = base_list + [[{key: _} for _ in kwarg_lists[key]] for key in kwarg_lists]
    cart_prod = list(itertools.product(*flipped_dict_list))
    return [{_key: dct[_key] for dct in cart_prod[i] for _key in dct} for i in range(len(cart_prod))]
