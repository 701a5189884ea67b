"""Drop-in for ``backend/sglm.py`` (import as ``import sglm`` / ``import sglm_``).

``GLM`` keeps the reference's constructor, attributes and methods (backend/sglm.py:24-385)
and its estimator dispatch (:95-130), but the estimator classes it instantiates are the
MI355X-engine ones of ``sglm_hip.estimators`` (same signatures as the scikit-learn classes
the reference uses), so ``fit`` / ``fit_set`` / ``predict`` / ``score`` run on the GPU.

Behaviour fixed on purpose (SURVEY.md §7 "Reference defects"), API unchanged:
  * ``coef_``/``intercept_`` are read from ``model.coef_``/``model.intercept_`` for every
    family (the reference reads pyglmnet's ``beta_``/``beta0_`` for Poisson/Gamma/Tweedie
    and raises AttributeError, :246-251);
  * ``alpha == 0`` without ``l1_ratio``/``max_iter`` no longer raises KeyError (:97-99);
  * ``NotYetImplementedError`` is defined (the reference raises an undefined name).
Logistic/Multinomial and the PCA warm-start are out of scope.
"""
from __future__ import annotations

import time
from typing import Tuple, Union

import numpy as np
import pandas as pd
import scipy.stats

from sglm_hip.estimators import (ElasticNet, Lasso, LinearRegression, LogisticRegression,  # noqa: F401
                                 NotYetImplementedError, PoissonRegressor, Ridge,
                                 TweedieRegressor, host_matrix)


class GLM():
    """Generalized Linear Model on the MI355X engine (API of backend/sglm.py:24-147)."""

    model = None
    model_name_options = {'Normal', 'Gaussian', 'Poisson', 'Tweedie', 'Gamma', 'Logistic',
                          'Binomial', 'Multinomial'}
    tweedie_lookup = {'Normal': 0, 'Gaussian': 0, 'Poisson': 1, 'Gamma': 2}

    def __init__(self, model_name, beta0_=None, beta_=None, score_method='mse', *args, **kwargs):
        if 'warm_start' not in kwargs and (beta0_ is not None or isinstance(beta_, np.ndarray)):
            kwargs['warm_start'] = True

        self.model_name = model_name
        if model_name in {'Normal', 'Gaussian'}:
            if 'alpha' in kwargs and kwargs['alpha'] == 0:
                kwargs.pop('alpha')
                kwargs.pop('l1_ratio', None)
                kwargs.pop('max_iter', None)
                kwargs.pop('warm_start', None)
                Base = LinearRegression
            elif 'l1_ratio' in kwargs and kwargs['l1_ratio'] == 0:
                del kwargs['l1_ratio']
                kwargs.pop('warm_start', None)
                Base = Ridge
            elif 'l1_ratio' in kwargs and kwargs['l1_ratio'] == 1:
                del kwargs['l1_ratio']
                Base = Lasso
            else:
                Base = ElasticNet
        elif model_name in {'Poisson', 'Gamma'}:
            kwargs['power'] = self.tweedie_lookup[model_name]
            Base = TweedieRegressor
        elif model_name in {'Tweedie'}:
            Base = TweedieRegressor
        elif model_name in {'Logistic', 'Multinomial'}:
            kwargs['multi_class'] = 'multinomial' if model_name == 'Multinomial' else 'auto'
            kwargs['n_jobs'] = kwargs['n_jobs'] if 'n_jobs' in kwargs else -1
            Base = LogisticRegression
        elif model_name in {'PCA Normal', 'PCA Gaussian'}:
            Base = LinearRegression
        else:
            print('Distribution not yet implemented.')
            raise NotYetImplementedError(model_name)

        self.Base = Base
        self.kwargs = kwargs
        self.model = self.Base(*args, **kwargs)

        if beta0_ is not None:
            self.model.intercept_ = beta0_
            self.beta0_ = beta0_
        if isinstance(beta_, np.ndarray):
            self.beta_ = np.copy(beta_)
            self.model.coef_ = self.beta_

        if score_method == 'r2':
            self.score = self.r2_score
        else:
            self.score = self.neg_mse_score

    def neg_mse_score(self, X, y):
        """backend/sglm.py:150-167."""
        pred = self.predict(X)
        resid = (y - pred)
        return -np.mean(resid ** 2)

    def r2_score(self, X, y):
        """backend/sglm.py:169-184 (R^2 for Gaussian estimators, D^2 for Tweedie)."""
        return self.model.score(X, y)

    def pca_fit(self, X, y):
        """backend/sglm.py:186-223 — PCA warm start; its only reference use is discarded
        (backend/sglm_cv.py:273-282), so the engine does not implement it."""
        raise NotYetImplementedError("pca_fit: the discarded PCA warm-up is out of scope")

    def fit(self, X, y, *args):
        """backend/sglm.py:225-251 — one engine fit."""
        self.model.fit(X, y, *args)
        self.coef_ = self.model.coef_
        self.beta_ = self.coef_
        self.intercept_ = self.model.intercept_
        self.beta0_ = self.intercept_

    def _set_fitted(self, coef, intercept, n_iter=0):
        """Install coefficients computed by the batched grid engine."""
        self.model._set_fitted(coef, intercept, n_iter)
        self.coef_ = self.model.coef_
        self.beta_ = self.coef_
        self.intercept_ = self.model.intercept_
        self.beta0_ = self.intercept_

    def fit_set(self, X, y, X_test, y_test, cv_coefs, cv_intercepts, cv_scores_train,
                cv_scores_test, iter_cv, *args, resids=[], mean_resids=[], id_fit='None',
                verbose=0):
        """backend/sglm.py:254-312: fit, then write coefficients/scores in place."""
        if verbose > 1:
            start = time.time()
            print(f'Fitting: {self.kwargs} — {id_fit}')
        # each of X / X_test is packed into HBM once for the fit, both scores and the
        # residuals (the reference re-reads them from host memory four times)
        Xv = host_matrix(X) if type(X) == pd.DataFrame else X
        Xtv = host_matrix(X_test) if type(X_test) == pd.DataFrame else X_test
        self.model._resident = {}
        try:
            for a in (Xv, Xtv):
                if id(a) not in self.model._resident:
                    self.model._resident[id(a)] = (a, self.model._design(a))
            self.fit(Xv, y, *args)
            if verbose > 1:
                print(f'Done with: {self.kwargs} — {id_fit} — in {time.time() - start}')
            cv_coefs[:, iter_cv] = self.coef_
            cv_intercepts[iter_cv] = self.intercept_
            cv_scores_train[iter_cv] = self.score(Xv, y)
            cv_scores_test[iter_cv] = self.score(Xtv, y_test)
            residuals, mean_residuals = self.get_residuals(Xtv, y_test)
        finally:
            self.model._resident = None
        resids.append(residuals)
        mean_resids.append(mean_residuals)

    def get_residuals(self, X: Union[np.ndarray, pd.DataFrame],
                      y: Union[np.ndarray, pd.Series]) -> Tuple[np.ndarray, np.ndarray]:
        residuals = (y - self.predict(X))
        mean_residuals = (y - np.mean(y))
        return residuals, mean_residuals

    def predict(self, X: Union[np.ndarray, pd.DataFrame]) -> np.ndarray:
        if type(X) == pd.DataFrame:
            X = host_matrix(X)
        return self.model.predict(X)          # a lagged frame (sglm_hip.lagframe) stays resident

    def log_likelihood(self, prediction, truth) -> float:
        """backend/sglm.py:349-385 (Gaussian only, as in the reference)."""
        if self.model_name in {'Normal', 'Gaussian'}:
            resid = truth - prediction
            std = np.std(resid)
            return np.sum(scipy.stats.norm.logpdf(resid, loc=0, scale=std))
        raise NotYetImplementedError(self.model_name)


def calc_R2(residuals: np.ndarray, mean_residuals: np.ndarray) -> float:
    """backend/sglm.py:388-408."""
    rss = np.sum(residuals ** 2)
    tss = np.sum(mean_residuals ** 2)
    if tss == 0:
        return 0
    return 1 - rss / tss


def fit_GLM(X, y, model_name='Gaussian', *args, **kwargs):
    """Fit a GLM (sglm/sglm/models/sglm.py:461-485; backend/sglm_ez.py:149-171)."""
    glm = GLM(model_name, *args, **kwargs)
    glm.fit(X, y)
    return glm
