"""Float64 CPU restatement of the GLM objectives the reference fits — TEST INFRASTRUCTURE.

The reference (``backend/sglm.py:95-130``) hands every fit to a scikit-learn estimator;
the arithmetic therefore lives in sklearn (pinned ``scikit_learn==0.24.2`` at
``requirements.txt:7``; this container has 1.7.2 — the minimisers are identical, only the
lbfgs path differs).  This module restates those objectives:

* Gaussian, ``alpha == 0``  -> ``LinearRegression``: centred min-norm least squares
  (``sklearn/linear_model/_base.py:701``, scipy ``lstsq``/gelsd).
* Gaussian, ``l1_ratio == 0`` -> ``Ridge``: ``||y - Xw - b||^2 + alpha ||w||^2`` on centred
  data, no 1/n (``sklearn/linear_model/_ridge.py:201-213``).
* Poisson / Gamma / Tweedie -> ``TweedieRegressor``:
  ``mean_i loss(y_i, eta_i) + alpha/2 ||w||^2`` with the half-Tweedie losses of
  ``sklearn/_loss/loss.py`` and ``link='auto'`` (log for power > 0, identity otherwise)
  (``sklearn/linear_model/_glm/glm.py:172-322``, ``_linear_loss.py:37-54``).
  Solved here by damped Newton with sklearn's Armijo constants
  (``sklearn/linear_model/_glm/_newton_solver.py:201-260``) to tight tolerance, i.e. the
  minimiser the reference's lbfgs approaches.
* Lasso / ElasticNet -> ``1/(2n)||y - Xw - b||^2 + a*rho*|w|_1 + a(1-rho)/2 ||w||^2``
  (``sklearn/linear_model/_coordinate_descent.py:420-422``), cyclic coordinate descent on
  centred data.

Everything here is float64 and deliberately simple; it is the checker and the CPU
baseline, never the product.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import scipy.linalg


# ----------------------------------------------------------------------------- losses
def tweedie_link_is_log(power: float, link: str = "auto") -> bool:
    """``TweedieRegressor._get_loss`` (sklearn glm.py:898-911)."""
    if link == "auto":
        return power > 0
    return link == "log"


def half_loss(power: float, log_link: bool, y: np.ndarray, eta: np.ndarray):
    """Per-sample half-Tweedie loss (without its y-only constant), d/d eta, d2/d eta2.

    HalfSquaredError: 0.5 (eta - y)^2; HalfPoisson: exp(eta) - y eta;
    HalfGamma: eta + y exp(-eta); HalfTweedie(p): exp((2-p)eta)/(2-p) - y exp((1-p)eta)/(1-p)
    (sklearn/_loss/loss.py HalfTweedieLoss / HalfTweedieLossIdentity).
    """
    y = np.asarray(y, dtype=np.float64)
    eta = np.asarray(eta, dtype=np.float64)
    if not log_link:
        if power == 0:
            r = eta - y
            return 0.5 * r * r, r, np.ones_like(eta)
        # identity link, power != 0 (HalfTweedieLossIdentity)
        p = power
        mu = eta
        if p == 1:
            loss = mu - y * np.log(mu)
            return loss, 1 - y / mu, y / mu ** 2
        if p == 2:
            loss = np.log(mu) + y / mu
            return loss, 1 / mu - y / mu ** 2, -1 / mu ** 2 + 2 * y / mu ** 3
        loss = mu ** (2 - p) / (2 - p) - y * mu ** (1 - p) / (1 - p)
        g = mu ** (1 - p) - y * mu ** (-p)
        h = (1 - p) * mu ** (-p) + p * y * mu ** (-p - 1)
        return loss, g, h
    if power == 0:
        mu = np.exp(eta)
        loss = 0.5 * (mu - y) ** 2
        return loss, (mu - y) * mu, (2 * mu - y) * mu
    if power == 1:
        mu = np.exp(eta)
        return mu - y * eta, mu - y, mu
    if power == 2:
        e = np.exp(-eta)
        return eta + y * e, 1 - y * e, y * e
    p = power
    a = np.exp((2 - p) * eta)
    b = np.exp((1 - p) * eta)
    loss = a / (2 - p) - y * b / (1 - p)
    return loss, a - y * b, (2 - p) * a - (1 - p) * y * b


def loss_constant(power: float, y: np.ndarray) -> np.ndarray:
    """``constant_to_optimal_zero`` of the half-Tweedie losses (sklearn/_loss/loss.py)."""
    y = np.asarray(y, dtype=np.float64)
    if power == 0:
        return -0.5 * y * y
    if power == 1:
        with np.errstate(divide="ignore", invalid="ignore"):
            ylogy = np.where(y > 0, y * np.log(np.where(y > 0, y, 1.0)), 0.0)
        return ylogy - y
    if power == 2:
        return -np.log(y) - 1
    p = power
    return np.power(np.maximum(y, 0), 2 - p) / (1 - p) / (2 - p)


def inverse_link(log_link: bool, eta):
    return np.exp(eta) if log_link else eta


# ----------------------------------------------------------------------------- specs
@dataclass
class FitSpec:
    """What ``GLM.__init__`` (backend/sglm.py:95-130) selects, reduced to an objective."""
    kind: str                 # 'ols' | 'ridge' | 'lasso' | 'enet' | 'tweedie'
    alpha: float = 1.0
    l1_ratio: float = 0.0
    power: float = 0.0
    link: str = "auto"
    fit_intercept: bool = True
    max_iter: int = 100
    tol: float = 1e-4


def spec_from_glm_kwargs(model_name: str, kwargs: dict) -> FitSpec:
    """Restates the estimator dispatch of ``backend/sglm.py:91-130`` (kwargs not mutated)."""
    kw = dict(kwargs)
    kw.pop("warm_start", None)
    fi = kw.get("fit_intercept", True)
    if model_name in ("Normal", "Gaussian"):
        if "alpha" in kw and kw["alpha"] == 0:
            return FitSpec("ols", alpha=0.0, fit_intercept=fi)
        alpha = kw.get("alpha", 1.0)
        if "l1_ratio" in kw and kw["l1_ratio"] == 0:
            return FitSpec("ridge", alpha=alpha, fit_intercept=fi,
                           max_iter=kw.get("max_iter", None) or 0, tol=kw.get("tol", 1e-4))
        if "l1_ratio" in kw and kw["l1_ratio"] == 1:
            return FitSpec("lasso", alpha=alpha, l1_ratio=1.0, fit_intercept=fi,
                           max_iter=kw.get("max_iter", 1000), tol=kw.get("tol", 1e-4))
        return FitSpec("enet", alpha=alpha, l1_ratio=kw.get("l1_ratio", 0.5), fit_intercept=fi,
                       max_iter=kw.get("max_iter", 1000), tol=kw.get("tol", 1e-4))
    if model_name in ("Poisson", "Gamma", "Tweedie"):
        power = {"Poisson": 1.0, "Gamma": 2.0}.get(model_name, kw.get("power", 0.0))
        return FitSpec("tweedie", alpha=kw.get("alpha", 1.0), power=power,
                       link=kw.get("link", "auto"), fit_intercept=fi,
                       max_iter=kw.get("max_iter", 100), tol=kw.get("tol", 1e-4))
    raise NotImplementedError(model_name)


# ----------------------------------------------------------------------------- solvers
def _augment(X, fit_intercept):
    X = np.asarray(X, dtype=np.float64)
    if fit_intercept:
        return np.hstack([X, np.ones((X.shape[0], 1))])
    return X


def fit_ols(X, y, fit_intercept=True):
    """``LinearRegression.fit`` dense path: centre, scipy lstsq (min-norm), intercept."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    cond = max(X.shape) * np.finfo(np.float64).eps      # _base.py:699-701 cut-off
    if fit_intercept:
        xm = X.mean(axis=0)
        ym = y.mean()
        coef = scipy.linalg.lstsq(X - xm, y - ym, cond=cond)[0]
        return coef, float(ym - xm @ coef)
    return scipy.linalg.lstsq(X, y, cond=cond)[0], 0.0


def fit_ols_chunks(chunks, fit_intercept=True):
    """``LinearRegression.fit`` for a design too large to hold densely: float64 sums of
    [X, 1]^T [X, 1] and [X, 1]^T y over row chunks ((X_chunk, y_chunk) pairs), then the
    centred normal equations solved by scipy lstsq on the Gram (the same minimiser as the dense
    lstsq of ``fit_ols`` for a full-rank design; test infrastructure for full-size grids)."""
    G = c = None
    n = 0.0
    for Xc, yc in chunks:
        Xc = np.asarray(Xc, dtype=np.float64)
        Xa = np.hstack([Xc, np.ones((Xc.shape[0], 1))])
        g, cc = Xa.T @ Xa, Xa.T @ np.asarray(yc, dtype=np.float64)
        G, c = (g, cc) if G is None else (G + g, c + cc)
        n += Xc.shape[0]
    p = G.shape[0] - 1
    if not fit_intercept:
        return scipy.linalg.lstsq(G[:p, :p], c[:p])[0], 0.0
    xm, ym = G[:p, p] / n, c[p] / n
    Gc = G[:p, :p] - n * np.outer(xm, xm)
    cc = c[:p] - n * xm * ym
    coef = scipy.linalg.lstsq(Gc, cc)[0]
    return coef, float(ym - xm @ coef)


def fit_ridge(X, y, alpha, fit_intercept=True):
    """``Ridge`` cholesky solver on centred data (sklearn/_ridge.py:201-213)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if fit_intercept:
        xm = X.mean(axis=0)
        ym = y.mean()
        Xc, yc = X - xm, y - ym
    else:
        xm, ym, Xc, yc = np.zeros(X.shape[1]), 0.0, X, y
    A = Xc.T @ Xc
    A[np.diag_indices_from(A)] += alpha
    coef = scipy.linalg.solve(A, Xc.T @ yc, assume_a="pos")
    return coef, float(ym - xm @ coef) if fit_intercept else 0.0


def weighted_gram(Xa, h, chunk=65536):
    """Xa^T diag(h) Xa in float64.  For h >= 0 it is accumulated over row chunks with BLAS
    dsyrk on sqrt(h)-scaled rows (half the flops of a GEMM and no n x p' temporary: the
    full-size checks run this on a 1M x 2001 design); otherwise a plain GEMM."""
    n, pa = Xa.shape
    if np.any(h < 0):
        return (Xa * h[:, None]).T @ Xa
    from scipy.linalg.blas import dsyrk
    H = np.zeros((pa, pa))
    for i in range(0, n, chunk):
        A = Xa[i:i + chunk] * np.sqrt(h[i:i + chunk])[:, None]
        # A is C-ordered (rows x pa), so A.T is a Fortran (pa x rows) array: dsyrk(trans=0)
        # forms A.T @ A (upper triangle) without a copy
        H = dsyrk(1.0, A.T, beta=1.0, c=H, trans=0, lower=0, overwrite_c=1)
    return np.triu(H) + np.triu(H, 1).T


def null_space(Xa):
    """Orthonormal basis of null(Xa) (float64): right singular vectors whose singular value
    is below lstsq's cut-off max(n, p) eps sigma_max (sklearn _base.py:699-701); for tall
    designs the eigenvectors of Xa^T Xa below the squared cut-off."""
    n, pa = Xa.shape
    cut = max(n, pa) * np.finfo(np.float64).eps
    if n * pa <= 5e7:
        _, sv, vt = np.linalg.svd(Xa, full_matrices=False)
        return vt[sv <= cut * sv[0]].T
    ev, V = np.linalg.eigh(Xa.T @ Xa)
    return V[:, ev <= max(cut * cut, 1e-13) * ev[-1]]


def min_norm(Xa, coef, fit_intercept):
    """The minimum-|w| point (w: the coefficients, not the intercept) of the solution set
    coef + null(Xa): lstsq's answer on a rank-deficient design (centred lstsq = min |w| over
    the same set), and the limit of lbfgs from w = 0, which stays in the row space."""
    live = np.flatnonzero(np.any(Xa != 0.0, axis=0))    # all-zero columns keep their 0
    N = null_space(Xa[:, live])
    if N.shape[1] == 0:
        return coef
    nw = live.size - 1 if (fit_intercept and live[-1] == Xa.shape[1] - 1) else live.size
    c = np.linalg.lstsq(N[:nw], coef[live[:nw]], rcond=None)[0]
    out = coef.copy()
    out[live] -= N @ c
    return out


def fit_tweedie_newton(X, y, alpha, power, link="auto", fit_intercept=True,
                       tol=1e-12, max_iter=200, coef0=None, return_iters=False,
                       augmented=False):
    """Damped Newton on ``mean_i loss_i + alpha/2 ||w||^2`` (sklearn glm.py:172-322).

    Start: w = 0, b = link(mean y) (glm.py:247-259).  Armijo backtracking with sklearn's
    constants beta = 1/2, sigma = 2^-11 (_newton_solver.py:214).  Stops when the Newton
    step is below ``tol * (1 + |coef|_inf)`` or ``max|grad| <= tol`` (criterion 1 of
    _newton_solver.py:323-330).  Rank-deficient Hessians (alpha = 0 with all-zero
    columns) fall back to the minimum-norm Newton step, and an unpenalised fit ends at the
    minimum-norm point of its solution set (``min_norm``).  ``augmented``: X already carries
    the intercept's ones column as its LAST column (large designs: no hstack copy).
    """
    y = np.asarray(y, dtype=np.float64)
    if augmented:
        if not fit_intercept:
            raise ValueError("augmented=True implies fit_intercept=True")
        Xa = np.asarray(X, dtype=np.float64)
    else:
        Xa = _augment(X, fit_intercept)
    n, pa = Xa.shape
    log_link = tweedie_link_is_log(power, link)
    pen = np.full(pa, float(alpha))
    if fit_intercept:
        pen[-1] = 0.0
    coef = np.zeros(pa)
    if coef0 is not None:
        coef[:] = coef0
    elif fit_intercept:
        ym = y.mean()
        coef[-1] = math.log(ym) if log_link else ym

    def objective(c, eta=None):
        eta = Xa @ c if eta is None else eta
        return half_loss(power, log_link, y, eta)[0].mean() + 0.5 * np.dot(pen * c, c)

    it = 0
    eta = Xa @ coef
    for it in range(1, max_iter + 1):
        _, g_i, h_i = half_loss(power, log_link, y, eta)
        grad = Xa.T @ g_i / n + pen * coef
        if np.max(np.abs(grad)) <= tol * 1e-3:
            it -= 1
            break
        H = weighted_gram(Xa, h_i) / n
        H[np.diag_indices_from(H)] += pen
        zero = np.diag(H) == 0.0          # all-zero column, alpha = 0: coefficient stays put
        H[zero, zero] = 1.0
        try:
            c, low = scipy.linalg.cho_factor(H)
            step = -scipy.linalg.cho_solve((c, low), grad)
        except np.linalg.LinAlgError:
            step = -scipy.linalg.lstsq(H, grad)[0]
        f0 = objective(coef, eta)
        gs = float(grad @ step)
        d_eta = Xa @ step
        t = 1.0
        for _ in range(40):
            f1 = objective(coef + t * step, eta + t * d_eta)
            if f1 - f0 <= 2.0 ** -11 * t * gs or abs(f1 - f0) <= 1e-16 * abs(f0):
                break
            t *= 0.5
        coef = coef + t * step
        eta = eta + t * d_eta
        if np.max(np.abs(t * step)) <= tol * (1 + np.max(np.abs(coef))):
            break
    if alpha == 0.0:
        coef = min_norm(Xa, coef, fit_intercept)
    if fit_intercept:
        out = coef[:-1].copy(), float(coef[-1])
    else:
        out = coef.copy(), 0.0
    return (out + (it,)) if return_iters else out


def fit_enet_cd(X, y, alpha, l1_ratio, fit_intercept=True, tol=1e-12, max_iter=100000):
    """Cyclic coordinate descent for ElasticNet/Lasso on centred data (cd_fast restated)."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n, p = X.shape
    if fit_intercept:
        xm, ym = X.mean(axis=0), y.mean()
        Xc, yc = X - xm, y - ym
    else:
        xm, ym, Xc, yc = np.zeros(p), 0.0, X, y
    w = fit_enet_cd_gram(Xc.T @ Xc, Xc.T @ yc, n, alpha, l1_ratio, tol, max_iter)
    return w, float(ym - xm @ w) if fit_intercept else 0.0


def fit_enet_cd_gram(G, c, n, alpha, l1_ratio, tol=1e-12, max_iter=100000):
    """The cyclic coordinate descent of ``fit_enet_cd`` given the (centred) Gram G = Xc^T Xc
    and c = Xc^T yc of n rows (cd_fast's precomputed-Gram form); returns w."""
    G = np.asarray(G, dtype=np.float64)
    c = np.asarray(c, dtype=np.float64)
    p = G.shape[0]
    l1 = alpha * l1_ratio * n
    l2 = alpha * (1.0 - l1_ratio) * n
    w = np.zeros(p)
    q = -c.copy()          # = G w - c
    diag = np.diag(G).copy()
    for _ in range(max_iter):
        wmax = dmax = 0.0
        for j in range(p):
            if diag[j] == 0.0:
                continue
            wj = w[j]
            rho = -(q[j] - diag[j] * wj)
            new = np.sign(rho) * max(abs(rho) - l1, 0.0) / (diag[j] + l2)
            if new != wj:
                q += G[:, j] * (new - wj)
                w[j] = new
            dmax = max(dmax, abs(new - wj))
            wmax = max(wmax, abs(new))
        if wmax == 0.0 or dmax / wmax < tol:
            break
    return w


def fit(spec: FitSpec, X, y, tight=True):
    """Fit one spec to (X, y); returns (coef, intercept)."""
    if spec.kind == "ols":
        return fit_ols(X, y, spec.fit_intercept)
    if spec.kind == "ridge":
        return fit_ridge(X, y, spec.alpha, spec.fit_intercept)
    if spec.kind in ("lasso", "enet"):
        return fit_enet_cd(X, y, spec.alpha, spec.l1_ratio, spec.fit_intercept)
    if spec.kind == "tweedie":
        return fit_tweedie_newton(X, y, spec.alpha, spec.power, spec.link, spec.fit_intercept,
                                  tol=1e-12 if tight else spec.tol,
                                  max_iter=200 if tight else spec.max_iter)
    raise NotImplementedError(spec.kind)


def predict(spec: FitSpec, coef, intercept, X):
    eta = np.asarray(X, dtype=np.float64) @ coef + intercept
    if spec.kind == "tweedie":
        return inverse_link(tweedie_link_is_log(spec.power, spec.link), eta)
    return eta


def r2_score(spec: FitSpec, coef, intercept, X, y):
    """``model.score``: R^2 for the Gaussian estimators, D^2 for Tweedie (glm.py:371-444)."""
    y = np.asarray(y, dtype=np.float64)
    eta = np.asarray(X, dtype=np.float64) @ coef + intercept
    if spec.kind != "tweedie":
        ssr = np.sum((y - eta) ** 2)
        sst = np.sum((y - y.mean()) ** 2)
        if sst == 0:
            return 1.0 if ssr == 0 else 0.0
        return 1.0 - ssr / sst
    log_link = tweedie_link_is_log(spec.power, spec.link)
    const = loss_constant(spec.power, y).mean()
    dev = half_loss(spec.power, log_link, y, eta)[0].mean()
    ym = y.mean()
    eta0 = math.log(ym) if log_link else ym
    dev0 = half_loss(spec.power, log_link, y, np.full_like(y, eta0))[0].mean()
    return 1.0 - (dev + const) / (dev0 + const)


def neg_mse_score(spec: FitSpec, coef, intercept, X, y):
    """``GLM.neg_mse_score`` (backend/sglm.py:150-167)."""
    r = np.asarray(y, dtype=np.float64) - predict(spec, coef, intercept, X)
    return -np.mean(r ** 2)


def calc_R2(residuals, mean_residuals):
    """``calc_R2`` (backend/sglm.py:388-408)."""
    rss = np.sum(np.asarray(residuals) ** 2)
    tss = np.sum(np.asarray(mean_residuals) ** 2)
    return 0 if tss == 0 else 1 - rss / tss


def newton_flops(n, p_aug):
    """Algorithmic flop of one IRLS iteration: n p'(p'+1) + 4 n p' + p'^3/3 + 2p'^2."""
    return n * p_aug * (p_aug + 1) + 4 * n * p_aug + p_aug ** 3 / 3 + 2 * p_aug ** 2
