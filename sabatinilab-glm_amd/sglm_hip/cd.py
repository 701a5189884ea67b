"""Lasso / ElasticNet on the MI355X: MFMA Gram per mask + float64 Gram-space coordinate
descent per fit (sglm_enet_cd).  Replaces sklearn's cd_fast behind backend/sglm.py:106-110.

sklearn stops at its duality-gap tolerance (default tol=1e-4); the engine iterates to
max|dw| <= 1e-10 max|w| (or ``max(max_iter, 10000)`` sweeps) so that results sit at the
minimiser that tight-tolerance sklearn fixtures pin.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from . import engine as E

CD_TOL = 1e-10


def enet_batch(prob: E.Problem, objectives, reqs):
    """Solve one ElasticNet fit per request; returns (FitResults, eta tensor [B][ld]).
    Grams and their centred float64 forms are formed once per distinct mask and shared
    (sglm_hip.enet); X^T(m y) once per distinct (response, mask)."""
    from . import enet
    d = prob.design
    B, P, ld, p = len(reqs), d.P, d.ld, d.p
    bf = E._scratch().buf.get(B, P, ld, d.device)
    grams = enet.SharedGrams(prob)
    pairs = list(dict.fromkeys((r.resp, r.mask) for r in reqs))
    ci = {pm: i for i, pm in enumerate(pairs)}
    c = enet.xty(prob, pairs)
    fits = [{"mask": r.mask, "alpha": o.alpha, "l1_ratio": o.l1_ratio,
             "fit_intercept": r.fit_intercept, "max_iter": max(o.max_iter, 1)}
            for o, r in zip(objectives, reqs)]
    w, b, sw, conv = enet.solve(prob, grams, fits, c, [ci[(r.resp, r.mask)] for r in reqs])
    beta = np.zeros((B, P), dtype=np.float64)
    beta[:, :p] = w
    beta[:, p] = b
    bf.beta.copy_(torch.from_numpy(beta.astype(np.float32)))
    d.eta(bf.beta, bf.eta)
    res = [E.FitResult(coef=w[k].copy(), intercept=float(b[k]) if reqs[k].fit_intercept else 0.0,
                       n_iter=int(sw[k]), converged=bool(conv[k])) for k in range(B)]
    return res, bf.eta


def enet_fit(prob, objectives, masks, resps, coef0=None):
    reqs = [E.FitReq(E.FAM_SQUARED, 0.0, 0.0, m, r, o.fit_intercept, o.max_iter)
            for o, m, r in zip(objectives, masks, resps)]
    res, _ = enet_batch(prob, objectives, reqs)
    return res
