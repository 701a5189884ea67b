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
    """Solve one ElasticNet fit per request; returns (FitResults, eta tensor [B][ld])."""
    d = prob.design
    B, P, ld, n, p = len(reqs), d.P, d.ld, d.n, d.p
    dev = d.device
    st = E._stream()
    bf = E._BUF.get(B, P, ld, dev)
    bf.prob, bf.fit_mask = prob, np.array([r.mask for r in reqs])
    fit_resp = torch.tensor([r.resp for r in reqs], dtype=torch.int32, device=dev)
    fit_mask = torch.tensor([r.mask for r in reqs], dtype=torch.int32, device=dev)
    bf.eta.zero_()
    _lib.call("sglm_link_update", E.FAM_SQUARED, 0.0, n, ld, B, E._p(bf.eta), E._p(prob.Y),
              E._p(prob.M), E._p(fit_resp), E._p(fit_mask), E._p(bf.W), E._p(bf.R), st)
    d.xtr(bf.R, B, bf.g)
    c = -bf.g                                            # X^T (m y)
    # one Gram per distinct mask (W = mask), copied to every fit that uses it
    reps = {}
    for k, r in enumerate(reqs):
        reps.setdefault(r.mask, k)
    rep_idx = np.array(sorted(reps.values()), dtype=np.int32)
    E._syrk(d, bf, rep_idx, (n + 31) // 32, (P // 256) * (P // 256 + 1) // 2, None, st,
            exact=True)
    for k, r in enumerate(reqs):
        rk = reps[r.mask]
        if rk != k:
            bf.H[k].copy_(bf.H[rk])
    cnt = np.array([float(prob.masks[r.mask].astype(np.float64).sum()) for r in reqs])
    l1 = np.array([o.alpha * o.l1_ratio for o in objectives]) * cnt
    l2 = np.array([o.alpha * (1.0 - o.l1_ratio) for o in objectives]) * cnt
    l1d = torch.from_numpy(l1).to(dev)
    l2d = torch.from_numpy(l2).to(dev)
    fi = torch.tensor([int(r.fit_intercept) for r in reqs], dtype=torch.int32, device=dev)
    fits = torch.arange(B, dtype=torch.int32, device=dev)
    coef = torch.zeros((B, P), dtype=torch.float64, device=dev)
    sweeps = torch.zeros(B, dtype=torch.int32, device=dev)
    max_sweeps = int(max(max(o.max_iter for o in objectives), 10000))
    cw = E._work(_lib.query("sglm_enet_work_bytes", p, B), dev)
    _lib.call("sglm_enet_cd", E._p(bf.H), P, p, E._p(fits), B, E._p(c), E._p(l1d), E._p(l2d),
              E._p(fi), max_sweeps, CD_TOL, E._p(coef), E._p(sweeps), E._p(cw), st)
    bf.beta.copy_(coef.to(torch.float32))
    bf.prob = bf.keep = None
    d.eta(bf.beta, bf.eta)
    ch = coef.cpu().numpy()
    sw = sweeps.cpu().numpy()
    res = [E.FitResult(coef=ch[k, :p].copy(), intercept=float(ch[k, p]) if reqs[k].fit_intercept else 0.0,
                       n_iter=int(sw[k]), converged=bool(sw[k] < max_sweeps)) for k in range(B)]
    return res, bf.eta


def enet_fit(prob, objectives, masks, resps, coef0=None):
    reqs = [E.FitReq(E.FAM_SQUARED, 0.0, 0.0, m, r, o.fit_intercept, o.max_iter)
            for o, m, r in zip(objectives, masks, resps)]
    res, _ = enet_batch(prob, objectives, reqs)
    return res
