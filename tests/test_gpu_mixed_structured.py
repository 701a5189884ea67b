"""The mixed event design on the structured-Gram path (what ``bench.py --config c4mixed`` times),
at 200,000 rows: 50 events x 40 lags (0/1, the C4 layout) + the production design's two
unshifted continuous counters (cumcount^2 / 5000, pp_design_mat.py:167-172; the design
sglm_cb_concat_make_design_mat.py:224-244, 310 fits), Poisson/log.

Path under test: ``Design.from_events(E, ..., extra=counters)`` -> a mixed design (bit-planes for
the lag block, the counters as a float64 block at their own positions, the ones column after
them) -> every Hessian of the grid from ``sglm_lag_gram_w`` over the events (the ones column
index passed as ``pones``) with the continuous rows / columns written from the float64 block
afterwards (``engine._mix_hess``); ``LAG_GRAM_W_MIXED`` is on by default.  The reference's fit
is sklearn TweedieRegressor(power=1, alpha) inside backend/sglm.py:112-115 / 241, so parity is
to the exact minimiser of the same objective:

* every fit of a 5-split x 20-lambda grid (+ 20 refits) converged, and its float64 Newton
  distance |H^-1 g|_inf -- g and H in float64 from the dense design INCLUDING the counters, on
  the device -- is <= 1e-5 of max|coef| (intercept: <= 1e-5 max(1, |b|));
* one split fit against the float64 CPU oracle (oracle/glm_ref.fit_tweedie_newton) at 1e-4;
* the Hessian the structured path forms (lag block from the events, continuous rows from the
  float64 block) against the float64 Gram X^T diag(w) X of the dense design, within f32
  summation noise (the lag and ones columns among themselves with w rounded to bf16, as both
  Gram kernels round it; the continuous rows with w exact, as _mix_hess forms them).
"""
import numpy as np
import pandas as pd
import pytest

from oracle import glm_ref

pytestmark = pytest.mark.gpu
LAMS = tuple(float(a) for a in np.logspace(-4, 1, 20))


def _dense(s, extra, torch):
    """float64 device design: lag columns, the two counters, the ones column (the engine's
    column order: coefficients come back in it)."""
    m = s.E.shape[1]
    k = extra.shape[0]
    Ed = torch.from_numpy(s.E).cuda().to(torch.float64)
    Xd = torch.empty((s.N, s.p + k + 1), dtype=torch.float64, device="cuda")
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        Xd[:, bi * m:(bi + 1) * m] = Ed[r0 - sh:r0 - sh + s.N]
    Xd[:, s.p:s.p + k] = torch.from_numpy(extra.T).cuda()
    Xd[:, -1] = 1.0
    return Xd


@pytest.fixture(scope="module")
def mixed200(engine):
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    s = synth.make(N=200_000, m=50, L=20, family="poisson", rho=0.02, seed=4)
    extra = synth.prod_counters(s.trial, seed=1)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, extra=extra)
    assert d.k == 2 and d.cont is not None and d.p == s.p + 2
    assert E.LAG_GRAM_W_MIXED and E._lagw(d) is not None
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, a, "n", True, 100) for a in LAMS]
    launches = []
    orig = E._lag_gram_w

    def counted(dd, lg, bf, fits, st, ev=None):
        launches.append(int(np.asarray(fits).size))
        return orig(dd, lg, bf, fits, st, ev)

    E._lag_gram_w = counted
    try:
        st = E.IrlsStats()
        res = grid.run(d, s.y, cv_idx, objs, [0] * len(LAMS), stats=st)
    finally:
        E._lag_gram_w = orig
    return s, extra, d, cv_idx, res, st, launches


def test_mixed_grid_takes_the_structured_gram(mixed200):
    s, extra, d, cv_idx, res, st, launches = mixed200
    assert launches and sum(launches) == st.gram_fits - st.lag_grams, (launches, st.gram_fits)
    for r in res:
        assert r["converged"], r["n_iter"]
    assert st.stops["stagnation"] == 0 and st.stops["line_search_failed"] == 0, st.stops


def test_mixed_grid_newton_distance_every_fit(mixed200):
    import torch
    s, extra, d, cv_idx, res, st, launches = mixed200
    Xd = _dense(s, extra, torch)
    yd = torch.from_numpy(s.y).cuda()
    n, pa = Xd.shape
    masks = []
    for k in range(5):
        mk = torch.zeros(n, dtype=torch.float64, device="cuda")
        mk[torch.from_numpy(np.asarray(cv_idx[k][0])).cuda()] = 1.0
        masks.append(mk)
    masks.append(torch.ones(n, dtype=torch.float64, device="cuda"))
    worst, checked = 0.0, 0
    for j, alpha in enumerate(LAMS):
        r = res[j]
        fits = [(r["cv_coefs"][:, k], r["cv_intercepts"][k]) for k in range(5)]
        fits.append((r["refit_coef"], r["refit_intercept"]))
        for k, (coef, b) in enumerate(fits):
            assert coef.shape == (pa - 1,)
            mk = masks[k]
            beta = torch.from_numpy(np.r_[coef, b]).cuda()
            wmu = mk * torch.exp(Xd @ beta)
            pen = torch.full((pa,), alpha * float(mk.sum()), dtype=torch.float64, device="cuda")
            pen[-1] = 0.0
            g = Xd.t() @ (wmu - mk * yd) + pen * beta
            H = Xd.t() @ (Xd * wmu[:, None])
            H.diagonal().add_(pen)
            step = torch.linalg.solve(H, g)
            dist = float(step[:-1].abs().max()) / float(beta[:-1].abs().max())
            dist_b = float(step[-1].abs()) / max(1.0, abs(float(b)))
            worst = max(worst, dist)
            checked += 1
            assert dist <= 1e-5, (j, alpha, k, dist)
            assert dist_b <= 1e-5, (j, alpha, k, dist_b)
    assert checked == 120
    print(f"mixed 200k: worst float64 Newton distance {worst:.2e} over 120 fits")


def test_mixed_split_fit_vs_oracle(mixed200):
    import torch
    s, extra, d, cv_idx, res, st, launches = mixed200
    j = 5
    tr = np.asarray(cv_idx[0][0])
    Xa = _dense(s, extra, torch)[torch.from_numpy(tr).cuda()].cpu().numpy()
    c, b = glm_ref.fit_tweedie_newton(Xa, s.y[tr], LAMS[j], 1.0, tol=1e-10, max_iter=50,
                                      augmented=True)
    got = res[j]["cv_coefs"][:, 0]
    assert np.max(np.abs(got - c)) / np.max(np.abs(c)) < 1e-4
    assert abs(res[j]["cv_intercepts"][0] - b) < 1e-4 * max(1.0, abs(b))


def test_mixed_structured_hessian_vs_float64_gram(mixed200, monkeypatch):
    """H[k] = X^T diag(w_k) X from the structured path (lag and ones block from the events with
    bf16(w), continuous rows and columns from the float64 block with w exact) against float64."""
    import torch
    from types import SimpleNamespace
    from sglm_hip import engine as E
    s, extra, d, cv_idx, res, st, launches = mixed200
    monkeypatch.setattr(E, "_lagw_pays", lambda dd, lg, nact: True)
    fits = np.array([1, 3, 4], dtype=np.int32)
    rng = np.random.default_rng(2)
    W = torch.zeros((5, d.ld), dtype=torch.float32, device="cuda")
    for k in fits:
        W[k, :d.n] = torch.from_numpy(((rng.random(d.n) < 0.8)
                                       * np.exp(rng.normal(-1, 0.7, d.n))).astype(np.float32))
    bf = SimpleNamespace(W=W, H=torch.zeros((5, d.P, d.P), device="cuda"), prob=None)
    E._syrk(d, bf, fits, 0, 0, None, 0, exact=True)
    torch.cuda.synchronize()
    Xd = _dense(s, extra, torch)
    pl, pa = s.p, Xd.shape[1]
    for k in fits:
        w = W[k, :d.n].to(torch.float64)
        wb = W[k, :d.n].to(torch.bfloat16).to(torch.float64)
        # continuous rows / columns: exact weights; the lag and ones columns among themselves:
        # bf16 weights (the Gram kernels' rounding)
        Hx = Xd.t() @ (Xd * w[:, None])
        lo = torch.cat([torch.arange(pl, device="cuda"), torch.tensor([pa - 1], device="cuda")])
        Xl = Xd[:, lo]
        Hx[lo[:, None], lo[None, :]] = Xl.t() @ (Xl * wb[:, None])
        # the engine's layout: design column c at row / column c, the ones column at d.p
        Hg = bf.H[k][:pa, :pa].to(torch.float64)
        iu = torch.triu_indices(pa, pa, device="cuda")
        a, b = Hg[iu[0], iu[1]], Hx[iu[0], iu[1]]
        assert torch.isfinite(a).all()
        err = float((a - b).abs().max()) / float(b.abs().max())
        assert err <= 2e-6, (int(k), err)
