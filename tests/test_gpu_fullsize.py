"""Full-size parity at the BASELINE.json configs the bench runs (C4) and the C5 path at p=2000.

C4 (configs[3]) -- EXACTLY the timed bench configuration: Poisson/log, 1,000,000 rows x 2000
time-shifted 0/1 predictors (P = 2048), trial-id GroupShuffleSplit splits (seed 3), the 20
lambdas np.logspace(-4, 1, 20) x (5 splits + refit) = 120 fits, through ``grid.run`` as
bench.py calls it (bf16 bit-plane Gram, Hessian reuse, lambda-neighbour sharing and
cross-mask aliasing at the default tolerances).  The reference's loop is
cv_glm_single_params per lambda (backend/sglm_cv.py:42-206) with sklearn
TweedieRegressor(power=1) (backend/sglm.py:112-115).  Checks:

* every fit converged on the step criterion (no stagnation / line-search-failure stops), and
  the grid actually exercised the lambda-neighbour sharing chain and cross-mask aliasing;
* every fit's float64 Newton distance |H^-1 g|_inf to the minimiser, with g and H formed in
  float64 from the exact design on the device (torch float64, the property checker, not the
  product), is <= 1e-5 of max|beta| -- ten times inside the north-star Poisson bar (1e-4) --
  for ALL 120 fits;
* against the float64 CPU oracle (oracle/glm_ref.fit_tweedie_newton, damped Newton to 1e-10)
  at 1e-4 relative: split 0 and the refit at lambda index 0 (the ill-conditioned end), and the
  split-0 fits at lambda index 5 and 12 (mid-path, where the sharing chain hands Hessians from
  neighbour to neighbour);
* the grid cut into 8 rank shares (grid.run(..., simulate=(r, 8)): each share solved as a rank
  of an 8-GPU run solves it) merges to the unsharded grid at 1e-5.

C5 (configs[4] path): Gaussian elastic net l1_ratio 0.5 through ``enet.cv_enet_path`` at
p = 2000 (200k rows, 3 responses x 3 alphas x (5 splits + refit)), so the coordinate-descent
kernel runs its multi-coordinate-per-thread path (8 coordinates per thread): every fit's
float64 KKT residual on the device, and four fits against the oracle CD at 1e-5.
"""
import time

import numpy as np
import pandas as pd
import pytest

from oracle import glm_ref

pytestmark = pytest.mark.gpu
TOL_POIS, TOL_GAUSS = 1e-4, 1e-5
LAMS_C4 = tuple(float(a) for a in np.logspace(-4, 1, 20))     # bench.py's grid


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _host_augmented(s):
    """Dense float64 X with the ones column last (N x p+1), host."""
    m = s.E.shape[1]
    Xa = np.empty((s.N, s.p + 1))
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        Xa[:, bi * m:(bi + 1) * m] = s.E[r0 - sh:r0 - sh + s.N]
    Xa[:, s.p] = 1.0
    return Xa


def _device_augmented(s, torch):
    m = s.E.shape[1]
    Ed = torch.from_numpy(s.E).cuda().to(torch.float64)
    Xd = torch.empty((s.N, s.p + 1), dtype=torch.float64, device="cuda")
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        Xd[:, bi * m:(bi + 1) * m] = Ed[r0 - sh:r0 - sh + s.N]
    Xd[:, s.p] = 1.0
    return Xd


def _objectives(E):
    from sglm_hip.estimators import Objective
    return [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, a, "n", True, 100) for a in LAMS_C4]


@pytest.fixture(scope="module")
def c4(engine):
    from sglm_hip import engine as E, folds, grid, synth
    t0 = time.time()
    s = synth.make(N=1_000_000, m=50, L=20, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    assert d.P == 2048
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    st = E.IrlsStats()
    res = grid.run(d, s.y, cv_idx, _objectives(E), [0] * len(LAMS_C4), stats=st)
    print(f"c4 grid: {time.time() - t0:.1f} s, stops {st.stops}, grams {st.gram_fits}, "
          f"kept {st.reused}, shared {st.shared}, aliased {st.aliased}")
    return s, d, cv_idx, res, st


def test_c4_grid_converged_on_step_criterion(c4):
    s, d, cv_idx, res, st = c4
    assert len(res) == 20
    for r in res:
        assert r["converged"], r["n_iter"]
        assert len(r["n_iter"]) == 6
    assert st.stops["stagnation"] == 0 and st.stops["line_search_failed"] == 0, st.stops
    assert st.stops["max_iter"] == 0, st.stops
    # the timed configuration's approximate-Hessian paths all ran
    assert st.shared > 0 and st.aliased > 0 and st.reused > 0, (st.shared, st.aliased, st.reused)


def test_c4_newton_distance_float64_every_fit(c4):
    """The float64 Newton step s = H^-1 g to the exact minimiser, for all 120 fits, float64 on
    the device: coefficients max|s_j| <= 1e-5 max|beta_j| (j < p, the relative measure of the
    north-star bar), intercept |s_p| <= 1e-5 max(1, |b|) (the intercept bar of every parity
    test here).  The intercept is kept apart: at strong penalties the coefficients shrink to
    ~1e-3 while the intercept stays O(1), so a 1e-8 intercept offset (f32 predictor rounding)
    divided by max|coef| would measure nothing about the coefficients."""
    import torch
    s, d, cv_idx, res, st = c4
    Xd = _device_augmented(s, torch)
    yd = torch.from_numpy(s.y).cuda()
    n, pa = Xd.shape
    masks = []
    for k in range(5):
        m = torch.zeros(n, dtype=torch.float64, device="cuda")
        m[torch.from_numpy(np.asarray(cv_idx[k][0])).cuda()] = 1.0
        masks.append(m)
    masks.append(torch.ones(n, dtype=torch.float64, device="cuda"))
    worst, worst_b, checked = 0.0, 0.0, 0
    for j, alpha in enumerate(LAMS_C4):
        r = res[j]
        fits = [(r["cv_coefs"][:, k], r["cv_intercepts"][k]) for k in range(5)]
        fits.append((r["refit_coef"], r["refit_intercept"]))
        for k, (coef, b) in enumerate(fits):
            m = masks[k]
            cnt = float(m.sum())
            beta = torch.from_numpy(np.r_[coef, b]).cuda()
            wmu = m * torch.exp(Xd @ beta)
            pen = torch.full((pa,), alpha * cnt, dtype=torch.float64, device="cuda")
            pen[-1] = 0.0
            g = Xd.t() @ (wmu - m * yd) + pen * beta             # sum-objective gradient
            H = Xd.t() @ (Xd * wmu[:, None])
            H.diagonal().add_(pen)
            step = torch.linalg.solve(H, g)
            dist = float(step[:-1].abs().max()) / float(beta[:-1].abs().max())
            dist_b = float(step[-1].abs()) / max(1.0, abs(float(b)))
            worst = max(worst, dist)
            worst_b = max(worst_b, dist_b)
            checked += 1
            assert dist <= 1e-5, (j, alpha, k, dist)
            assert dist_b <= 1e-5, (j, alpha, k, dist_b)
            del H, wmu, g
    assert checked == 120
    print(f"c4 worst float64 Newton distance over 120 fits: coefficients {worst:.2e} of "
          f"max|coef|, intercept {worst_b:.2e}")


@pytest.fixture(scope="module")
def c4_host(c4):
    s = c4[0]
    return _host_augmented(s)


@pytest.mark.parametrize("j", [0, 5, 12])
def test_c4_split_fit_vs_oracle(c4, c4_host, j):
    """Split 0 (800k train rows) at lambda index j vs the float64 oracle."""
    s, d, cv_idx, res, st = c4
    tr = np.asarray(cv_idx[0][0])
    t0 = time.time()
    c, b = glm_ref.fit_tweedie_newton(c4_host[tr], s.y[tr], LAMS_C4[j], 1.0, tol=1e-10,
                                      max_iter=50, augmented=True)
    print(f"oracle split fit (lambda {LAMS_C4[j]:.3g}) {time.time() - t0:.1f} s")
    assert rel(res[j]["cv_coefs"][:, 0], c) < TOL_POIS
    assert abs(res[j]["cv_intercepts"][0] - b) < TOL_POIS * max(1.0, abs(b))


def test_c4_refit_vs_oracle(c4, c4_host):
    """The full-data refit at lambda = 1e-4 (1M rows) vs the float64 oracle."""
    s, d, cv_idx, res, st = c4
    t0 = time.time()
    c, b = glm_ref.fit_tweedie_newton(c4_host, s.y, LAMS_C4[0], 1.0, tol=1e-10, max_iter=50,
                                      augmented=True)
    print(f"oracle refit {time.time() - t0:.1f} s")
    assert rel(res[0]["refit_coef"], c) < TOL_POIS
    assert abs(res[0]["refit_intercept"] - b) < TOL_POIS * max(1.0, abs(b))


def test_c4_eight_rank_shares_merge_to_the_unsharded_grid(c4):
    """The timed grid cut into 8 rank shares, each solved exactly as a rank of the 8-GPU run
    solves it, merged (grid.merge_results' input) and assembled == the unsharded grid."""
    from sglm_hip import engine as E, grid
    s, d, cv_idx, full, st = c4
    objs = _objectives(E)
    rolls = [0] * len(objs)
    groups = [{"cv_idx": cv_idx, "objectives": objs, "rolls": rolls}]
    plan = grid.plan_fits(groups, s.N)
    merged, seen = {}, []
    for r in range(8):
        share = grid.run(d, s.y, cv_idx, objs, rolls, simulate=(r, 8))
        assert sorted(share) == grid.rank_share(plan, groups, r, 8)
        seen += list(share)
        merged.update(share)
    assert sorted(seen) == list(range(120))
    out = grid.assemble(groups, plan, merged, s.p)[0]
    for a, b in zip(out, full):
        assert a["converged"] and b["converged"]
        assert rel(a["cv_coefs"], b["cv_coefs"]) < 1e-5
        assert rel(a["cv_intercepts"], b["cv_intercepts"]) < 1e-5
        assert rel(a["refit_coef"], b["refit_coef"]) < 1e-5
        assert np.max(np.abs(a["cv_scores_test"] - b["cv_scores_test"])) < 1e-6


def test_chol_solve_p2048_lookahead_chain(engine):
    """Blocked Cholesky at P = 2048 (32 block steps, look-ahead depth 4), the C4 size:
    factor + solve, kept-factor re-solve and the mixed chain, vs float64 numpy."""
    import torch
    from sglm_hip import _lib
    rng = np.random.default_rng(2048)
    P, B, pa = 2048, 3, 2001
    H = np.zeros((B, P, P), np.float32)
    g = np.zeros((B, P))
    Ms = []
    for k in range(B):
        A = rng.normal(size=(6000, pa)) * (1.0 + k)
        M = A.T @ A
        H[k, :pa, :pa] = M
        g[k, :pa] = rng.normal(size=pa)
        Ms.append(M)
    dsh = np.full((B, P), -1.0, np.float32)
    dsh[:, :pa - 1] = 50.0
    dsh[:, pa - 1] = 0.0
    pen = np.r_[np.full(pa - 1, 50.0), 0.0]
    Hd = torch.from_numpy(H).cuda()
    gd = torch.from_numpy(g).cuda()
    dshd = torch.from_numpy(dsh).cuda()
    out = torch.zeros((B, P), dtype=torch.float32, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
    fits = torch.tensor([2, 0, 1], dtype=torch.int32, device="cuda")
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8, device="cuda")
    _lib.call("sglm_chol_solve_ex", Hd.data_ptr(), P, fits.data_ptr(), B, gd.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), 1, B,
              cw.data_ptr(), 0)
    x = out.cpu().numpy()
    assert np.all(info.cpu().numpy() == 0)
    for k in range(B):
        ref = -np.linalg.solve(Ms[k] + np.diag(pen), g[k, :pa])
        assert rel(x[k, :pa], ref) < 1e-3, k
        assert np.all(x[k, pa:] == 0)
    # kept factors, new right-hand sides
    g2 = np.zeros((B, P))
    g2[:, :pa] = rng.normal(size=(B, pa))
    g2d = torch.from_numpy(g2).cuda()
    _lib.call("sglm_chol_solve_ex", Hd.data_ptr(), P, fits.data_ptr(), B, g2d.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), 0, B,
              cw.data_ptr(), 0)
    x2 = out.cpu().numpy()
    for k in range(B):
        assert rel(x2[k, :pa], -np.linalg.solve(Ms[k] + np.diag(pen), g2[k, :pa])) < 1e-3, k
    # mixed chain: fit 1 refactored from a new matrix, fits 0 and 2 keep their factors
    A1 = rng.normal(size=(6000, pa))
    M1 = A1.T @ A1
    H1 = np.zeros((P, P), np.float32)
    H1[:pa, :pa] = M1
    Hd[1].copy_(torch.from_numpy(H1))
    order = torch.tensor([1, 0, 2], dtype=torch.int32, device="cuda")
    _lib.call("sglm_chol_solve_mixed", Hd.data_ptr(), P, order.data_ptr(), B, 1, g2d.data_ptr(),
              dshd.data_ptr(), out.data_ptr(), info.data_ptr(), frozen.data_ptr(), B,
              cw.data_ptr(), 0)
    x3 = out.cpu().numpy()
    for k, M in ((0, Ms[0]), (1, M1), (2, Ms[2])):
        assert rel(x3[k, :pa], -np.linalg.solve(M + np.diag(pen), g2[k, :pa])) < 1e-3, k


ALPHAS_C5 = (1e-3, 1e-2, 1e-1)


@pytest.fixture(scope="module")
def c5(engine):
    from sglm_hip import engine as E, enet, folds, synth
    t0 = time.time()
    s = synth.make(N=200_000, m=50, L=20, family="gaussian", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(5)
    Y = np.stack([s.y + rng.normal(0, 1, s.N) for _ in range(3)], 1)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    st = {}
    out = enet.cv_enet_path(d, Y, cv_idx, ALPHAS_C5, l1_ratio=0.5, max_iter=1000, stats=st)
    print(f"c5 path: {time.time() - t0:.1f} s, {st}")
    return s, Y, cv_idx, out, st


def test_c5_enet_kkt_float64_every_fit(c5):
    """ElasticNet optimality (sklearn objective, _coordinate_descent.py:420-422) for all 54
    fits in float64 on the device: with r = m (y - Xw - b) and c = X^T r / n_m,
    |c_j - a(1-rho) w_j - a rho sign(w_j)| for w_j != 0 and max(|c_j| - a rho, 0) for w_j = 0,
    relative to a rho; plus sum r = 0 (intercept)."""
    import torch
    s, Y, cv_idx, out, st = c5
    m_ = s.E.shape[1]
    Xd = _device_augmented(s, torch)[:, : s.p]
    Yd = torch.from_numpy(Y).cuda()
    n = s.N
    worst = 0.0
    nnz = 0
    for r in range(Y.shape[1]):
        for j, a in enumerate(ALPHAS_C5):
            res = out[r][j]
            assert res["converged"], (r, j, res["n_iter"])
            fits = [(cv_idx[k][0], res["cv_coefs"][:, k], res["cv_intercepts"][k]) for k in range(5)]
            fits.append((None, res["refit_coef"], res["refit_intercept"]))
            for rows, w, b in fits:
                msk = torch.zeros(n, dtype=torch.float64, device="cuda")
                if rows is None:
                    msk.fill_(1.0)
                else:
                    msk[torch.from_numpy(np.asarray(rows)).cuda()] = 1.0
                nm = float(msk.sum())
                wd = torch.from_numpy(w).cuda()
                resid = msk * (Yd[:, r] - Xd @ wd - b)
                c = (Xd.t() @ resid) / nm
                l1, l2 = a * 0.5, a * 0.5
                nz = wd != 0
                v = torch.where(nz, (c - l2 * wd - l1 * torch.sign(wd)).abs(),
                                (c.abs() - l1).clamp_min(0))
                viol = float(v.max()) / l1
                worst = max(worst, viol)
                nnz += int(nz.sum())
                assert viol < 1e-6, (r, j, rows is None, viol)
                # intercept: mean residual 0.  X^T(m y) accumulates in f32 inside the MFMA
                # (float64 across row slabs), which leaves ~1e-8 in the mean; bar 1e-7 (the
                # north-star Gaussian bar is 1e-5 relative)
                assert abs(float(resid.sum())) / nm < 1e-7
    assert nnz > 0
    print(f"c5 worst KKT violation / (a rho): {worst:.2e}, nonzeros {nnz}")


def test_c5_enet_fits_vs_oracle(c5):
    """Two responses x (split 0, refit) at alpha = 1e-2 against the oracle's cyclic CD."""
    s, Y, cv_idx, out, st = c5
    X = s.dense_X()
    j, a = 1, ALPHAS_C5[1]
    tr = np.asarray(cv_idx[0][0])
    for r in (0, 2):
        c, b = glm_ref.fit_enet_cd(X[tr], Y[tr, r], a, 0.5)
        assert rel(out[r][j]["cv_coefs"][:, 0], c) < TOL_GAUSS, r
        assert abs(out[r][j]["cv_intercepts"][0] - b) < TOL_GAUSS * max(1.0, abs(b))
        c, b = glm_ref.fit_enet_cd(X, Y[:, r], a, 0.5)
        assert rel(out[r][j]["refit_coef"], c) < TOL_GAUSS, r
        assert abs(out[r][j]["refit_intercept"] - b) < TOL_GAUSS * max(1.0, abs(b))
