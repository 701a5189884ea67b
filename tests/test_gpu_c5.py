"""C5 at its configured size (BASELINE.json configs[4]): 64 responses x the
1M x 2000 lag design, Gaussian elastic net l1_ratio 0.5 over the 20 alphas of
np.logspace(-4, 1, 20), 5 trial-id splits + refit per (response, alpha) = 7,680 fits -- the
exact workload `bench.py --config c5` times.

The reference runs one simple_cv_fit per response (er_refactored_from_scratch_cleanup.py:
388-452) on sklearn ElasticNet (backend/sglm.py:109-110).  Checks:
* EVERY fit satisfies the ElasticNet optimality conditions of the sklearn objective
  (_coordinate_descent.py:420-422) in float64: with r = m (y - X w - b) and c = X^T r / n_m,
  |c_j - a(1-rho) w_j - a rho sign(w_j)| (w_j != 0) and max(|c_j| - a rho, 0) (w_j = 0), relative
  to a rho, <= 1e-6; mean residual <= 1e-7 (intercept).  The residuals of all 64 responses of
  one (mask, alpha) are one float64 GEMM pair on the device against the dense float64 design.
* Two mid-path fits (split 0 and the refit at alphas 4 and 7 of the 9 with a non-empty support) equal the oracle's cyclic CD
  (oracle/glm_ref.fit_enet_cd_gram on the float64 centred Gram of the same rows) at 1e-5.
"""
import time

import numpy as np
import pandas as pd
import pytest

from oracle import glm_ref

pytestmark = pytest.mark.gpu
TOL_GAUSS = 1e-5
R_C5, K_C5, NLAM = 64, 5, 20


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


@pytest.fixture(scope="module")
def c5_full(engine):
    import torch
    from sglm_hip import engine as E, enet, folds, synth
    t0 = time.time()
    s = synth.make(N=1_000_000, m=50, L=20, family="gaussian", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(5)                     # bench.py bench_c5's responses
    Y = np.stack([s.y + rng.normal(0, 1, s.N) for _ in range(R_C5)], 1)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K_C5)
    alphas = np.logspace(-4, 1, NLAM)
    st = {}
    out = enet.cv_enet_path(d, Y, cv_idx, alphas, l1_ratio=0.5, max_iter=1000, stats=st)
    torch.cuda.synchronize()
    print(f"C5 path ({st.get('fits')} fits): {time.time() - t0:.1f} s incl. setup, {st}")
    del d
    # dense float64 augmented design on the device (test infrastructure only)
    m = s.E.shape[1]
    Ed = torch.from_numpy(s.E).cuda().to(torch.float64)
    Xd = torch.empty((s.N, s.p + 1), dtype=torch.float64, device="cuda")
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        Xd[:, bi * m:(bi + 1) * m] = Ed[r0 - sh:r0 - sh + s.N]
    Xd[:, s.p] = 1.0
    del Ed
    return s, Y, cv_idx, alphas, out, st, Xd


def test_c5_full_size_every_fit_kkt(c5_full):
    import torch
    s, Y, cv_idx, alphas, out, st, Xd = c5_full
    assert st["fits"] == R_C5 * NLAM * (K_C5 + 1) == 7680
    n, p = s.N, s.p
    Yd = torch.from_numpy(Y).cuda()
    worst, worst_mean, nnz, checked, bad = 0.0, 0.0, 0, 0, 0
    per_alpha = [0.0] * NLAM
    masks = [np.asarray(tr) for tr, _ in cv_idx] + [None]
    for k, rows in enumerate(masks):
        msk = torch.zeros(n, dtype=torch.float64, device="cuda")
        if rows is None:
            msk.fill_(1.0)
        else:
            msk[torch.from_numpy(rows).cuda()] = 1.0
        nm = float(msk.sum())
        for j, a in enumerate(alphas):
            W = np.zeros((p + 1, R_C5))
            for r in range(R_C5):
                res = out[r][j]
                assert res["converged"], (r, j, res["n_iter"])
                if rows is None:
                    W[:p, r], W[p, r] = res["refit_coef"], res["refit_intercept"]
                else:
                    W[:p, r], W[p, r] = res["cv_coefs"][:, k], res["cv_intercepts"][k]
            Wd = torch.from_numpy(W).cuda()
            resid = msk[:, None] * (Yd - Xd @ Wd)               # n x 64, float64
            C = (Xd[:, :p].t() @ resid) / nm                      # p x 64
            l1, l2 = a * 0.5, a * 0.5
            wd = Wd[:p]
            nz = wd != 0
            v = torch.where(nz, (C - l2 * wd - l1 * torch.sign(wd)).abs(),
                            (C.abs() - l1).clamp_min(0))
            viol = (v.max(0).values / l1).cpu().numpy()
            mres = (resid.sum(0).abs() / nm).cpu().numpy()
            worst = max(worst, float(viol.max()))
            worst_mean = max(worst_mean, float(mres.max()))
            per_alpha[j] = max(per_alpha[j], float(viol.max()))
            bad += int(np.sum(viol >= 1e-6)) + int(np.sum(mres >= 1e-7))
            nnz += int(nz.sum())
            checked += R_C5
            del resid, C, v
    print(f"C5 full size: {checked} fits, worst KKT / (a rho) {worst:.2e}, worst |mean r| "
          f"{worst_mean:.2e}, nonzeros {nnz}; worst per alpha "
          + " ".join(f"{v:.1e}" for v in per_alpha))
    assert checked == 7680 and nnz > 0
    assert bad == 0, (bad, worst, worst_mean)


def test_c5_full_size_mid_path_vs_oracle(c5_full):
    """Split 0 and the refit at alphas[4] and alphas[7], responses 0 and 63, against the
    oracle's cyclic CD on the float64 centred Gram of the same rows."""
    import torch
    s, Y, cv_idx, alphas, out, st, Xd = c5_full
    n, p = s.N, s.p
    tr = np.asarray(cv_idx[0][0])
    for rows in (tr, None):
        Xr = Xd[torch.from_numpy(rows).cuda()] if rows is not None else Xd
        nr = Xr.shape[0]
        Xm = Xr[:, :p].mean(0)
        Xc = Xr[:, :p] - Xm
        G = (Xc.t() @ Xc).cpu().numpy()
        for r in (0, R_C5 - 1):
            yr = torch.from_numpy(Y[rows, r] if rows is not None else Y[:, r]).cuda()
            ym = float(yr.mean())
            c = (Xc.t() @ (yr - ym)).cpu().numpy()
            for j in (4, 7):
                w = glm_ref.fit_enet_cd_gram(G, c, nr, float(alphas[j]), 0.5)
                b = ym - float(Xm.cpu().numpy() @ w)
                res = out[r][j]
                got_w = res["refit_coef"] if rows is None else res["cv_coefs"][:, 0]
                got_b = res["refit_intercept"] if rows is None else res["cv_intercepts"][0]
                assert np.count_nonzero(w) > 0, (j, "choose alphas with a non-empty support")
                assert rel(got_w, w) < TOL_GAUSS, (rows is None, r, j, rel(got_w, w))
                assert abs(got_b - b) < TOL_GAUSS * max(1.0, abs(b))
        del Xc, Xr
