"""§8(a) rows A1/A2/A7/A8/A10/A13 through the drop-in API on the MI355X, against sklearn
fixtures (tests/golden/api.npz, tests/golden/make_golden.py::api_extras) and the oracle.

* A8  ``GLM.fit_set`` (backend/sglm.py:254-312): in-place writes into caller-owned arrays,
  residual lists appended;
* A10 ``cv_glm_single_params`` (backend/sglm_cv.py:42-206): ``roll`` popped, ``resp_list``
  appended, refit on un-rolled y;
* A13 ``SGLM_worker`` (backend/sglm_cv.py:15-40): worker threads draining a queue of fit_set
  tasks (bounded waits, no deadlock);
* A1  warm start (backend/sglm.py:91-92,134-140): ``beta0_``/``beta_`` seed the engine;
* A2  ``GLM('Tweedie', power=1.5)`` (backend/sglm.py:116-117) against sklearn;
* A7  ``r2_score`` = sklearn's D^2 for the Tweedie family (backend/sglm.py:184).
"""
import queue
import threading

import numpy as np
import pandas as pd
import pytest

from oracle import cv_ref, glm_ref

pytestmark = pytest.mark.gpu
TOL_POIS = 1e-4
TR, TE = np.arange(0, 2400), np.arange(2400, 3000)


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_tweedie_explicit_power_and_d2_vs_sklearn(engine, golden):
    import sglm
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    for key in ("tw15", "tw12"):
        glm = sglm.GLM("Tweedie", power=float(g[f"{key}_power"]), alpha=float(g[f"{key}_alpha"]),
                       score_method="r2")
        glm.fit(X[TR], y[TR])
        assert rel(glm.coef_, g[f"{key}_coef"]) < TOL_POIS, key
        assert abs(glm.intercept_ - float(g[f"{key}_b"])) < TOL_POIS
        assert abs(glm.score(X[TR], y[TR]) - float(g[f"{key}_d2_train"])) < 1e-6, key
        assert abs(glm.score(X[TE], y[TE]) - float(g[f"{key}_d2_test"])) < 1e-6, key
    glm = sglm.GLM("Poisson", alpha=float(g["pois_alpha"]), score_method="r2")
    glm.fit(X[TR], y[TR])
    assert abs(glm.score(X[TE], y[TE]) - float(g["pois_d2_test"])) < 1e-6
    glm = sglm.GLM("Gamma", alpha=0.05, score_method="r2")
    glm.fit(g["gam_X"], g["gam_y"])
    assert abs(glm.score(g["gam_X"], g["gam_y"]) - float(g["gam_d2"])) < 1e-6


def test_warm_start_from_beta(engine, golden):
    """beta0_/beta_ reach the engine: from sklearn's preset start the same minimiser; from the
    minimiser itself the fit stops within two Newton steps (a cold start takes more)."""
    import sglm
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    glm = sglm.GLM("Poisson", beta0_=float(g["warm_b0"]), beta_=g["warm_w0"].copy(), alpha=0.01)
    assert glm.model.warm_start
    glm.fit(X[TR], y[TR])
    assert rel(glm.coef_, g["warm_coef"]) < TOL_POIS
    cold = sglm.GLM("Poisson", alpha=0.01)
    cold.fit(X[TR], y[TR])
    hot = sglm.GLM("Poisson", beta0_=float(g["warm_b"]), beta_=g["warm_coef"].copy(), alpha=0.01)
    hot.fit(X[TR], y[TR])
    assert rel(hot.coef_, g["warm_coef"]) < TOL_POIS
    assert hot.model.n_iter_ <= 2 < cold.model.n_iter_, (hot.model.n_iter_, cold.model.n_iter_)
    # through the CV path: cv_glm_single_params passes beta_/beta0_ to every fit
    import sglm_cv
    cv_idx = [(TR, TE)]
    r = sglm_cv.cv_glm_single_params(X, y, cv_idx, "Poisson", {"alpha": 0.01},
                                     beta_=g["warm_coef"].copy(), beta0_=float(g["warm_b"]),
                                     resp_list=[])
    assert rel(r["cv_coefs"][:, 0], g["warm_coef"]) < TOL_POIS


def test_fit_set_in_place_and_residual_lists(engine, golden):
    import sglm
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    K = 3
    folds = [(np.setdiff1d(np.arange(3000), np.arange(k, 3000, K)), np.arange(k, 3000, K))
             for k in range(K)]
    p = X.shape[1]
    cv_coefs, cv_b = np.zeros((p, K)), np.zeros(K)
    s_tr, s_te = np.zeros(K), np.zeros(K)
    resids, mresids = [], []
    for k, (tr, te) in enumerate(folds):
        glm = sglm.GLM("Poisson", alpha=0.01)
        glm.fit_set(X[tr], y[tr], X[te], y[te], cv_coefs, cv_b, s_tr, s_te, k,
                    resids=resids, mean_resids=mresids)
    spec = glm_ref.FitSpec("tweedie", alpha=0.01, power=1.0)
    for k, (tr, te) in enumerate(folds):
        c, b = glm_ref.fit_tweedie_newton(X[tr], y[tr], 0.01, 1.0)
        assert rel(cv_coefs[:, k], c) < TOL_POIS
        assert abs(cv_b[k] - b) < TOL_POIS * max(1, abs(b))
        assert abs(s_tr[k] - glm_ref.neg_mse_score(spec, c, b, X[tr], y[tr])) < 1e-6
        assert abs(s_te[k] - glm_ref.neg_mse_score(spec, c, b, X[te], y[te])) < 1e-6
        assert resids[k].shape == te.shape
        assert rel(resids[k], y[te] - glm_ref.predict(spec, c, b, X[te])) < 1e-5
        assert np.array_equal(mresids[k], y[te] - np.mean(y[te]))
    # the pooled R^2 a caller forms from the lists (backend/sglm.py:388-408)
    R2 = sglm.calc_R2(np.concatenate(resids), np.concatenate(mresids))
    assert np.isfinite(R2)


def test_cv_glm_single_params_resp_list_and_roll(engine, golden):
    import sglm_cv
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    folds = [(np.setdiff1d(np.arange(3000), np.arange(k, 3000, 3)), np.arange(k, 3000, 3))
             for k in range(3)]
    resp = []
    kw = {"alpha": 0.05, "roll": 5}
    r = sglm_cv.cv_glm_single_params(X, y, folds, "Poisson", kw, resp_list=resp, score_method="r2")
    assert "roll" not in kw                          # popped (backend/sglm_cv.py:95)
    assert len(resp) == 1 and resp[0] is r
    ref = cv_ref.cv_mult(X, y, folds, [{"model_name": "Poisson", "alpha": 0.05, "roll": 5}],
                         score_method="r2")["full_cv_results"][0]
    assert rel(r["cv_coefs"], ref["cv_coefs"]) < TOL_POIS
    assert np.max(np.abs(r["cv_scores_test"] - ref["cv_scores_test"])) < 1e-6
    assert abs(r["cv_R2_score"] - ref["cv_R2_score"]) < 1e-6
    assert rel(r["model"].coef_, ref["coef"]) < TOL_POIS       # refit on un-rolled y
    r2 = sglm_cv.cv_glm_single_params(X, y, folds, "Poisson", {"alpha": 0.5}, resp_list=resp)
    assert len(resp) == 2 and resp[1] is r2


def test_sglm_worker_threads_drain_fit_set_queue(engine, golden):
    """The reference's worker pattern (backend/sglm_cv.py:15-40, 162-170): fit_set tasks on a
    queue consumed by threads; every task completes, the threads exit on an empty queue."""
    import sglm
    import sglm_cv
    g = golden("api.npz")
    X, y = g["api_X"], g["api_y"]
    K = 4
    folds = [(np.setdiff1d(np.arange(3000), np.arange(k, 3000, K)), np.arange(k, 3000, K))
             for k in range(K)]
    p = X.shape[1]
    cv_coefs, cv_b, s_tr, s_te = np.zeros((p, K)), np.zeros(K), np.zeros(K), np.zeros(K)
    resids, mresids = [], []
    q = queue.Queue()
    for k, (tr, te) in enumerate(folds):
        glm = sglm.GLM("Poisson", alpha=0.02)
        q.put((glm, (X[tr], y[tr], X[te], y[te], cv_coefs, cv_b, s_tr, s_te, k),
               {"resids": resids, "mean_resids": mresids}))
    workers = [sglm_cv.SGLM_worker(q) for _ in range(2)]
    ths = [threading.Thread(target=w.run_single) for w in workers]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
        assert not t.is_alive()
    assert q.empty() and len(resids) == K
    for k, (tr, te) in enumerate(folds):
        c, b = glm_ref.fit_tweedie_newton(X[tr], y[tr], 0.02, 1.0)
        assert rel(cv_coefs[:, k], c) < TOL_POIS, k
    # run_multi: cv_glm_single_params tasks
    resp = []
    q2 = queue.Queue()
    for a in (0.01, 0.1):
        q2.put(((X, y, folds, "Poisson", {"alpha": a}), {"resp_list": resp}))
    w = sglm_cv.SGLM_worker(q2)
    t = threading.Thread(target=w.run_multi)
    t.start()
    t.join(timeout=60)
    assert not t.is_alive() and len(resp) == 2


def test_poisson_grid_mixing_fit_intercept_vs_oracle(engine):
    """The reference's own parameter grids vary 'fit_intercept' (backend/sglm.py:512); fits of
    one fold that start at eta = log(mean y) and at eta = 0 are solved in ONE batch and must
    not share a first Hessian.  Every fold fit, refit and score vs the oracle."""
    import sglm_cv
    import sglm_ez
    from oracle import cv_ref
    from sglm_hip import synth
    s = synth.make(N=30_000, m=10, L=6, family="poisson", rho=0.05, seed=4, beta_scale=0.3)
    X = s.dense_X()
    np.random.seed(7)
    cv_idx = sglm_ez.cv_idx_by_trial_id(pd.DataFrame({"nTrial": s.trial}),
                                       trial_id_columns=["nTrial"], num_folds=3)
    kws = sglm_cv.generate_mult_params({"alpha": [1e-3, 1e-1], "fit_intercept": [True, False]},
                                       {"model_name": "Poisson"})
    ref = cv_ref.cv_mult(X, s.y, cv_idx, [dict(k) for k in kws])
    out = sglm_cv.cv_glm_mult_params(X, s.y, cv_idx, "Normal", kws)
    for r, q in zip(out["full_cv_results"], ref["full_cv_results"]):
        assert rel(r["cv_coefs"], q["cv_coefs"]) < 1e-4, r["glm_kwargs"]
        assert np.max(np.abs(r["cv_intercepts"] - q["cv_intercepts"])) < 1e-4
        assert rel(r["model"].coef_, q["coef"]) < 1e-4
        assert np.max(np.abs(r["cv_scores_test"] - q["cv_scores_test"])) < 1e-6
        if not r["glm_kwargs"].get("fit_intercept", True):
            assert np.all(r["cv_intercepts"] == 0.0)


def test_chain_graph_cache_is_bounded_and_survives_freed_buffers(engine):
    """The factor + inverse chain graphs (csrc/chol.hip) are an LRU of at most
    SGLM_CHOL_GRAPH_CAP (32) executables: two differently sized designs fitted back to back, the
    first one's buffers freed, 40 distinct chain shapes -- the cache never exceeds the bound, a
    clear empties it, and fits after it still match the oracle."""
    import gc
    import torch
    import sglm
    from sglm_hip import _lib, synth
    lib = _lib.load()
    lib.sglm_chol_graph_cache_clear()
    assert lib.sglm_chol_graph_cache_size() == 0
    fits = []
    for N, m, L in ((20_000, 8, 5), (12_000, 5, 7)):
        s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.05, seed=N, beta_scale=0.3)
        X = s.dense_X()
        glm = sglm.GLM("Poisson", alpha=0.01)
        glm.fit(X, s.y)
        c, b = glm_ref.fit_tweedie_newton(X, s.y, 0.01, 1.0)
        assert rel(glm.coef_, c) < TOL_POIS
        fits.append((X, s.y))
        del glm
        gc.collect()
        torch.cuda.empty_cache()
    assert 1 <= lib.sglm_chol_graph_cache_size() <= 32
    # 40 distinct chain shapes (n factored fits) through the C ABI on one stream
    P, B = 64, 40
    rng = np.random.default_rng(0)
    A = rng.normal(size=(B, 200, P))
    H = torch.from_numpy(np.einsum("bij,bik->bjk", A, A).astype(np.float32)).cuda()
    Minv = torch.empty_like(H)
    dsh = torch.zeros((B, P), dtype=torch.float32, device="cuda")
    delta = torch.zeros((B, P), dtype=torch.float32, device="cuda")
    info = torch.zeros(B, dtype=torch.int32, device="cuda")
    frozen = torch.zeros((B, P), dtype=torch.uint8, device="cuda")
    fl = torch.arange(B, dtype=torch.int32, device="cuda")
    cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8, device="cuda")
    s_ = torch.cuda.Stream()
    with torch.cuda.stream(s_):
        for n in range(1, B + 1):
            Hn = H.clone()
            _lib.call("sglm_chol_solve_inv", Hn.data_ptr(), Minv.data_ptr(), P, fl.data_ptr(),
                      None, None, n, n, None, 0, None, dsh.data_ptr(), delta.data_ptr(),
                      info.data_ptr(), frozen.data_ptr(), B, cw.data_ptr(), s_.cuda_stream)
            assert lib.sglm_chol_graph_cache_size() <= 32
    s_.synchronize()
    # the inverse of the last chain (all 40 fits) is right: U^-1 U^-T = H^-1
    M = Minv.double().cpu().numpy()
    Hh = H.double().cpu().numpy()
    for k in (0, 39):
        U = np.triu(M[k])
        assert np.max(np.abs(U @ U.T @ Hh[k] - np.eye(P))) < 1e-3
    assert lib.sglm_chol_graph_cache_clear() == 0
    assert lib.sglm_chol_graph_cache_size() == 0
    X, y = fits[0]
    glm = sglm.GLM("Poisson", alpha=0.01)
    glm.fit(X, y)
    c, b = glm_ref.fit_tweedie_newton(X, y, 0.01, 1.0)
    assert rel(glm.coef_, c) < TOL_POIS


def test_predict_reuses_the_packed_design_until_x_changes(engine):
    """predict / score on the same array reuse its packed design (content digest), an array
    changed in place is packed again (sklearn semantics), and a different estimator shares it."""
    import time
    import sglm
    from sglm_hip import estimators as est, synth
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    X = s.dense_X()
    est.clear_design_cache()
    glm = sglm.GLM("Poisson", alpha=0.01)
    glm.fit(X, s.y)
    t0 = time.perf_counter()
    p1 = glm.model.predict(X)
    t1 = time.perf_counter()
    p2 = glm.model.predict(X)
    t2 = time.perf_counter()
    print(f"predict: first {1e3 * (t1 - t0):.1f} ms, cached {1e3 * (t2 - t1):.1f} ms")
    np.testing.assert_array_equal(p1, p2)
    assert len(est._DESIGN_CACHE) >= 1
    X[:, 0] = 1.0 - X[:, 0]                       # changed in place: packed again
    p3 = glm.model.predict(X)
    ref = np.exp(X @ glm.coef_ + glm.intercept_)
    assert np.max(np.abs(p3 - ref) / ref) < 1e-5
    assert np.max(np.abs(p3 - p1)) > 0
    est.clear_design_cache()
    assert len(est._DESIGN_CACHE) == 0
