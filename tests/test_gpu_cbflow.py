"""The multi-session production flow of sglm_cb_concat_make_design_mat.py:244-363 through the
drop-in API, with the lagged frame resident on the device (bench.cb_flow replays it line by line:
convert_dtypes -> dropna(subset=y) -> get_dummies(session) -> timeshift -> .loc[flag == 0] ->
the trial constants assigned back -> dropna -> holdout_split_by_trial_id -> cv_idx_by_trial_id
(3 splits, test 20 %) -> drop nTrial -> simple_cv_fit OLS fit_intercept=False ->
training_fit_holdout_score).

The design is 0/1 event lags + the two continuous counters + one dummy per session on
non-contiguous setup rows (holdout trials removed), so it is a mixed design; the test asserts it
is built from the lagged frame's device sources, never by materialising the frame on the host
(``Design.from_host`` is made to fail), and holds every fold fit and the refit to the float64
normal equations of the materialised design (numpy lstsq, fit_intercept=False: what
LinearRegression computes, backend/sglm.py:96-101) at the Gaussian bar 1e-5.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL_GAUSS = 1e-5


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


@pytest.mark.parametrize("N,m,L,sessions", [(60_000, 6, 10, 4), (150_000, 12, 20, 3)])
def test_cb_flow_resident_vs_normal_equations(engine, monkeypatch, N, m, L, sessions):
    import bench
    from sglm_hip import synth
    from sglm_hip.lagframe import LagFrame
    df, ev, beta, gamma, offs = synth.cb_frame(N, m, -L, L, sessions=sessions, seed=N % 97)

    def no_host(*a, **k):
        raise AssertionError("the lagged frame's design went through Design.from_host")
    monkeypatch.setattr(engine.Design, "from_host", classmethod(no_host))
    out, hs, X_setup, y_setup, cv, xcols = bench.cb_flow(df, ev, -L, L, folds=3)
    assert isinstance(X_setup, LagFrame)
    assert list(X_setup.columns) == xcols
    nl = m * (2 * L + 1)
    assert len(xcols) == nl + 2 + sessions
    assert len(cv) == 3
    d = X_setup.design()
    assert d.k >= 2                                  # the counters: a mixed design
    monkeypatch.undo()
    X = X_setup.to_pandas().to_numpy(dtype=np.float64)
    y = y_setup.to_numpy(dtype=np.float64)
    assert np.isfinite(X).all() and np.isfinite(y).all()
    res = out[4]["full_cv_results"][0]
    for k in range(3):
        tr = np.asarray(cv[k][0])
        c = np.linalg.lstsq(X[tr], y[tr], rcond=None)[0]
        assert rel(res["cv_coefs"][:, k], c) < TOL_GAUSS, k
        assert res["cv_intercepts"][k] == 0.0
    c = np.linalg.lstsq(X, y, rcond=None)[0]
    assert rel(out[3].model.coef_, c) < TOL_GAUSS
    # the synthetic truth, to the noise level: the lags and the ENL counter (the ENLP counter's
    # values, <= 19^2 / 5000, carry too little variance at this size to pin its coefficient)
    assert np.max(np.abs(c[:nl] - beta.reshape(-1))) < 0.25
    assert abs(c[nl] - gamma[0]) < 0.1
    assert np.isfinite(hs)
