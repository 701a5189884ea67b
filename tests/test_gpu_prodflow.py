"""The reference's production OLS flow at full size on the MI355X (round 5).

er_refactored_from_scratch_cleanup.py:421-452: timeshift_vals (shifts 0, -20..-1, 1..20) ->
the NaN-row filter -> holdout_splits by trial id (20 %) -> cv_idx_by_trial_id (50 splits, test
20 %) -> simple_cv_fit (OLS, alpha 0, fit_intercept) -> training_fit_holdout_score, here on a
synthetic host frame of the logged size (1,900,992 rows, 18 events x 41 lags = 738 predictors;
02-create_features-lynne-f5.ipynb) through the drop-in API.  Two of the 50 fold fits and the
refit against the float64 oracle (normal equations summed over row chunks,
oracle/glm_ref.fit_ols_chunks) at the Gaussian bar 1e-5.
"""
import contextlib
import io

import numpy as np
import pytest

from oracle import glm_ref

pytestmark = pytest.mark.gpu
TOL_GAUSS = 1e-5
L, K = 20, 50


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def test_prod50_folds_vs_oracle(engine):
    import sglm_ez
    from sglm_hip import synth
    df, ev, beta, b0 = synth.ols_frame(1_900_992, 18, -L, L, seed=11)
    with contextlib.redirect_stdout(io.StringIO()):
        dfrel = sglm_ez.timeshift_cols(df, ev, neg_order=-L, pos_order=L)
        xcols = sglm_ez.add_timeshifts_to_col_list(ev, ev, neg_order=-L, pos_order=L)
        dfrel = dfrel[dfrel[["nTrial"] + xcols + ["y"]].isna().sum(axis=1) == 0]
        np.random.seed(30186)
        hold = sglm_ez.holdout_split_by_trial_id(dfrel, id_cols=["nTrial"], perc_holdout=0.2)
        setup = dfrel.loc[~hold]
        cv_idx = sglm_ez.cv_idx_by_trial_id(setup, trial_id_columns=["nTrial"], num_folds=K,
                                            test_size=0.2)
        kws = [{"alpha": 0.0, "l1_ratio": 0.0, "max_iter": 1000, "fit_intercept": True}]
        out = sglm_ez.simple_cv_fit(setup[xcols], setup["y"], cv_idx, kws, model_type="Normal",
                                    score_method="r2")
    assert len(cv_idx) == K
    res = out[4]["full_cv_results"][0]
    E = df[ev].to_numpy(dtype=np.float64)
    y = df["y"].to_numpy()
    pos = setup.positions()
    shifts = [0] + list(range(-L, 0)) + list(range(1, L + 1))

    def chunks(rows, step=131072):
        for a in range(0, rows.size, step):
            r = rows[a:a + step]
            X = np.empty((r.size, len(shifts) * len(ev)))
            for bi, sh in enumerate(shifts):
                X[:, bi * len(ev):(bi + 1) * len(ev)] = E[r - sh]
            yield X, y[r]
    for k in (0, 1):
        rows = pos[np.asarray(cv_idx[k][0])]
        c, b = glm_ref.fit_ols_chunks(chunks(rows))
        assert rel(res["cv_coefs"][:, k], c) < TOL_GAUSS
        assert abs(res["cv_intercepts"][k] - b) < TOL_GAUSS * max(1.0, abs(b))
    c, b = glm_ref.fit_ols_chunks(chunks(pos))
    assert rel(out[3].model.coef_, c) < TOL_GAUSS
    assert abs(out[3].model.intercept_ - b) < TOL_GAUSS * max(1.0, abs(b))
    # the synthetic truth, to the noise level
    assert np.max(np.abs(c - beta.reshape(-1))) < 0.1
