"""Package layout of the reference (sglm.models.*, sglm.features.*) next to the backend
bare-name modules: imports, aliases, the package's own fold/holdout key
scheme against the oracle and scikit-learn (host integer work: CPU)."""
import numpy as np
import pandas as pd

from oracle import folds_ref


def test_package_aliases_resolve():
    import sglm
    import sglm_
    import sglm_cv
    import sglm_ez
    from sglm.features import setup_model_fit, sglm_pp as f_pp
    from sglm.models import eval as m_eval, sglm as m_sglm, sglm_cv as m_cv, split_data
    assert m_sglm.GLM is sglm.GLM is sglm_.GLM
    assert m_sglm.calc_R2 is sglm.calc_R2 and callable(m_sglm.fit_GLM)
    assert m_cv.cv_glm_mult_params is sglm_cv.cv_glm_mult_params
    assert m_cv.simple_cv_fit is sglm_ez.simple_cv_fit
    assert f_pp.timeshift_cols is sglm_ez.timeshift_cols
    for name in ("timeshift", "timeshift_multiple", "shift", "zscore", "diff",
                 "bucket_ids_by_timeframe", "get_column_nums", "cv_idx_from_bucket_ids"):
        assert callable(getattr(f_pp, name))
    for name in ("timeshift_vals", "timeshift_vals_by_dict", "X_cols_dict_to_default",
                 "xy_pairs_to_widest_orders", "multi_file_analysis_prep",
                 "single_file_analysis_prep"):
        assert callable(getattr(setup_model_fit, name))
    for name in ("holdout_split_by_trial_id", "holdout_splits", "cv_idx_by_trial_id",
                 "cv_idx_from_bucket_ids"):
        assert callable(getattr(split_data, name))
    assert m_eval.calc_l1(np.array([1.0, -2.0])) == 3.0
    assert m_eval.calc_l2(np.array([1.0, -2.0])) == 5.0


def _frame(seed=5, n=3000):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"nTrial_filenum": np.repeat(np.arange(n // 30), 30)[:n],
                         "iBlock": rng.integers(0, 13, n) // 3,
                         "x": rng.random(n)})


def test_package_cv_idx_two_key_columns_vs_oracle_and_sklearn():
    from sklearn.model_selection import GroupShuffleSplit
    from sglm.models import split_data
    df = _frame()
    cols = ["nTrial_filenum", "iBlock"]
    np.random.seed(11)
    got = split_data.cv_idx_by_trial_id(df, trial_id_columns=cols, num_folds=4)
    codes = folds_ref.trial_bucket_codes([df[c].values for c in cols], package_style=True)
    np.random.seed(11)
    ref = folds_ref.cv_idx_from_bucket_ids(codes, num_folds=4)
    np.random.seed(11)
    sk = list(GroupShuffleSplit(n_splits=4, test_size=0.25).split(df, None, codes))
    for (a, b), (c, d), (e, f) in zip(got, ref, sk):
        assert np.array_equal(a, c) and np.array_equal(b, d)
        assert np.array_equal(a, e) and np.array_equal(b, f)
    # the backend scheme joins extra columns differently -> different groups
    bk = folds_ref.trial_bucket_codes([df[c].values for c in cols], package_style=False)
    assert len(np.unique(codes)) == len(np.unique(bk))


def test_package_holdout_without_replacement():
    from sglm.models import split_data
    df = _frame(seed=7)
    cols = ["nTrial_filenum", "iBlock"]
    np.random.seed(21)
    hold = split_data.holdout_split_by_trial_id(df, id_cols=cols, perc_holdout=0.3)
    codes = folds_ref.trial_bucket_codes([df[c].values for c in cols], package_style=True)
    G = int(codes.max() + 1)
    np.random.seed(21)
    test_ids = np.random.choice(G, size=int(G * 0.3), replace=False)
    assert np.array_equal(hold.values, np.isin(codes, test_ids))
    assert len(np.unique(codes[hold.values])) == int(G * 0.3)      # no repeated groups
    setup, holdout, h2 = split_data.holdout_splits(df, id_cols=cols, perc_holdout=0.3)
    assert len(setup) + len(holdout) == len(df)


def test_setup_model_fit_dict_helpers():
    from sglm.features import setup_model_fit as smf
    d = smf.X_cols_dict_to_default({"a": (0, 0), "b": (-3, 2), "c": None}, -5, 5)
    assert d == {"a": (-5, 5), "b": (-3, 2), "c": (-5, 5)}
    w = smf.xy_pairs_to_widest_orders([{"X_cols": {"a": (-2, 3), "b": (-1, 1)}},
                                       {"X_cols": {"a": (-4, 1), "c": (0, 2)}}])
    assert w == {"a": (-4, 3), "b": (-1, 1), "c": (0, 2)}


def test_glm_data_roundtrip_and_output_formats(tmp_path):
    """sglm_save.GLM_data: a fitted GLM (coefficients set as after a fit) pickles with the
    container and loads back; coef_/intercept_ in the reference's np.save formats."""
    import pickle
    import sglm
    import sglm_save
    glm = sglm.GLM("Normal", alpha=1.0, l1_ratio=0.0)
    glm._set_fitted(np.arange(5, dtype=np.float64) / 7, 0.25, 3)
    gd = sglm_save.GLM_data(str(tmp_path), "run.pkl")
    gd.set_uid("u1")
    gd.set_X_cols(["a", "b", "c", "d", "e"])
    gd.set_gss_info(5, 0.2, 0.2)
    gd.set_timeshifts(-20, 20)
    gd.append_fit_results("y", {"alpha": 1.0}, glm_model=glm, scores={"tr_witi": 0.5})
    gd.save()
    back = sglm_save.GLM_data(str(tmp_path), "run.pkl")
    back.load()
    fr = back.data["fit_results"][0]
    assert back.data["uid"] == "u1" and fr["scores"]["holdout_noiti"] is None
    assert np.array_equal(fr["glm_model_gss"].coef_, glm.coef_)
    assert fr["glm_model_gss"].intercept_ == 0.25
    with open(tmp_path / "raw.pkl", "wb") as f:          # a bare dict file loads too
        pickle.dump({"fit_results": []}, f)
    raw = sglm_save.GLM_data(str(tmp_path), "raw.pkl")
    raw.load()
    assert raw.data == {"fit_results": []}
    np.save(tmp_path / "coef.npy", glm.coef_)
    np.save(tmp_path / "icpt.npy", glm.intercept_)
    c, b = np.load(tmp_path / "coef.npy"), np.load(tmp_path / "icpt.npy")
    assert c.dtype == np.float64 and c.shape == (5,) and b.shape == () and float(b) == 0.25
