"""The device-resident production flow (sglm_hip.lagframe): sglm_ez.timeshift_cols returns a
LagFrame whose lag columns stay on the device; the reference driver's operations
(er_refactored_from_scratch_cleanup.py:421-452) -- the NaN-row filter, .loc holdout splits,
trial-id folds, column selections, simple_cv_fit, fit / predict -- run without the N x (mK)
host block, and give the values / results of the materialised DataFrame (SGLM_LAGFRAME=0,
the reference's own timeshift_multiple arithmetic, backend/sglm_pp.py:58-103)."""
import numpy as np
import pandas as pd
import pytest

from oracle import pp_ref

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _frame(N=3000, m=4, seed=0, nan_rows=(5, 77)):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({f"ev{a}": (rng.random(N) < 0.1).astype(np.float64) for a in range(m)})
    df["sig"] = rng.normal(size=N)
    df["cnt"] = rng.integers(0, 5, N)                          # an int column (not shifted)
    df.insert(0, "nTrial", np.arange(N) // 50)
    df.loc[list(nan_rows), "ev1"] = np.nan
    df.index = pd.RangeIndex(100, 100 + N)                      # a non-default index
    return df


def test_lagframe_matches_materialised_frame(engine):
    import sglm_ez
    import sglm_pp
    from sglm_hip.lagframe import LagFrame
    df = _frame()
    cols = ["ev0", "ev1", "ev2", "sig"]
    lf = sglm_ez.timeshift_cols(df, cols, neg_order=-3, pos_order=2)
    assert isinstance(lf, LagFrame)
    sglm_pp.LAGFRAME = False
    try:
        ref = sglm_ez.timeshift_cols(df, cols, neg_order=-3, pos_order=2)
    finally:
        sglm_pp.LAGFRAME = True
    assert isinstance(ref, pd.DataFrame) and not isinstance(ref, LagFrame)
    assert list(lf.columns) == list(ref.columns)
    assert lf.index.equals(ref.index) and lf.shape == ref.shape
    mat = lf.to_pandas()
    pd.testing.assert_frame_equal(mat, ref)
    # the reference arithmetic restated (oracle): shift-major blocks, NaN fill
    idx = [df.columns.get_loc(c) for c in cols]
    exp = pp_ref.timeshift_multiple(df.values.astype(float), idx,
                                    [0] + list(range(-3, 0)) + list(range(1, 3)))
    assert np.array_equal(lf.values, exp, equal_nan=True)
    # the flow's operations
    xcols = sglm_ez.add_timeshifts_to_col_list(cols, cols, neg_order=-3, pos_order=2)
    nn = lf[["nTrial"] + xcols].isna().sum(axis=1)
    pd.testing.assert_series_equal(nn, ref[["nTrial"] + xcols].isna().sum(axis=1),
                                   check_dtype=False)
    keep = (nn == 0) & (lf["cnt"] != 0)
    f1, r1 = lf[keep], ref[keep]
    assert isinstance(f1, LagFrame)
    pd.testing.assert_frame_equal(f1.to_pandas(), r1)
    pd.testing.assert_frame_equal(lf.dropna().to_pandas(), ref.dropna())
    pd.testing.assert_frame_equal(lf.dropna(subset=["ev0_-3", "sig_2"]).to_pandas(),
                                  ref.dropna(subset=["ev0_-3", "sig_2"]))
    hold = f1["nTrial"] % 3 == 0
    pd.testing.assert_frame_equal(f1.loc[~hold].to_pandas(), r1.loc[~hold])
    pd.testing.assert_frame_equal(f1.loc[hold, xcols].to_pandas(), r1.loc[hold, xcols])
    pd.testing.assert_frame_equal(f1.iloc[10:20].to_pandas(), r1.iloc[10:20])
    pd.testing.assert_series_equal(f1["ev2_-2"], r1["ev2_-2"])
    pd.testing.assert_frame_equal(f1[["nTrial", "cnt"]], r1[["nTrial", "cnt"]])
    assert f1.copy().shape == r1.shape and len(repr(f1)) > 0
    pd.testing.assert_frame_equal(f1.head(7), r1.head(7))
    pd.testing.assert_frame_equal(f1.tail(3), r1.tail(3))
    g = f1.copy()
    g["pred"] = np.arange(len(g), dtype=float)
    r2 = r1.copy()
    r2["pred"] = np.arange(len(r2), dtype=float)
    pd.testing.assert_frame_equal(g.to_pandas(), r2)
    # anything else materialises (a pandas method the frame does not implement)
    assert np.allclose(f1.mean().values, r1.mean().values, equal_nan=True)


def test_lagframe_design_equals_host_design(engine):
    """The device design of a filtered lagged frame equals the design packed from the
    materialised values: contiguous rows (the canonical lag layout -> from_events, with its
    LagStructure) and a holdout-filtered (non-contiguous) row set (row gather)."""
    import sglm_ez
    from sglm_hip import engine as E
    df = _frame(N=4000, nan_rows=())
    cols = ["ev0", "ev1", "ev2", "ev3"]
    lf = sglm_ez.timeshift_cols(df, cols, neg_order=-4, pos_order=3)
    xcols = sglm_ez.add_timeshifts_to_col_list(cols, cols, neg_order=-4, pos_order=3)
    f1 = lf[lf[xcols].isna().sum(axis=1) == 0]
    assert f1._span() is not None                     # the filter leaves one row range
    import sglm_pp
    sglm_pp.LAGFRAME = False
    try:
        ref = sglm_ez.timeshift_cols(df, cols, neg_order=-4, pos_order=3)
    finally:
        sglm_pp.LAGFRAME = True
    r1 = ref[ref[xcols].isna().sum(axis=1) == 0]
    assert f1.index.equals(r1.index)
    pd.testing.assert_series_equal(f1["nTrial"], r1["nTrial"])
    pd.testing.assert_series_equal(f1[xcols].isna().sum(axis=1),
                                   r1[xcols].isna().sum(axis=1), check_dtype=False)
    pd.testing.assert_frame_equal(f1.to_pandas(), r1)
    X1 = f1[xcols]
    d1 = X1.design()
    assert d1.lag is not None                         # event-correlation Gram / gradient path
    h = E.Design.from_host(X1.values)
    assert (d1.n, d1.p, d1.P) == (h.n, h.p, h.P)
    assert bool((d1.xb == h.xb).all())
    hold = (f1["nTrial"] % 4 == 1).values
    X2 = f1[~hold][xcols]
    d2 = X2.design()
    h2 = E.Design.from_host(X2.values)
    assert d2.lag is None and bool((d2.xb == h2.xb).all())
    assert d2.xbits is not None and bool((d2.xbits == h2.xbits).all())
    with pytest.raises(ValueError, match="NaN"):
        lf[xcols].design()                            # unfiltered edge rows hold NaN


def test_production_flow_resident_equals_host_path_c3(engine):
    """C3 shape (Poisson 100k x 500: 25 events x lags -10..9), the driver's flow from a host
    event DataFrame: timeshift_cols -> isna filter -> holdout split (.loc) -> trial-id folds ->
    simple_cv_fit over 3 alphas -> training_fit_holdout_score; resident (LagFrame) vs the
    materialised DataFrame path, folds bit-exact, coefficients and scores at 1e-5 / 1e-6."""
    import sglm_ez
    import sglm_pp
    from sglm_hip import synth
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    Nr, m = s.E.shape
    r0 = s.L - 1
    ev = [f"e{a}" for a in range(m)]
    df = pd.DataFrame(s.E.astype(np.float64), columns=ev)
    df.insert(0, "nTrial", ((np.arange(Nr) - r0) // 100).astype(np.float64))
    y = np.full(Nr, np.nan)
    y[r0:r0 + s.N] = s.y
    df["y"] = y
    alphas = [float(v) for v in np.logspace(-4, 1, 20)[[0, 10, 19]]]

    def flow():
        dfrel = sglm_ez.timeshift_cols(df, ev, neg_order=-s.L, pos_order=s.L - 1)
        xcols = sglm_ez.add_timeshifts_to_col_list(ev, ev, neg_order=-s.L, pos_order=s.L - 1)
        dfrel = dfrel[dfrel[["nTrial"] + xcols + ["y"]].isna().sum(axis=1) == 0]
        np.random.seed(11)
        hold = sglm_ez.holdout_split_by_trial_id(dfrel, id_cols=["nTrial"], perc_holdout=0.2)
        setup, holdout = dfrel.loc[~hold].copy(), dfrel.loc[hold].copy()
        cv_idx = sglm_ez.cv_idx_by_trial_id(setup, trial_id_columns=["nTrial"], num_folds=4)
        kws = [{"model_name": "Poisson", "alpha": a} for a in alphas]
        out = sglm_ez.simple_cv_fit(setup[xcols], setup["y"], cv_idx, kws, model_type="Normal",
                                    score_method="r2")
        best = dict(out[2])
        best["model_name"] = "Poisson"
        glm, hs, hm = sglm_ez.training_fit_holdout_score(setup[xcols], setup["y"],
                                                         holdout[xcols], holdout["y"], best)
        pred = glm.predict(holdout[xcols])
        return cv_idx, out, glm, hs, hm, pred, type(dfrel)

    cv_a, out_a, glm_a, hs_a, hm_a, pred_a, typ_a = flow()
    sglm_pp.LAGFRAME = False
    try:
        cv_b, out_b, glm_b, hs_b, hm_b, pred_b, typ_b = flow()
    finally:
        sglm_pp.LAGFRAME = True
    assert typ_a.__name__ == "LagFrame" and typ_b is pd.DataFrame
    for (a, b), (c, d) in zip(cv_a, cv_b):
        assert np.array_equal(a, c) and np.array_equal(b, d)
    for ra, rb in zip(out_a[4]["full_cv_results"], out_b[4]["full_cv_results"]):
        assert rel(ra["cv_coefs"], rb["cv_coefs"]) < 1e-5
        assert np.max(np.abs(ra["cv_scores_test"] - rb["cv_scores_test"])) < 1e-6
        assert abs(ra["cv_R2_score"] - rb["cv_R2_score"]) < 1e-6
        assert rel(ra["model"].coef_, rb["model"].coef_) < 1e-5
    assert out_a[2] == out_b[2]
    assert rel(glm_a.coef_, glm_b.coef_) < 1e-5
    assert abs(hs_a - hs_b) < 1e-6 and abs(hm_a - hm_b) < 1e-6 * max(1.0, abs(hm_b))
    assert rel(pred_a, pred_b) < 1e-5


def test_lagframe_snapshot_and_uploads(engine):
    """The lagged frame takes the caller's columns when it is made: a column assignment, a
    column drop and an in-place row drop of the caller's frame afterwards change nothing (the
    reference's timeshift_multiple returns a copy); source columns uploaded by separate calls
    (0/1 ones as bit rows, a real one as float64, one of them a second time) give the host
    values; the occurrence list sized by the host counts equals the one sized on the device."""
    import torch
    import sglm_ez
    import sglm_pp
    from sglm_hip import engine as E
    df = _frame(N=2500, seed=5, nan_rows=())
    cols = ["ev0", "ev1", "ev2", "sig"]
    sglm_pp.LAGFRAME = False
    try:
        ref = sglm_ez.timeshift_cols(df.copy(), cols, neg_order=-2, pos_order=2)
    finally:
        sglm_pp.LAGFRAME = True
    lf = sglm_ez.timeshift_cols(df, cols, neg_order=-2, pos_order=2)
    df["ev0"] = 7.0                              # assignment replaces the caller's column
    df.drop(columns=["sig"], inplace=True)
    df.drop(index=df.index[:300], inplace=True)  # shorter than the frame's row count
    pd.testing.assert_frame_equal(lf.to_pandas(), ref)
    src = lf._src
    # uploads in two calls: 0/1 columns first, then a real column with one repeated name
    src.upload(["ev2", "ev0"])
    src.upload(["sig", "ev2"])
    assert src.bits(["ev0", "ev2"]) is not None and src.bits(["sig"]) is None
    Ed, idx = src.device(["ev0", "sig", "ev2"])
    got = Ed[idx].cpu().numpy()
    exp = np.stack([ref["ev0"].to_numpy(), ref["sig"].to_numpy(), ref["ev2"].to_numpy()])
    assert np.array_equal(got, exp, equal_nan=True)
    # the occurrence list: sized from the host pack's counts == sized on the device
    B = src.bits(["ev0", "ev1", "ev2"])
    ones = sum(src.ones(c) for c in ("ev0", "ev1", "ev2"))
    a = E.LagStructure.build(None, [0, 1, -1], 1, 2400, False, ebits=B, nnz=ones, n_raw=2500)
    b = E.LagStructure.build(None, [0, 1, -1], 1, 2400, False, ebits=B, nnz=None, n_raw=2500)
    assert torch.equal(a.occ, b.occ) and torch.equal(a.tbeg, b.tbeg)
    assert torch.equal(a.tend, b.tend)


def test_lagframe_is_a_dataframe(engine, tmp_path):
    """The lagged frame passes isinstance(x, pd.DataFrame) (the reference's timeshift_multiple
    returns one, backend/sglm_pp.py:485): the flow's operations stay lazy, and any other pandas
    use -- pd.concat, set_index, to_parquet, get_dummies, insert, pickling -- sees exactly the
    materialised DataFrame."""
    import pickle
    import sglm_ez
    import sglm_pp
    from sglm_hip.lagframe import LagFrame
    df = _frame(seed=3)
    cols = ["ev0", "ev1", "sig"]
    lf = sglm_ez.timeshift_cols(df, cols, neg_order=-2, pos_order=2)
    sglm_pp.LAGFRAME = False
    try:
        ref = sglm_ez.timeshift_cols(df, cols, neg_order=-2, pos_order=2)
    finally:
        sglm_pp.LAGFRAME = True
    assert isinstance(lf, LagFrame) and isinstance(lf, pd.DataFrame) and lf.is_lazy
    r1 = ref.dropna()
    # the flow's operations keep it lazy
    xcols = sglm_ez.add_timeshifts_to_col_list(cols, cols, neg_order=-2, pos_order=2)
    k = lf[lf[["nTrial"] + xcols].isna().sum(axis=1) == 0]
    k2 = k.loc[k["nTrial"] % 3 == 0, xcols]
    k2["extra"] = 1.0
    assert k.is_lazy and k2.is_lazy and lf.is_lazy
    assert isinstance(k2, pd.DataFrame)
    # pandas uses of the frame: the materialised values
    f1 = lf.dropna()
    pd.testing.assert_frame_equal(pd.concat([f1, r1.iloc[:5]]), pd.concat([r1, r1.iloc[:5]]))
    assert not f1.is_lazy
    pd.testing.assert_frame_equal(lf.dropna().set_index("nTrial"), r1.set_index("nTrial"))
    fn = tmp_path / "f.parquet"
    lf.dropna().to_parquet(fn)
    pd.testing.assert_frame_equal(pd.read_parquet(fn), r1)
    pd.testing.assert_frame_equal(pd.get_dummies(lf.dropna(), columns=["cnt"]),
                                  pd.get_dummies(r1, columns=["cnt"]))
    h = lf.dropna()
    h.insert(0, "z", 2.0)
    r = r1.copy()
    r.insert(0, "z", 2.0)
    pd.testing.assert_frame_equal(h, r)
    assert list(h.columns) == list(r.columns) and h.shape == r.shape
    pd.testing.assert_series_equal(h["z"], r["z"])
    q = pickle.loads(pickle.dumps(lf.dropna()))
    assert type(q) is pd.DataFrame
    pd.testing.assert_frame_equal(q, r1)
    # arithmetic and reductions as pandas gives them
    pd.testing.assert_series_equal(lf.dropna().sum(), r1.sum())
    pd.testing.assert_frame_equal(lf.dropna() * 2, r1 * 2)


def test_lagframe_lag_block_with_extra_columns(engine):
    """A contiguous lagged frame whose columns are the canonical lag block followed by unshifted
    extra columns -- the production design's counters, an assigned (overlay) column and a 0/1
    dummy (sglm_cb_concat_make_design_mat.py:286, 310) -- builds its design from the events
    (LagStructure: structured Gram and correlation start) with the extras as the float64 block
    of a mixed design, never from a host copy; its fits equal the host-packed design's."""
    import sglm_ez
    from sglm_hip import engine as E
    rng = np.random.default_rng(5)
    df = _frame(N=6000, nan_rows=())
    df["cnt2"] = (rng.integers(0, 40, len(df)) ** 2) / 5000.0    # a continuous counter
    df["dum"] = (np.arange(len(df)) >= 3000).astype(np.float64)   # a session dummy
    cols = ["ev0", "ev1", "ev2", "ev3"]
    lf = sglm_ez.timeshift_cols(df, cols, neg_order=-3, pos_order=3)
    xcols = sglm_ez.add_timeshifts_to_col_list(cols, cols, neg_order=-3, pos_order=3)
    f1 = lf[lf[xcols].isna().sum(axis=1) == 0]
    f1["asg"] = np.linspace(0.0, 1.0, len(f1))                    # an assigned column
    X = f1[xcols + ["cnt2", "dum", "asg"]]
    host = X.to_pandas().to_numpy(dtype=np.float64)
    calls = []
    orig = E.Design.from_host.__func__

    def spy(cls, *a, **k):
        calls.append(1)
        return orig(cls, *a, **k)
    E.Design.from_host = classmethod(spy)
    try:
        d = X.design()
    finally:
        E.Design.from_host = classmethod(orig)
    assert not calls
    assert d.lag is not None and d.k == 3 and d.p == len(xcols) + 3
    assert E._lagw(d) is not None
    y = rng.poisson(np.exp(0.3 * host[:, 0] - 0.2 * host[:, -1] + 0.5)).astype(float)
    import sglm
    g1 = sglm.GLM("Poisson", alpha=1e-3)
    g1.fit(X, y)
    g2 = sglm.GLM("Poisson", alpha=1e-3)
    g2.fit(host, y)
    assert rel(g1.coef_, g2.coef_) < 1e-4
    assert abs(g1.intercept_ - g2.intercept_) < 1e-4 * max(1.0, abs(g2.intercept_))
