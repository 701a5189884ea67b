"""pp_design_mat on the MI355X (the event design matrix before the
timeshift) against the pandas formulation of /root/reference/pp_design_mat.py:6-205
(oracle/designmat_pandas.py, itself pinned to the explicit-walk oracle in
tests/test_designmat_cpu.py).  Every column: name, order, values with NaN positions; dtypes
equal wherever pandas yields a numpy dtype (float64 where pandas yields object / nullable).
The reference's KeyError('flag') without interactions (:196) is fixed in both (documented)."""
import io
import contextlib
import warnings

import numpy as np
import pandas as pd
import pytest

from oracle import designmat_pandas as P

pytestmark = pytest.mark.gpu
warnings.filterwarnings("ignore", category=FutureWarning)


def as_f64(s):
    return s.to_numpy(dtype=np.float64, na_value=np.nan)


def assert_same_frame(got, ref):
    assert list(got.columns) == list(ref.columns)
    assert got.index.equals(ref.index)
    for c in ref.columns:
        np.testing.assert_array_equal(as_f64(got[c]), as_f64(ref[c]), err_msg=c)
        rd = ref[c].dtype
        if isinstance(rd, np.dtype) and rd.kind in "iufb":
            assert got[c].dtype == rd, (c, got[c].dtype, rd)
        else:                                    # object / nullable in pandas
            assert got[c].dtype == np.float64, (c, got[c].dtype, rd)


def session(trials, seed, **kw):
    from sglm_hip import synth
    return synth.designmat_session(trials, seed, **kw)


CASES = [
    dict(),
    dict(nth_licks=[1, 2]),
    dict(nth_licks=[2, 1, 3]),
    dict(nth_licks=[1, 1]),
    dict(nth_licks=[0]),
    dict(interactions={"Reward": ["Consumption", "Cue"]}),
    dict(interactions={"Reward": ["Consumption", "Cue"], "h2": ["Select", "ENLP"]}),
    dict(states=["Select", "Consumption"], interactions={"h2": ["Cons"]}),
]


@pytest.mark.parametrize("kw", CASES)
def test_make_design_mat_vs_pandas(engine, kw):
    import pp_design_mat
    ts, tr = session(300, 3)
    ts_ref = ts.copy()
    ref = P.make_design_mat(ts_ref, tr, verbose=False, **kw)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        got = pp_design_mat.make_design_mat(ts, tr, **kw)
    assert_same_frame(got, ref)
    # the reference's side effect on the caller's frame (:160) and its print (:202)
    np.testing.assert_array_equal(ts["Lick"].to_numpy(), ts_ref["Lick"].to_numpy())
    assert ts["Lick"].dtype == ts_ref["Lick"].dtype
    cue_like = [c for c in ref.columns if c.endswith("cue")]
    s = ref.groupby("nTrial")[cue_like].sum().sum(axis=1)
    assert buf.getvalue().strip() == f"trials_without_dummies = {s.loc[s == 0].index.values!r}"


def test_unordered_rows_take_the_sort_path(engine):
    """Rows shuffled (index labels kept): every nTrial group is scattered, so the grouping
    radix-sorts; pandas groups by value wherever the rows sit."""
    import pp_design_mat
    from sglm_hip import designmat
    ts, tr = session(200, 5)
    rng = np.random.default_rng(0)
    ts = ts.iloc[rng.permutation(len(ts))]
    kw = dict(nth_licks=[1, 2], interactions={"Reward": ["Consumption", "Cue"]})
    ref = P.make_design_mat(ts.copy(), tr, verbose=False, **kw)
    with contextlib.redirect_stdout(io.StringIO()):
        got = pp_design_mat.make_design_mat(ts.copy(), tr, **kw)
    assert_same_frame(got, ref)
    import torch
    key = torch.from_numpy(ts["nTrial"].to_numpy()).cuda()
    g = designmat.group_rows(key)
    assert not g.sorted
    g2 = designmat.group_rows(torch.from_numpy(np.sort(ts["nTrial"].to_numpy())).cuda())
    assert g2.sorted


def test_group_rows_vs_numpy(engine):
    """sglm_group_rows: perm = the stable argsort of the valid keys, segments at key changes;
    ordered and unordered keys, NaN keys anywhere, -0.0 == 0.0, two keys."""
    import torch
    from sglm_hip import designmat
    rng = np.random.default_rng(1)
    for n, ordered in ((1, True), (5000, True), (7, False), (70001, False), (300_000, False),
                       (40_000, "wide")):
        if ordered == "wide":                       # every digit pass of the radix path
            k = rng.standard_normal(n) * 10.0 ** rng.integers(-300, 300, n)
            k[::7] = k[3]                           # repeated keys (groups of many rows)
        else:
            k = np.sort(rng.integers(-5, 40, n).astype(np.float64)) if ordered is True else \
                rng.integers(-5, 40, n).astype(np.float64)
        k[rng.random(n) < 0.05] = np.nan
        k[k == 0] = -0.0
        k2 = rng.integers(0, 3, n).astype(np.float64)
        k2[rng.random(n) < 0.02] = np.nan
        for two in (False, True):
            kk = torch.from_numpy(k).cuda()
            g = designmat.group_rows(kk, torch.from_numpy(k2).cuda() if two else None)
            m, ns, srt = g.counts.cpu().tolist()
            if ordered is not True:
                assert srt == 0
            valid = ~np.isnan(k) & (~np.isnan(k2) if two else True)
            rows = np.flatnonzero(valid)
            kz = np.where(k == 0, 0.0, k)
            want = rows[np.lexsort((rows, k2[rows], kz[rows]))] if two else \
                rows[np.argsort(kz[rows], kind="stable")]
            assert m == want.size
            np.testing.assert_array_equal(g.perm[:m].cpu().numpy(), want)
            ks = np.stack([kz[want], k2[want] if two else np.zeros(m)], 1)
            heads = np.r_[0, np.flatnonzero(np.any(ks[1:] != ks[:-1], 1)) + 1] if m else []
            assert ns == len(heads)
            np.testing.assert_array_equal(g.seg[:ns + 1].cpu().numpy(), np.r_[heads, m])


def test_helpers_vs_pandas(engine):
    """classify_lick_state, pull_lick_from_bout, event_interactions_dummies,
    add_heatmap_columns called on their own, as notebooks do."""
    import pp_design_mat as D
    ts, tr = session(150, 7)
    ts["Lick"] = (~np.isnan(ts.iSpout)).astype("int")
    states = ["Select", "Consumption", "ENLP"]
    a = D.classify_lick_state(ts, states)
    b = P.lick_states(ts, states)
    assert_same_frame(a, b)
    for pos, keep in (([1], False), ([3, 1], True), ([0, 2], False)):
        assert_same_frame(D.pull_lick_from_bout(b, pos, keep_only_nth_lick=keep),
                          P.pull_nth_licks(b, pos, keep_only_nth_lick=keep))
    tri = tr.set_index("nTrial").convert_dtypes()
    pulled = P.pull_nth_licks(b, [1], keep_only_nth_lick=True)
    for states_, tt, drop in ((["Consumption"], "Reward", True), (["Select", "ENLP"], "h2", False)):
        assert_same_frame(
            D.event_interactions_dummies(pulled, tri, states_, tt, drop_non_interaction=drop),
            P.interact(pulled, tri, states_, tt, drop_non_interaction=drop))
    with pytest.raises(UnboundLocalError):
        D.event_interactions_dummies(pulled, tri, ["Consumption"], "Reward", as_dummy=False)
    assert_same_frame(D.add_heatmap_columns(ts, tri), P.heatmap_columns(ts, tri))


def test_errors_like_the_reference(engine):
    import pp_design_mat
    ts, tr = session(20, 9)
    with pytest.raises(KeyError):                  # no state yields 'con_lick' (:51)
        pp_design_mat.make_design_mat(ts.copy(), tr, states=["Select"])
    dup = pd.concat([tr, tr.iloc[:1]])
    with pytest.raises(pd.errors.InvalidIndexError):          # map on a non-unique index
        pp_design_mat.make_design_mat(ts.copy(), dup)


def test_large_session_vs_pandas(engine):
    """20,000 trials (~1.5M rows): the group walks at scale, ordered path."""
    import pp_design_mat
    ts, tr = session(20_000, 11)
    kw = dict(interactions={"Reward": ["Consumption", "Cue"], "h2": ["Select"]})
    ref = P.make_design_mat(ts.copy(), tr, verbose=False, **kw)
    with contextlib.redirect_stdout(io.StringIO()):
        got = pp_design_mat.make_design_mat(ts.copy(), tr, **kw)
    assert_same_frame(got, ref)
