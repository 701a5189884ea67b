"""gen_signal_df.generate_signal_df on the MI355X (sglm_scatter_rows + sglm_signal_trials
through the C ABI) vs the CPU oracle (oracle/signal_ref.py): the whole output frame --
values, NaN positions, dtypes, column order, row order and index labels (duplicated rows keep
their label) -- must be identical."""
import numpy as np
import pandas as pd
import pytest

from oracle import signal_ref as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g():
    import torch
    assert torch.cuda.is_available()
    from sglm.features import gen_signal_df
    return gen_signal_df


def _same_frame(a, b):
    pd.testing.assert_frame_equal(a, b, check_exact=True, check_index_type="equiv")


@pytest.mark.parametrize("n_trials,seed,kb,ka", [
    (60, 0, -20, 20), (60, 1, -20, 20), (300, 2, -20, 20), (120, 3, -2, 2), (120, 4, 0, 0),
    (120, 5, 3, -4), (120, 6, -40, 0), (80, 7, 5, 30), (1, 8, -20, 20), (2, 9, -20, 20),
])
def test_signal_frame_vs_oracle(g, n_trials, seed, kb, ka):
    sig, table = ref.synthetic_session(n_trials, seed, past_end=min(2, n_trials - 1))
    out, tab = g.signal_frame(sig, table, trial_bounds_before_center_in=kb,
                              trial_bounds_after_side_out=ka)
    want, _ = ref.signal_frame(sig, table, k_before=kb, k_after=ka)
    _same_frame(out, want)
    assert tab is table
    if (kb, ka) == (-20, 20) and n_trials >= 60:
        assert out["dupe"].any()


def test_signal_shorter_than_bounds(g):
    # every nTrial is NaN: the reference concatenates one empty run -> an empty frame
    sig, table = ref.synthetic_session(3, 10)
    sig = sig.iloc[:15].copy()
    out, _ = g.signal_frame(sig, table)
    want, _ = ref.signal_frame(sig, table)
    assert len(out) == 0 and list(out.columns) == list(want.columns)


def test_empty_signal_raises(g):
    sig, table = ref.synthetic_session(5, 11)
    with pytest.raises(ValueError):
        g.signal_frame(sig.iloc[:0].copy(), table)


def test_duplicate_label_raises(g):
    sig, table = ref.synthetic_session(20, 12)
    table.loc[3, "photometrySideInIndex"] = table.loc[2, "photometrySideInIndex"]
    with pytest.raises(ValueError):
        g.signal_frame(sig, table)


def test_generate_signal_df_csv(g, tmp_path):
    sig, table = ref.synthetic_session(150, 13)
    sp, tp = tmp_path / "signal.csv", tmp_path / "table.csv"
    sig.to_csv(sp, index=False)
    table.to_csv(tp, index=False)
    out, tab = g.generate_signal_df(str(sp), str(tp))
    want, _ = ref.signal_frame(pd.read_csv(sp), pd.read_csv(tp))
    _same_frame(out, want)
    pd.testing.assert_frame_equal(tab, pd.read_csv(tp))


@pytest.mark.parametrize("n,seed", [(2047, 0), (2048, 1), (2049, 2), (3_000_001, 3)])
def test_trial_runs_vs_sorted_formulation(g, n, seed):
    # chunk boundaries of the scans and > 1024 chunks; dense starts / ends so runs are short
    from sglm_hip import signal
    rng = np.random.default_rng(seed)
    ci = np.where(rng.random(n) < 0.02, 1.0, np.nan)
    so = np.where(rng.random(n) < 0.02, 1.0, np.nan)
    for kb, ka in ((-20, 20), (7, -3)):
        nt, ne, d, src, dup = signal.trial_runs(ci, so, kb, ka)
        wnt, wne, wd = ref.shifted_counts(ci, so, kb, ka)
        np.testing.assert_array_equal(nt, wnt)
        np.testing.assert_array_equal(ne, wne)
        np.testing.assert_array_equal(d, wd)
        wsrc, wdup = ref.row_map_sorted(wnt, wd)
        np.testing.assert_array_equal(src, wsrc)
        np.testing.assert_array_equal(dup, wdup)
        assert dup.any() or kb > 0


def test_aligned_columns_labels_outside_signal(g):
    from sglm_hip import signal
    rows = np.array([0, 5, 9, 12, -1], dtype=np.int64)      # 12 and -1 are not signal rows
    vals = np.stack([np.arange(5.0), -np.arange(5.0)])
    out = signal.aligned_columns(10, rows, vals)
    want = np.full((2, 10), np.nan)
    want[:, [0, 5, 9]] = vals[:, :3]
    np.testing.assert_array_equal(out, want)
