"""gen_signal_df.generate_signal_df (sglm/sglm/features/gen_signal_df.py:327-470) on the CPU:
the oracle (oracle/signal_ref.py) against hand-computed cases, its two formulations of the
duplication loop against each other, the drop-in's host-side trial-table steps against the
oracle, and the drop-in refusing to run without the GPU kernels."""
import numpy as np
import pandas as pd
import pytest

from oracle import signal_ref as ref


def _flags(n, rows):
    x = np.full(n, np.nan)
    x[list(rows)] = 1.0
    return x


def test_trial_runs_known_answer():
    # center ins at rows 1, 4; side outs at 3, 6; bounds -2 / +2:
    # cumsum(start) = 0 1 1 1 2 2 2 2 2 2 2 2 -> nTrial = 1 1 2 2 2 2 2 2 2 2 nan nan
    # cumsum(end)   = 0 0 0 1 1 1 2 2 2 2 2 2 -> nEnd   = nan nan 0 0 0 1 1 1 2 2 2 2
    n = 12
    ci, so = _flags(n, (1, 4)), _flags(n, (3, 6))
    nt, ne, d = ref.shifted_counts(ci, so, -2, 2)
    np.testing.assert_array_equal(nt, [1, 1, 2, 2, 2, 2, 2, 2, 2, 2, np.nan, np.nan])
    np.testing.assert_array_equal(ne, [np.nan, np.nan, 0, 0, 0, 1, 1, 1, 2, 2, 2, 2])
    src, dup = ref.row_map_sorted(nt, d)
    np.testing.assert_array_equal(src, [0, 1, 2, 3, 4, 2, 3, 4, 5, 6, 7, 8, 9])
    np.testing.assert_array_equal(dup, [0, 0, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0])
    sig = pd.DataFrame({"x": np.arange(n, dtype=float)})
    sig["photometryCenterInIndex"], sig["photometrySideOutIndex"] = ci, so
    # the loop formulation, on the same columns (no table: drive signal_frame's tail directly)
    sig["nTrial"], sig["nEndTrial"], sig["diffTrialNums"] = nt, ne, d
    pieces = []
    for v in pd.unique(sig["nTrial"]):
        run = sig[sig["nTrial"] == v]
        pieces += [run[run["diffTrialNums"] > 1], run]
    assert list(pd.concat(pieces).index) == list(src)


@pytest.mark.parametrize("kb,ka", [(-20, 20), (-2, 2), (0, 0), (3, -4), (5, 30), (-40, 0)])
@pytest.mark.parametrize("seed", [0, 1])
def test_row_map_two_formulations(seed, kb, ka):
    sig, table = ref.synthetic_session(60, seed)
    out, _ = ref.signal_frame(sig, table, k_before=kb, k_after=ka)
    src, dup = ref.row_map_sorted(*_counts(out, sig, kb, ka))
    np.testing.assert_array_equal(out.index.to_numpy(), src)
    np.testing.assert_array_equal(out["dupe"].to_numpy(), dup)
    if (kb, ka) in ((-20, 20), (-40, 0)):
        assert out["dupe"].any()


def _counts(out, sig, kb, ka):
    # nTrial / diffTrialNums of the signal rows before duplication (NaN for the dropped rows)
    rows = ~out["dupe"].to_numpy()
    base = out[rows]
    nt = np.full(len(sig), np.nan)
    d = np.full(len(sig), np.nan)
    nt[base.index] = base["nTrial"]
    d[base.index] = base["diffTrialNums"]
    return nt, d


@pytest.mark.parametrize("seed", [0, 3, 4])
def test_shifted_counts_match_pandas(seed):
    sig, table = ref.synthetic_session(80, seed)
    out, _ = ref.signal_frame(sig, table)
    t = ref.trial_table(table)
    ci = np.full(len(sig), np.nan)
    so = np.full(len(sig), np.nan)
    for col, arr in (("photometryCenterInIndex", ci), ("photometrySideOutIndex", so)):
        v = t[(t["hasAllPhotometryData"] > 0) & (t[col] >= 0)][col].to_numpy().astype(np.int64)
        arr[v[v < len(sig)]] = 1.0
    nt, ne, d = ref.shifted_counts(ci, so, -20, 20)
    base = out[~out["dupe"]]
    np.testing.assert_array_equal(base["nEndTrial"].to_numpy(), ne[base.index])
    np.testing.assert_array_equal(base["nTrial"].to_numpy(), nt[base.index])


def test_labels_known_answer():
    # previous trial rewarded -> 'A' (first trial: shift(1) NaN is True); current rewarded on
    # the same side -> 'A', other side 'B', unrewarded same 'a', other 'b'
    rew = np.array([1, 1, 0, 0, 1])
    left = np.array([1, 1, 0, 0, 0])
    right = 1 - left
    lab, side, rw = ref.ab_labels(rew, left, right)
    assert list(lab) == ["AB", "AA", "Ab", "aa", "aA"]
    assert list(side) == ["RL", "LL", "Lr", "rr", "rR"]
    assert list(rw) == ["A", "A", "a", "a", "A"]


@pytest.mark.parametrize("seed", [0, 5, 6])
def test_dropin_table_steps_vs_oracle(seed):
    from sglm.features import gen_signal_df as g
    _, table = ref.synthetic_session(200, seed)
    df_t = g.generate_Ab_labels(table)
    lab, side, rw = ref.ab_labels(table["wasRewarded"], table["choseLeft"], table["choseRight"])
    keep = table.dropna().index
    assert df_t.index.equals(keep)
    assert list(df_t["label"]) == list(lab[keep])
    assert list(df_t["label_side"]) == list(side[keep])
    assert list(df_t["label_rewarded"]) == list(rw[keep])
    assert (df_t["label"] == df_t["word"]).all()
    t = df_t.copy()
    t[ref.INDEX_COLS] = g.matlab_indexing_to_python(t[ref.INDEX_COLS])
    fixed = g.replace_missed_center_out_indexes(t)
    want = ref.repair_center_out(t["photometryCenterInIndex"], t["photometryCenterOutIndex"])
    np.testing.assert_array_equal(fixed["photometryCenterOutIndex"].to_numpy(), want)
    changed = (t["photometryCenterOutIndex"].to_numpy() != want).sum()
    assert changed > 0


def test_center_out_repair_known_answer():
    ci = np.array([10., 30., 50., 70.])
    co = np.array([35., 35., 55., 52.])      # trial 0 carried trial 1's center out; 2 > 3
    np.testing.assert_array_equal(ref.repair_center_out(ci, co), [10., 35., 50., 52.])


def test_dropin_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sglm.features import gen_signal_df as g
    from sglm_hip import _lib
    sig, table = ref.synthetic_session(20, 0)
    with pytest.raises(_lib.HipEngineUnavailable):
        g.signal_frame(sig, table)


def test_oracle_duplicate_label_raises():
    sig, table = ref.synthetic_session(20, 1)
    table.loc[3, "photometrySideInIndex"] = table.loc[2, "photometrySideInIndex"]
    with pytest.raises(ValueError):
        ref.signal_frame(sig, table)
