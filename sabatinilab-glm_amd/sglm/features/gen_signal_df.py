"""Drop-in for ``sglm.features.gen_signal_df`` (sglm/sglm/features/gen_signal_df.py): a
photometry signal file (one row per sample) joined with its behaviour trial table (one row per
trial) into the per-sample frame the GLM design is built from.

Trial-level work stays on the host and keeps the reference's pandas semantics (pinned
pandas 1.1.3): the Ab/Rl labels of each trial (``generate_Ab_labels``, :112-157), MATLAB to
Python indices (:225-239), the center-out index repair loop (:159-210).  The per-sample work
runs on the MI355X (``sglm_hip.signal``, csrc/prep.hip):

* every trial-table column the reference aligns onto the signal by index label
  (``signal_df[col] = df_t_tmp.set_index(col)[...]``, :394-427) -- 5 index columns x
  (indicator, rewarded, unrewarded) plus 8 label indicators for the side in/out indices -- is
  one scatter of the trial rows into NaN-filled sample columns (``sglm_scatter_rows``);
* nTrial / nEndTrial (cumulative counts of center-in / side-out samples, shifted by the trial
  bounds, :429-434) are device scans; the per-trial duplication of overlapping samples
  (:437-458) -- a Python loop over every trial value filtering the whole frame, O(trials x
  samples) in the reference -- is a row map built from four scans (``sglm_signal_trials``),
  applied with one ``take``.

Output values and row order are the reference's; the aligned label-indicator columns are
float64 (the pinned pandas gives uint8 dummies, float64 after alignment).
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from sglm_hip import signal as _sig

TABLE_INDEX_COLUMNS = ['photometryCenterInIndex', 'photometryCenterOutIndex',
                       'photometrySideInIndex', 'photometrySideOutIndex',
                       'photometryFirstLickIndex']
BASIS_AA_COLS = ['AA', 'Aa', 'aA', 'aa', 'AB', 'Ab', 'aB', 'ab']
_SIDE_COLS = ('photometrySideInIndex', 'photometrySideOutIndex')


def _put_letters(label_series, loc, cases):
    """Copy of ``label_series`` with the character at ``loc`` replaced by ``char`` on the
    rows of each ``(mask, char)`` case (str.slice_replace on the selected rows)."""
    out = label_series.copy()
    for mask, char in cases:
        mask = pd.Series(mask, index=out.index).astype(bool)
        out.loc[mask] = out.loc[mask].str.slice_replace(loc, loc + 1, char)
    return out


def set_first_prv_trial_letter(prv_wasRewarded_series, label_series, loc=0):
    """'A' where the previous trial was rewarded, 'a' where not (gen_signal_df.py:12-33)."""
    prv = prv_wasRewarded_series
    return _put_letters(label_series, loc, [(prv, 'A'), (~prv, 'a')])


def set_current_trial_letter_switch(sameSide_series, wasRewarded_series, label_series, loc=1):
    """'A'/'B' rewarded on the same/other side, 'a'/'b' unrewarded (gen_signal_df.py:35-62)."""
    same, rew = sameSide_series, wasRewarded_series
    return _put_letters(label_series, loc, [(same & rew, 'A'), (~same & rew, 'B'),
                                            (same & ~rew, 'a'), (~same & ~rew, 'b')])


def set_current_trial_letter_side(choseRight, wasRewarded_series, label_series, loc=2):
    """'R'/'L' rewarded right/left, 'r'/'l' unrewarded (gen_signal_df.py:64-91)."""
    right, rew = choseRight, wasRewarded_series
    return _put_letters(label_series, loc, [(right & rew, 'R'), (~right & rew, 'L'),
                                            (right & ~rew, 'r'), (~right & ~rew, 'l')])


def check_Ab_labels(df_t):
    """The two letters of every label agree with (previous reward, reward, same side)
    (gen_signal_df.py:93-110): code(letter 0) + code(letter 1) == pwR + 2 wR + 4 sS."""
    df_t['pwR'] = df_t['prv_wasRewarded'].astype(int)
    df_t['wR'] = df_t['wasRewarded'].astype(int)
    df_t['sS'] = df_t['sameSide'].astype(int)
    first = df_t['label'].str.slice(0, 1).map({'a': 0, 'A': 1})
    second = df_t['label'].str.slice(1, 2).map({'b': 0, 'B': 2, 'a': 4, 'A': 6})
    assert ((first + second) == (df_t['pwR'] + 2 * df_t['wR'] + 4 * df_t['sS'])).all()


def generate_Ab_labels(df_t):
    """Ab (previous reward, current reward x switch), Rl side and reward labels per trial
    (gen_signal_df.py:112-157)."""
    df_t = df_t.copy()
    rew = df_t['wasRewarded'].astype(bool)
    df_t['wasRewarded'] = rew
    # shift(1) leaves NaN in the first trial, and NaN is truthy under astype(bool)
    df_t['prv_wasRewarded'] = rew.shift(1).astype(bool)
    df_t['prv_choseLeft'] = df_t['choseLeft'].shift(1).astype(bool)
    df_t['prv_choseRight'] = df_t['choseRight'].shift(1).astype(bool)
    df_t['sameSide'] = ((df_t['choseLeft'] == df_t['prv_choseLeft'])
                        & (df_t['choseRight'] == df_t['prv_choseRight'])).astype(bool)
    blank2 = pd.Series('  ', index=df_t.index)
    lab = set_first_prv_trial_letter(df_t['prv_wasRewarded'], blank2, loc=0)
    df_t['label'] = set_current_trial_letter_switch(df_t['sameSide'], rew, lab, loc=1)
    side = set_current_trial_letter_side(df_t['prv_choseRight'], df_t['prv_wasRewarded'],
                                         blank2, loc=0)
    df_t['label_side'] = set_current_trial_letter_side(df_t['choseRight'], rew, side, loc=1)
    df_t['label_rewarded'] = set_first_prv_trial_letter(rew, pd.Series(' ', index=df_t.index),
                                                        loc=0)
    for c in ('wasRewarded', 'prv_wasRewarded', 'prv_choseLeft', 'prv_choseRight'):
        df_t[c] = df_t[c].fillna(False).astype(int)
    df_t = df_t.dropna()
    check_Ab_labels(df_t)
    return df_t


def replace_missed_center_out_indexes(df_t, max_num_duplications=None, verbose=0):
    """Repeatedly set a center-out index that equals or exceeds the next trial's (a center out
    the detector carried into the next sample) to the trial's center-in index, until every
    positive center-out index is unique and increasing (gen_signal_df.py:159-210)."""
    df_t = df_t.copy()
    co = 'photometryCenterOutIndex'
    i = 0
    while True:
        pos = df_t[co] > 0
        counts = df_t.loc[pos, co].value_counts()
        top = counts.max() if len(counts) else np.nan
        nxt = df_t[co].shift(-1)
        hit = (df_t[co] >= nxt) & (nxt > 0) & pos
        df_t.loc[hit, co] = df_t.loc[hit, 'photometryCenterInIndex']
        if top == 1 and not hit.any():
            break
        if max_num_duplications and i > max_num_duplications:
            break
        i += 1
    if verbose > 0:
        print('# of iterations', i, '— Final max amount of duplicated Center Out Indices:', top)
    return df_t


def get_is_relevant_trial(hasAllData_srs, index_event_srs):
    return (hasAllData_srs > 0) & (index_event_srs >= 0)


def matlab_indexing_to_python(index_event_srs):
    return index_event_srs - 1


def get_is_not_iti(df):
    return df['nTrial'] != df['nEndTrial']


def get_trial_start(center_in_srs):
    return ((~center_in_srs.isna()) & (center_in_srs == 1)) * 1


def get_trial_end(center_out_srs):
    return ((~center_out_srs.isna()) & (center_out_srs == 1)) * 1


def signal_frame(signal_df, table_df, table_index_columns=TABLE_INDEX_COLUMNS,
                 basis_Aa_cols=BASIS_AA_COLS, trial_bounds_before_center_in=-20,
                 trial_bounds_after_side_out=20):
    """``generate_signal_df`` on frames already read (signal rows, trial table)."""
    signal_df = signal_df.copy()
    df_t = generate_Ab_labels(table_df)
    assert np.all(df_t['label'].dropna() == df_t['word'].dropna())
    dummies = pd.get_dummies(df_t['label'])
    for b in basis_Aa_cols:
        if b not in dummies.columns:
            df_t[b] = 0
    df_t[dummies.columns] = dummies
    df_t[table_index_columns] = matlab_indexing_to_python(df_t[table_index_columns])
    df_t = replace_missed_center_out_indexes(df_t, verbose=1)
    if signal_df.index.nunique() != len(signal_df.index):
        raise AssertionError("Error: Duplicate entries in signal_df.index")
    n = len(signal_df)
    # the signal's index labels -> positions (pandas aligns by label)
    labels = signal_df.index
    for col in table_index_columns:
        if [c for c in df_t.columns if c == col] != [col]:
            raise AssertionError(f"Error: Duplicate entries for {col}")
        tr = df_t[get_is_relevant_trial(df_t['hasAllPhotometryData'], df_t[col])]
        key = tr[col]
        if key.duplicated().any():
            raise ValueError("cannot reindex on an axis with duplicate labels")
        pos = labels.get_indexer(key.values)
        keep = pos >= 0
        r = tr['wasRewarded'].to_numpy(dtype=np.float64)
        vals = [np.where(r == r, 1.0, 0.0), r, 1.0 - r]
        names = [col, f'{col}r', f'{col}nr']
        if col in _SIDE_COLS:
            for b in basis_Aa_cols:
                vals.append(tr[b].fillna(0).to_numpy(dtype=np.float64))
                names.append(col + b)
        out = _sig.aligned_columns(n, pos[keep], np.stack(vals)[:, keep])
        for name, v in zip(names, out):
            signal_df[name] = v
    if n == 0:
        # the reference's loop runs over no nTrial value and concatenates nothing
        raise ValueError("No objects to concatenate")
    ntrial, nend, diff, src, dup = _sig.trial_runs(
        signal_df['photometryCenterInIndex'].to_numpy(dtype=np.float64),
        signal_df['photometrySideOutIndex'].to_numpy(dtype=np.float64),
        trial_bounds_before_center_in, trial_bounds_after_side_out)
    # an unshifted cumulative count stays int64 in pandas (no NaN introduced)
    if trial_bounds_before_center_in == 0:
        ntrial = ntrial.astype(np.int64)
    if trial_bounds_after_side_out == 0:
        nend = nend.astype(np.int64)
    if ntrial.dtype == nend.dtype == np.int64:
        diff = diff.astype(np.int64)
    signal_df['nTrial'] = ntrial
    signal_df['nEndTrial'] = nend
    signal_df['diffTrialNums'] = diff
    signal_df['dupe'] = False
    out = signal_df.take(src)
    out['nTrial'] = ntrial[src] - dup.astype(ntrial.dtype)
    out['dupe'] = dup
    out['wi_trial_keep'] = get_is_not_iti(out)
    return out, table_df


def generate_signal_df(signal_filename, table_filename,
                       table_index_columns=TABLE_INDEX_COLUMNS, basis_Aa_cols=BASIS_AA_COLS,
                       trial_bounds_before_center_in=-20, trial_bounds_after_side_out=20):
    """Same signature and return value as the reference (gen_signal_df.py:327-470):
    (signal_df, table_df)."""
    return signal_frame(pd.read_csv(signal_filename), pd.read_csv(table_filename),
                        table_index_columns, basis_Aa_cols, trial_bounds_before_center_in,
                        trial_bounds_after_side_out)
