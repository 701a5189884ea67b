"""CPU restatement of gen_signal_df.generate_signal_df (sglm/sglm/features/gen_signal_df.py:
327-470) -- TEST INFRASTRUCTURE (tests/ and bench.py's cpu_baseline leg only; the product is
sglm/features/gen_signal_df.py over the HIP kernels).

* ``ab_labels`` restates generate_Ab_labels (:112-157) as numpy boolean logic: the previous
  trial's values come from shift(1), whose leading NaN is True under astype(bool) (:129-131).
* ``repair_center_out`` restates replace_missed_center_out_indexes (:159-210) as an explicit
  walk over adjacent trials.
* ``signal_frame`` aligns the trial table onto the signal with ``Series.reindex`` (the
  mechanism behind the reference's label-aligned column assignment, :416-427), takes nTrial /
  nEndTrial from pandas cumsum + shift (:430-434) and runs the per-trial duplication loop over
  ``pd.unique`` of nTrial exactly as the reference does (:437-462).
* ``row_map_sorted`` is a second, sort-based formulation of that loop's row order (copies of
  a run's diffTrialNums > 1 rows first, then the run; NaN runs dropped) for sizes the loop
  cannot reach.

The reference pins pandas 1.1.3, whose get_dummies gives uint8 indicators; they are cast to
uint8 here so that alignment yields float64 under any pandas.  Parity pinning: the reference
cannot be imported here and its repository holds no fixture for this
function, so the restatement is pinned by pandas' own semantics of the operations it uses and
by the hand-computed cases in tests/test_signal_cpu.py.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

INDEX_COLS = ['photometryCenterInIndex', 'photometryCenterOutIndex', 'photometrySideInIndex',
              'photometrySideOutIndex', 'photometryFirstLickIndex']
BASIS = ['AA', 'Aa', 'aA', 'aa', 'AB', 'Ab', 'aB', 'ab']
SIDE_COLS = ('photometrySideInIndex', 'photometrySideOutIndex')


def ab_labels(rewarded, chose_left, chose_right):
    """(label, label_side, label_rewarded) string arrays of generate_Ab_labels."""
    rew = np.asarray(pd.Series(rewarded).astype(bool))
    left, right = np.asarray(chose_left), np.asarray(chose_right)
    prv = np.r_[True, rew[:-1]] if rew.size else rew
    prv_left = np.r_[True, left[:-1].astype(bool)] if rew.size else rew
    prv_right = np.r_[True, right[:-1].astype(bool)] if rew.size else rew
    same = (left == prv_left) & (right == prv_right)
    c0 = np.where(prv, 'A', 'a')
    c1 = np.select([same & rew, ~same & rew, same & ~rew], ['A', 'B', 'a'], 'b')
    rb, pr = right.astype(bool), prv_right.astype(bool)
    s0 = np.select([pr & prv, ~pr & prv, pr & ~prv], ['R', 'L', 'r'], 'l')
    s1 = np.select([rb & rew, ~rb & rew, rb & ~rew], ['R', 'L', 'r'], 'l')
    lab = np.char.add(c0, c1).astype(object)
    side = np.char.add(s0, s1).astype(object)
    return lab, side, np.where(rew, 'A', 'a').astype(object)


def repair_center_out(ci, co):
    """replace_missed_center_out_indexes: while a positive center-out index is repeated or
    a trial's center out is at or after the next trial's, set it to the trial's center in."""
    co = np.array(co, dtype=np.float64)
    ci = np.asarray(ci, dtype=np.float64)
    while True:
        vals = co[co > 0]
        most = np.unique(vals, return_counts=True)[1].max() if vals.size else np.nan
        nxt = np.r_[co[1:], np.nan]
        hit = (co >= nxt) & (nxt > 0) & (co > 0)
        co[hit] = ci[hit]
        if most == 1 and not hit.any():
            return co


def trial_table(table_df, index_cols=INDEX_COLS, basis=BASIS):
    """generate_signal_df's table steps (:376-391): labels, the word check, uint8 indicators of
    every basis label, MATLAB -> Python indices, the center-out repair."""
    t = table_df.copy()
    lab, _, _ = ab_labels(t['wasRewarded'], t['choseLeft'], t['choseRight'])
    t['label'] = lab
    t['wasRewarded'] = np.asarray(t['wasRewarded'].astype(bool)).astype(np.int64)
    t = t.dropna()
    assert (t['label'] == t['word']).all()
    for b in basis:
        t[b] = (t['label'] == b).astype(np.uint8)
    for c in index_cols:
        t[c] = t[c] - 1
    t['photometryCenterOutIndex'] = repair_center_out(t['photometryCenterInIndex'],
                                                      t['photometryCenterOutIndex'])
    return t


def signal_frame(signal_df, table_df, index_cols=INDEX_COLS, basis=BASIS, k_before=-20,
                 k_after=20):
    """(signal_df, table_df) as generate_signal_df returns them."""
    t = trial_table(table_df, index_cols, basis)
    sig = signal_df.copy()
    for col in index_cols:
        sel = t[(t['hasAllPhotometryData'] > 0) & (t[col] >= 0)].set_index(col)
        r = sel['wasRewarded']
        sig[col] = ((r == r) * 1).reindex(sig.index)
        sig[col + 'r'] = r.reindex(sig.index)
        sig[col + 'nr'] = 1 - sig[col + 'r']
        if col in SIDE_COLS:
            for b in basis:
                sig[col + b] = sel[b].fillna(0).reindex(sig.index)
    starts = ((sig['photometryCenterInIndex'] == 1) & sig['photometryCenterInIndex'].notna()) * 1
    ends = ((sig['photometrySideOutIndex'] == 1) & sig['photometrySideOutIndex'].notna()) * 1
    sig['nTrial'] = starts.cumsum().shift(k_before)
    sig['nEndTrial'] = ends.cumsum().shift(k_after)
    sig['diffTrialNums'] = sig['nTrial'] - sig['nEndTrial']
    sig['dupe'] = False
    pieces = []
    for v in pd.unique(sig['nTrial']):
        run = sig[sig['nTrial'] == v]
        extra = run[run['diffTrialNums'] > 1].copy()
        if len(extra):
            extra['nTrial'] = extra['nTrial'] - 1
            extra['dupe'] = True
            pieces.append(extra)
        pieces.append(run)
    out = pd.concat(pieces, axis=0)
    out['wi_trial_keep'] = out['nTrial'] != out['nEndTrial']
    return out, table_df


def shifted_counts(center_in, side_out, k_before, k_after):
    """nTrial, nEndTrial, diffTrialNums as float64 arrays (numpy)."""
    def shift(x, k):
        y = np.full(x.size, np.nan)
        if k >= 0:
            y[k:] = x[:x.size - k] if k < x.size else []
        else:
            y[:k] = x[-k:] if -k < x.size else []
        return y
    a = shift(np.cumsum(np.asarray(center_in) == 1).astype(np.float64), k_before)
    b = shift(np.cumsum(np.asarray(side_out) == 1).astype(np.float64), k_after)
    return a, b, a - b


def row_map_sorted(ntrial, diff):
    """(src, dupe) of the duplication loop by sorting: rows keyed (nTrial, copy-before-row,
    position); nTrial is a shifted cumulative count, so its runs are contiguous and ordered."""
    ntrial = np.asarray(ntrial, dtype=np.float64)
    idx = np.flatnonzero(~np.isnan(ntrial))
    with np.errstate(invalid='ignore'):
        cp = idx[np.asarray(diff)[idx] > 1]
    src = np.concatenate([cp, idx])
    first = np.concatenate([np.zeros(cp.size, np.int8), np.ones(idx.size, np.int8)])
    order = np.lexsort((src, first, ntrial[src]))
    return src[order], first[order] == 0


def synthetic_session(n_trials, seed, **kw):
    """The seeded session generator of the product's synthetic data (sglm_hip/synth.py)."""
    from sglm_hip import synth
    return synth.signal_session(n_trials, seed, **kw)
