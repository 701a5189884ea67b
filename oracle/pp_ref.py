"""CPU restatement of the reference timeshift expansion — TEST INFRASTRUCTURE.

* ``shift``               — backend/sglm_pp.py:298-357: s > 0 moves rows down (fill on top),
                            s < 0 moves rows up (fill at the bottom).
* ``timeshift``           — backend/sglm_pp.py:23-56 + shifted_cols_to_numpy 409-434.
* ``timeshift_multiple``  — backend/sglm_pp.py:58-103 + concat_all_shifts 436-457
                            (shift-major column order, one block per shift amount).
* ``timeshift_cols_layout`` — backend/sglm_ez.py:102-123 shift list ``[0] + neg..-1 + 1..pos``.
* ``timeshift_by_dict``   — sglm/sglm/features/setup_model_fit.py:43-96 (event-major, lag 0
                            duplicated, NaN rows at the extreme lags dropped).

numpy only; pinned by the known answers of backend/test/test_sglm_pp.py:20-151.
"""
from __future__ import annotations

import numpy as np


def shift(a, s, fill_value=np.nan):
    a = np.asarray(a)
    if s == 0:
        return a
    blanks = np.ones((abs(s), a.shape[1])) * fill_value
    if s > 0:
        return np.concatenate((blanks, a), axis=0)[:-s, :]
    return np.concatenate((a, blanks), axis=0)[-s:, :]


def timeshift(X, shift_inx=(), shift_amt=1, keep_non_inx=False, fill_value=np.nan):
    X = np.asarray(X)
    inx = list(range(X.shape[1])) if len(shift_inx) == 0 else list(shift_inx)
    shifted = shift(X[:, inx], shift_amt, fill_value)
    if keep_non_inx:
        out = X.copy()
        out[:, inx] = shifted
        return out
    return shifted.copy()


def timeshift_multiple(X, shift_inx=(), shift_amt_list=(-1, 0, 1), unshifted_keep_all=True,
                       fill_value=np.nan):
    blocks = [timeshift(X, shift_inx, s, keep_non_inx=(s == 0 and unshifted_keep_all),
                        fill_value=fill_value) for s in shift_amt_list]
    return np.concatenate(blocks, axis=1)


def shift_list(neg_order, pos_order):
    return [0] + list(range(neg_order, 0)) + list(range(1, pos_order + 1))


def timeshift_by_dict(X, orders, keep_nans=False):
    """Event-major expansion: X columns, then for each column c: lags neg_c..pos_c (incl. 0)."""
    X = np.asarray(X, dtype=np.float64)
    blocks = [X]
    where = {}
    col = X.shape[1]
    neg = pos = None
    for c, (neg, pos) in orders.items():
        for s in range(neg, pos + 1):
            blocks.append(shift(X[:, [c]], s, np.nan))
            where[(c, s)] = col
            col += 1
    # setup_model_fit.py:88-94 drops on '<col>_<neg>' / '<col>_<pos>' using the orders of
    # the LAST dict entry for every column (loop-variable reuse), if such a column exists.
    extreme = [where[(c, s)] for s in (neg, pos) for c in orders if (c, s) in where]
    out = np.concatenate(blocks, axis=1)
    if not keep_nans and extreme:
        out = out[~np.isnan(out[:, extreme]).any(axis=1)]
    return out
