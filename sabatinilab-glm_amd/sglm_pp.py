"""Drop-in for ``backend/sglm_pp.py`` (import as ``import sglm_pp``).

The lag expansion (``shift`` / ``timeshift`` / ``timeshift_multiple``; backend/sglm_pp.py:
23-103, 298-486) runs on the MI355X through ``sglm_timeshift_expand`` — one kernel for all
requested (column, shift) pairs instead of one thread + np.concatenate per shift.  pandas
bookkeeping (column names ``f"{col}_{s}"``, shift-major block order, dtype behaviour of the
reference's ``iloc`` assignments) is reproduced on the host.

Fold generation (``bucket_ids_by_timeframe``, ``cv_idx_from_bucket_ids``) is host integer
work, bit-exact with the reference's sklearn ``GroupShuffleSplit`` (see sglm_hip.folds).
``zscore`` / ``diff`` / ``detrend_data`` are cheap host preprocessing, out of the GPU scope
 and kept as numpy/pandas.
"""
from __future__ import annotations

from typing import List, Optional, Union

import numpy as np
import pandas as pd
import scipy.signal  # noqa: F401  (reference imports it; kept for API parity)

from sglm_hip import folds as _folds
from sglm_hip.lagframe import LagFrame
from sglm_hip.timeshift import shift_columns as _shift_columns

# timeshift_multiple on a DataFrame returns a device-resident LagFrame (SGLM_LAGFRAME=0: the
# materialised DataFrame)
LAGFRAME = __import__("os").environ.get("SGLM_LAGFRAME", "1") == "1"


# ----------------------------------------------------------------------------- helpers
def get_numpy_version(X: Union[np.ndarray, pd.DataFrame]) -> np.ndarray:
    return X.values if type(X) == pd.DataFrame else X


def _shift_dtype(arr: np.ndarray, shift_amt: int, fill_value) -> np.dtype:
    """dtype the reference's np.concatenate([ones*fill, X]) produces (sglm_pp.py:312-357)."""
    if shift_amt == 0:
        return arr.dtype
    return np.result_type(arr.dtype, np.asarray(np.ones(1) * fill_value).dtype)


def shift(setup_array: np.ndarray, shift_amt: int, fill_value: Optional[float] = np.nan) -> np.ndarray:
    """Shift all columns down (s > 0) or up (s < 0); backend/sglm_pp.py:298-319."""
    setup_array = np.asarray(setup_array)
    if shift_amt == 0:
        return setup_array
    dt = _shift_dtype(setup_array, shift_amt, fill_value)
    m = setup_array.shape[1]
    return _shift_columns(setup_array.astype(dt, copy=False), np.arange(m), np.full(m, shift_amt),
                          fill_value, dt)


def concat_start_crop_end(blanks: np.ndarray, X_to_shift: np.ndarray):
    return shift(X_to_shift, blanks.shape[0], blanks.reshape(-1)[0] if blanks.size else np.nan)


def concat_end_crop_start(blanks: np.ndarray, X_to_shift: np.ndarray):
    return shift(X_to_shift, -blanks.shape[0], blanks.reshape(-1)[0] if blanks.size else np.nan)


def shifted_cols_to_pandas(X: pd.DataFrame, shifted_X: np.ndarray, shift_inx: list,
                           keep_non_inx: bool) -> pd.DataFrame:
    return_setup = X.copy()
    # column-by-position replacement: the shifted column's dtype (float64 when NaN-filled)
    # replaces the original, as iloc assignment upcast under the reference's pandas 1.1.3;
    # an in-place iloc write into int columns is deprecated in pandas 2
    shifted_X = np.asarray(shifted_X)
    for q, col in enumerate(np.atleast_1d(shift_inx)):
        return_setup.isetitem(int(col), shifted_X[:, q])
    if not keep_non_inx:
        return_setup = return_setup.iloc[:, shift_inx]
    return return_setup


def shifted_cols_to_numpy(X: np.ndarray, shifted_X: np.ndarray, shift_inx: list,
                          keep_non_inx: bool) -> np.ndarray:
    if keep_non_inx:
        return_setup = X.copy()
        return_setup[:, shift_inx] = shifted_X
    else:
        return_setup = shifted_X.copy()
    return return_setup


def shifted_cols_to_original_type(X, shifted_X, shift_inx, keep_non_inx):
    if type(X) == pd.DataFrame:
        return shifted_cols_to_pandas(X, shifted_X, shift_inx, keep_non_inx)
    return shifted_cols_to_numpy(X, shifted_X, shift_inx, keep_non_inx)


# ----------------------------------------------------------------------------- timeshift
def timeshift(X, shift_inx=[], shift_amt=1, keep_non_inx=False, dct=None, fill_value=np.nan):
    """backend/sglm_pp.py:23-56."""
    npX = np.asarray(get_numpy_version(X))
    shift_inx = list(range(npX.shape[1])) if len(shift_inx) == 0 else list(shift_inx)
    if shift_amt == 0:
        shifted_X = npX[:, shift_inx]
    else:
        dt = _shift_dtype(npX, shift_amt, fill_value)
        shifted_X = _shift_columns(npX.astype(dt, copy=False), shift_inx,
                                   np.full(len(shift_inx), shift_amt), fill_value, dt)
    out = shifted_cols_to_original_type(X, shifted_X, shift_inx, keep_non_inx)
    if dct is not None:
        dct[shift_amt] = out
    return out


def timeshift_multiple(X, shift_inx=[], shift_amt_list=[-1, 0, 1], unshifted_keep_all=True,
                       fill_value=np.nan):
    """backend/sglm_pp.py:58-103: all shifts in one kernel launch, shift-major blocks.

    A DataFrame input with the reference's NaN fill returns a ``LagFrame``
    (sglm_hip.lagframe): the same columns, index and values, with the lag columns kept as
    (source column, shift) specs over a device copy of the shifted columns instead of a
    materialised N x (m K) float64 block -- the NaN filter, the trial-id folds and the fits of
    the production flow read them there; any other use materialises them (``to_pandas()``).
    SGLM_LAGFRAME=0 returns the materialised DataFrame."""
    if isinstance(X, LagFrame):
        X = X.to_pandas()
    if (type(X) == pd.DataFrame and LAGFRAME and isinstance(fill_value, float)
            and np.isnan(fill_value)
            and len(shift_amt_list) > 0):
        inx = list(range(X.shape[1])) if len(shift_inx) == 0 else list(shift_inx)
        if all(pd.api.types.is_numeric_dtype(X.dtypes.iloc[i]) for i in inx):
            lf = LagFrame.from_shifts(X, shift_inx, shift_amt_list, unshifted_keep_all)
            if lf is not None:
                return lf
    npX = np.asarray(get_numpy_version(X))
    inx = list(range(npX.shape[1])) if len(shift_inx) == 0 else list(shift_inx)
    nz = [s for s in shift_amt_list if s != 0]
    shifted = {}
    if nz:
        dt = _shift_dtype(npX, 1, fill_value)
        cols = np.tile(np.asarray(inx), len(nz))
        shs = np.repeat(np.asarray(nz), len(inx))
        allv = _shift_columns(npX.astype(dt, copy=False), cols, shs, fill_value, dt)
        for b, s in enumerate(nz):
            shifted[s] = allv[:, b * len(inx):(b + 1) * len(inx)]
    blocks = []
    for s in shift_amt_list:
        keep = (s == 0 and unshifted_keep_all)
        sx = npX[:, inx] if s == 0 else shifted[s]
        blocks.append(shifted_cols_to_original_type(X, sx, inx, keep))
    return concat_all_shifts(X, shift_amt_list, blocks)


def concat_all_shifts(X, shift_amt_list: List[int], shifted_list):
    if type(X) == pd.DataFrame:
        return concat_pandas_shifts(shift_amt_list, shifted_list)
    return np.concatenate(shifted_list, axis=1)


def concat_pandas_shifts(shift_amt_list, shifted_list):
    ret = []
    for isa, shift_amt in enumerate(shift_amt_list):
        col_names = shifted_list[isa].columns
        sft = [f"{_}_{shift_amt}" for _ in col_names] if shift_amt != 0 else col_names
        ret.append(shifted_list[isa][col_names].rename(
            {col_names[i]: sft[i] for i in range(len(sft))}, axis=1))
    return pd.concat(ret, axis=1)


# ----------------------------------------------------------------------------- prep (host)
def zscore(X):
    """backend/sglm_pp.py:105-117."""
    return (X - X.mean(axis=0)) / X.std(axis=0)


def diff(X, diff_inx=[], n=1, axis=0, append_to_base=False, fill_value=np.nan, **kwargs):
    """backend/sglm_pp.py:120-190 (host numpy/pandas; not on the GPU path)."""
    typ = type(X)
    typ = pd.DataFrame if typ == pd.Series and append_to_base else typ
    if type(X) == pd.Series:
        X = pd.DataFrame(X)
    diff_inx = diff_inx if diff_inx else list(range(X.shape[1]))
    if type(X) == pd.DataFrame:
        column_names = [_ + '_diff' for _ in X.columns[diff_inx]]
        if append_to_base:
            column_names = list(X.columns) + column_names
        X_val = X.values
    else:
        X_val = X
    if len(X.shape) == 1:
        X_val = X_val.reshape((-1, 1))
    ret = np.diff(X_val[:, diff_inx], n=n, axis=axis, **kwargs)
    index = None
    if append_to_base:
        ret = np.concatenate([np.ones((n, ret.shape[1])) * fill_value, ret], axis=0)
        ret = np.concatenate([X_val, ret], axis=-1)
        if type(X) == pd.DataFrame:
            index = X.index
    elif type(X) == pd.DataFrame:
        index = X.index[1:]
    if type(X) == pd.DataFrame:
        ret = pd.DataFrame(ret, columns=column_names, index=index)
    if typ == pd.Series:
        ret = ret.iloc[:, 0]
    return ret


def get_column_nums(df, column_names=[]):
    """backend/sglm_pp.py:192-209."""
    ret = [df.columns.get_loc(_) for _ in column_names]
    if len([_ for _ in ret if type(_) == np.ndarray]):
        raise ValueError('Duplicate column found in X column names.')
    return ret


# ----------------------------------------------------------------------------- folds
def bucket_ids_by_timeframe(total_timesteps, timesteps_per_bucket=20):
    return _folds.bucket_ids_by_timeframe(total_timesteps, timesteps_per_bucket)


def cv_idx_from_bucket_ids(bucket_ids, X, y=None, num_folds=None, test_size=None):
    """backend/sglm_pp.py:236-264 — bit-exact GroupShuffleSplit on the global RNG."""
    return _folds.cv_idx_from_bucket_ids(np.asarray(bucket_ids), X, y, num_folds, test_size)


# ----------------------------------------------------------------------------- misc (host)
def min_max_scale(X, lower_bound, upper_bound):
    return (X - lower_bound) / (upper_bound - lower_bound)


def lambda_min_max(X: pd.Series) -> float:
    lower_bound = X.quantile(0.05)
    upper_bound = X.quantile(0.95)
    return min_max_scale(X.iloc[(len(X) + 1) // 2 - 1], lower_bound, upper_bound)


def detrend_data(X: pd.DataFrame, detrend_col: str, grouping_cols: List[str], window: int,
                 standardize: Optional[bool] = False) -> pd.DataFrame:
    if grouping_cols:
        return X.groupby(grouping_cols)[detrend_col].rolling(window=window * 2, center=True).apply(lambda_min_max)
    return X[detrend_col].rolling(window=window * 2, center=True).apply(lambda_min_max)
