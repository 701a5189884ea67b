"""``sglm.features.setup_model_fit`` (sglm/sglm/features/setup_model_fit.py): the package's
event-major lag expansion and the per-file analysis preparation built on it.

``timeshift_vals_by_dict`` (:43-96) restated: the original frame, then for every column of
the dict (in dict order) its lags neg..pos INCLUDING 0 (so ``col_0`` duplicates ``col``),
named ``f"{col}_{s}"``, each ``df[[col]].shift(s)`` (NaN fill, integer columns promoted to
float64 as pandas does); unless ``keep_nans``, rows with a NaN in an extreme-lag column are
dropped — the reference builds that subset from the (neg, pos) of the LAST dict entry for
every column (its loop variables leak, :88-94), which is kept.  All lags of one dtype group
are produced by ONE launch of the HIP lag kernel (``sglm_timeshift_expand``)."""
import numpy as np
import pandas as pd

from sglm.features import sglm_pp
from sglm_hip.timeshift import shift_columns


def timeshift_vals(dfrel, X_cols, neg_order=-20, pos_order=20, exclude_columns=None):
    """setup_model_fit.py:12-40."""
    if exclude_columns is not None:
        X_cols_reduced = [_ for _ in X_cols if _ not in exclude_columns]
    else:
        X_cols_reduced = X_cols
    dfrel = sglm_pp.timeshift_cols(dfrel, X_cols_reduced, neg_order=neg_order,
                                   pos_order=pos_order)
    X_cols_sftd = sglm_pp.add_timeshifts_to_col_list(X_cols, X_cols_reduced,
                                                     neg_order=neg_order, pos_order=pos_order)
    return dfrel, X_cols_sftd


def _shifted_dtype(dt):
    dt = np.dtype(dt)
    if dt.kind == "f":
        return dt
    if dt.kind in "iub":
        return np.dtype(np.float64)           # pandas promotes ints to float64 for the NaN
                                              # fill (bools to object: converted back below)
    raise TypeError(f"timeshift_vals_by_dict: column dtype {dt} is not numeric")


def timeshift_vals_by_dict(df, X_cols_dict, keep_nans=False):
    """setup_model_fit.py:43-96 -> (expanded frame, list of shifted column names)."""
    df = df.copy()
    names, pairs = [], []                      # (column, shift) in the reference's order
    neg_order = pos_order = None
    for X_col in X_cols_dict:
        neg_order, pos_order = X_cols_dict[X_col]
        for s in range(neg_order, pos_order + 1):
            pairs.append((X_col, s))
            names.append(X_col + '_' + str(s))
    blocks = {}
    groups = {}
    for j, (c, s) in enumerate(pairs):
        if s == 0:                             # shift(0) keeps the column and its dtype
            blocks[j] = df[c].values.copy()
            continue
        groups.setdefault(_shifted_dtype(df[c].dtype), []).append(j)
    for dt, js in groups.items():
        cols = sorted({pairs[j][0] for j in js}, key=list(df.columns).index)
        A = df[cols].to_numpy(dtype=dt)
        where = {c: i for i, c in enumerate(cols)}
        out = shift_columns(A, [where[pairs[j][0]] for j in js], [pairs[j][1] for j in js],
                            np.nan, dt)
        for k, j in enumerate(js):
            v = out[:, k]
            if df[pairs[j][0]].dtype.kind == "b":  # pandas: bool shifted with NaN -> object
                v = pd.Series(v).map({1.0: True, 0.0: False}).values
            blocks[j] = v
    shifted = pd.DataFrame({names[j]: blocks[j] for j in range(len(pairs))}, index=df.index)
    df = pd.concat([df, shifted], axis=1)
    if not keep_nans:
        na_drop_cols = ([X_col + '_' + str(neg_order) for X_col in X_cols_dict] +
                        [X_col + '_' + str(pos_order) for X_col in X_cols_dict])
        na_drop_cols = [_ for _ in na_drop_cols if _ in df.columns]
        df = df.dropna(subset=na_drop_cols)
    return df, list(names)


def X_cols_dict_to_default(X_cols_dict, neg_order=-20, pos_order=20):
    """setup_model_fit.py:98-105."""
    X_cols_dict = X_cols_dict.copy()
    for X_col in X_cols_dict:
        if X_cols_dict[X_col] == (0, 0) or X_cols_dict[X_col] is None:
            X_cols_dict[X_col] = (neg_order, pos_order)
    return X_cols_dict


def xy_pairs_to_widest_orders(X_y_pairings):
    """setup_model_fit.py:108-132."""
    widest = {}
    for xy_pair in X_y_pairings:
        X_dict = xy_pair['X_cols']
        for X_col in X_dict:
            neg_order, pos_order = X_dict[X_col][0], X_dict[X_col][1]
            if X_col not in widest:
                widest[X_col] = (neg_order, pos_order)
                continue
            lo, hi = widest[X_col]
            widest[X_col] = (min(lo, neg_order), max(hi, pos_order))
    return widest


def _read_signal_file(signal_fn, file_num, file_ids):
    df = pd.read_csv(signal_fn, index_col='index').copy()
    df['file_num'] = file_num
    df['signal_file'] = None if file_ids is None else file_ids[file_num]
    return df


def multi_file_analysis_prep(signal_files, X_cols_dict, file_ids=None):
    """setup_model_fit.py:135-183: shift per file (lags never cross sessions), concat, then
    the file-qualified trial ids."""
    signal_df_lst, X_cols_sftd_lst = [], []
    for file_num, signal_fn in enumerate(signal_files):
        tmp, sftd = timeshift_vals_by_dict(_read_signal_file(signal_fn, file_num, file_ids),
                                           X_cols_dict)
        signal_df_lst.append(tmp)
        X_cols_sftd_lst += [_ for _ in sftd if _ not in X_cols_sftd_lst]
    signal_df = pd.concat(signal_df_lst, axis=0).copy()
    signal_df['nTrial'] = signal_df['nTrial'].astype(int)
    signal_df['nEndTrial'] = signal_df['nEndTrial'].astype(int)
    max_num_trial = len(str(signal_df['nTrial'].max()))
    signal_df['nTrial_filenum'] = signal_df['nTrial'] + signal_df['file_num'] * 10 ** max_num_trial
    signal_df['nEndTrial_filenum'] = (signal_df['nEndTrial'] +
                                      signal_df['file_num'] * 10 ** max_num_trial)
    return [signal_df], X_cols_sftd_lst, None


def single_file_analysis_prep(signal_files, X_cols_dict, file_ids=None):
    """setup_model_fit.py:186-233."""
    X_cols_sftd_lst, signal_df_lst, signal_filenames = [], [], []
    for file_num, signal_fn in enumerate(signal_files):
        tmp = _read_signal_file(signal_fn, file_num, file_ids)
        tmp['nTrial'] = tmp['nTrial'].astype(int)
        tmp['nEndTrial'] = tmp['nEndTrial'].astype(int)
        max_num_trial = len(str(tmp['nTrial'].max()))
        tmp['nTrial_filenum'] = tmp['nTrial'] + tmp['file_num'] * 10 ** max_num_trial
        tmp['nEndTrial_filenum'] = tmp['nEndTrial'] + tmp['file_num'] * 10 ** max_num_trial
        tmp, sftd = timeshift_vals_by_dict(tmp, X_cols_dict)
        X_cols_sftd_lst += [_ for _ in sftd if _ not in X_cols_sftd_lst]
        signal_df_lst.append(tmp)
        signal_filenames.append(signal_fn.split('/')[-1].split('.')[0]
                                .replace('GLM_SIGNALS_', '').replace('INTERIM_', ''))
    return signal_df_lst, X_cols_sftd_lst, signal_filenames
