"""Drop-in for the hot-path part of ``backend/sglm_ez.py`` (import as ``import sglm_ez``).

Timeshift helpers (:14-147) call the GPU lag kernel through ``sglm_pp``; fold helpers
(:193-343) are bit-exact host integer work; ``simple_cv_fit`` (:347-389) and
``training_fit_holdout_score`` (:631-652) run the batched MI355X grid / a single engine fit.
The plotting helpers of the reference file are out of scope.
"""
from __future__ import annotations

import time

import numpy as np
import pandas as pd

import sglm_
import sglm_cv
import sglm_pp
from sglm_hip import folds as _folds


def timeshift_cols_by_signal_length(X, cols_to_shift, neg_order=0, pos_order=1, trial_id='nTrial',
                                    dummy_col='nothing', shift_amt_ratio=2.0):
    """backend/sglm_ez.py:14-74."""
    X = X.copy()
    if dummy_col not in X.columns:
        X[dummy_col] = 1
        created = True
    else:
        created = False
    min_num_ts, sft_orders = {}, {}
    for col in cols_to_shift:
        min_num_ts[col] = X.query(f'{col} > 0').groupby([trial_id, col])[dummy_col].count().min()
        col_nums = sglm_pp.get_column_nums(X, [col])
        shift_amt = max(min_num_ts[col] // shift_amt_ratio, 1)
        print(f'mnts: {min_num_ts[col]}, sar: {shift_amt_ratio}')
        neg_order_lst = list(np.arange(neg_order, 0, shift_amt))
        pos_order_lst = list(np.arange(shift_amt, pos_order + 1, shift_amt))
        sft_orders[col] = (neg_order_lst, pos_order_lst)
        X = sglm_pp.timeshift_multiple(X, shift_inx=col_nums,
                                       shift_amt_list=[0] + neg_order_lst + pos_order_lst)
    if created:
        X = X.drop(dummy_col, axis=1)
    return X, sft_orders


def add_timeshifts_by_sl_to_col_list(all_cols, shifted_cols, sft_orders):
    out_col_list = []
    for col in shifted_cols:
        out_col_list.extend([col + f'_{_}' for _ in sft_orders[col][0] + sft_orders[col][1]])
    return all_cols + out_col_list


def timeshift_cols(X, cols_to_shift, neg_order=0, pos_order=1):
    """backend/sglm_ez.py:102-123 — shifts [0] + neg..-1 + 1..pos in one kernel launch."""
    col_nums = sglm_pp.get_column_nums(X, cols_to_shift)
    return sglm_pp.timeshift_multiple(X, shift_inx=col_nums,
                                      shift_amt_list=[0] + list(range(neg_order, 0)) +
                                      list(range(1, pos_order + 1)))


def add_timeshifts_to_col_list(all_cols, shifted_cols, neg_order=0, pos_order=1):
    """backend/sglm_ez.py:126-147."""
    out_col_list = []
    for shift_amt in list(range(neg_order, 0)) + list(range(1, pos_order + 1)):
        out_col_list.extend([_ + f'_{shift_amt}' for _ in shifted_cols])
    return all_cols + out_col_list


def fit_GLM(X, y, model_name='Gaussian', *args, **kwargs):
    """backend/sglm_ez.py:149-171."""
    glm = sglm_.GLM(model_name, *args, **kwargs)
    glm.fit(X.values, y.values)
    return glm


def diff_cols(X, cols, append_to_base=True):
    col_nums = sglm_pp.get_column_nums(X, cols)
    return sglm_pp.diff(X, col_nums, append_to_base=append_to_base)


def cv_idx_by_timeframe(X, y=None, timesteps_per_bucket=20, num_folds=10, test_size=None):
    """backend/sglm_ez.py:193-216."""
    bucket_ids = sglm_pp.bucket_ids_by_timeframe(X.shape[0], timesteps_per_bucket=timesteps_per_bucket)
    return sglm_pp.cv_idx_from_bucket_ids(bucket_ids, X, y=y, num_folds=num_folds, test_size=test_size)


def holdout_split_by_trial_id(X, y=None, id_cols=['nTrial', 'iBlock'], strat_col=None,
                              strat_mode=None, perc_holdout=0.2):
    """backend/sglm_ez.py:219-308 (same global-RNG consumption; backend samples WITH
    replacement at :304 — kept)."""
    bucket_ids = _folds.trial_keys_codes(X, id_cols)
    num_bucket_ids = int(bucket_ids.max() + 1)
    if strat_col is not None:
        strat_df = X[[strat_col]].copy()
        strat_df['bucket_id'] = bucket_ids
        strat_groups = strat_df[strat_col].unique()
        distinct = [pd.Series(strat_df[strat_df[strat_col] == _]['bucket_id'].unique())
                    for _ in strat_groups]
        sizes = np.array([len(_) for _ in distinct])
        min_bucket_size = sizes.min()
        tr_b, te_b = [], []
        if strat_mode == 'balanced_train':
            k = int(min_bucket_size * (1 - perc_holdout))
            for b in distinct:
                tr_b.append(np.random.choice(b, k, replace=False))
                te_b.append(b[~b.isin(tr_b[-1])])
        elif strat_mode == 'balanced_test':
            k = int(min_bucket_size * perc_holdout)
            for b in distinct:
                te_b.append(np.random.choice(b, k, replace=False))
                tr_b.append(b[~b.isin(te_b[-1])])
        elif strat_mode == 'stratify':
            for b in distinct:
                te_b.append(np.random.choice(b, int(len(b) * perc_holdout), replace=False))
                tr_b.append(b[~b.isin(te_b[-1])])
        else:
            raise ValueError(f'Invalid strat_mode: {strat_mode}')
        test_ids = np.concatenate(te_b)
    else:
        test_ids = np.random.choice(num_bucket_ids, size=int(num_bucket_ids * perc_holdout))
    return bucket_ids.isin(test_ids)


def cv_idx_by_trial_id(X, y=None, trial_id_columns=[], num_folds=5, test_size=None):
    """backend/sglm_ez.py:311-343 — bit-exact with the reference's GroupShuffleSplit."""
    X = pd.DataFrame(X)
    bucket_ids = _folds.trial_keys_codes(X, trial_id_columns)
    return sglm_pp.cv_idx_from_bucket_ids(bucket_ids, X, y=y, num_folds=num_folds,
                                          test_size=test_size)


def simple_cv_fit(X, y, cv_idx, glm_kwarg_lst, model_type='Normal', verbose=0, score_method='mse'):
    """backend/sglm_ez.py:347-389."""
    Xv = X.values if hasattr(X, "values") and not isinstance(X, np.ndarray) else X
    yv = y.values if hasattr(y, "values") and not isinstance(y, np.ndarray) else y
    cv_results = sglm_cv.cv_glm_mult_params(Xv, yv, cv_idx, model_type, glm_kwarg_lst,
                                            verbose=verbose, score_method=score_method)
    return (cv_results['best_score'], cv_results['best_score_std'], cv_results['best_params'],
            cv_results['best_model'], cv_results)


def print_best_model_info(X_setup, best_score, best_params, best_model, start):
    """backend/sglm_ez.py:595-628."""
    print('\n---\n')
    print('Non-Zero Coeffs:')
    for ic, coef in enumerate(best_model.coef_):
        if np.abs(coef) > 1e-10:
            print(f'> {coef}: {X_setup.columns[ic]}')
    print(f'Best Score: {best_score}')
    print(f'Best Params: {best_params}')
    print(f'Best Model: {best_model}')
    print(f'Best Model — Intercept: {best_model.intercept_}')
    print(f'Overall RunTime: {time.time() - start}')
    print()


def training_fit_holdout_score(X_setup, y_setup, X_holdout, y_holdout, best_params):
    """backend/sglm_ez.py:631-652."""
    glm = fit_GLM(X_setup, y_setup, **best_params)
    holdout_score = glm.r2_score(X_holdout, y_holdout)
    holdout_neg_mse_score = glm.neg_mse_score(X_holdout, y_holdout)
    return glm, holdout_score, holdout_neg_mse_score
