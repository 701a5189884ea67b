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
from sglm_hip.estimators import host_matrix as _host_matrix
from sglm_hip.lagframe import LagFrame


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
    """backend/sglm_ez.py:102-123 — shifts [0] + neg..-1 + 1..pos.  A DataFrame comes back as
    a device-resident lagged frame (sglm_hip.lagframe.LagFrame, see sglm_pp.timeshift_multiple)."""
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
    glm.fit(X if isinstance(X, LagFrame) else _host_matrix(X), y.values)
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
    if not isinstance(X, LagFrame):
        X = pd.DataFrame(X)
    runs = _folds.trial_key_runs(X, trial_id_columns)
    if runs is not None and (y is None or len(y) == len(X)):
        # a sorted trial column: the same codes per run, the row lists written run by run
        if num_folds is None:
            num_folds = int(runs[0].max()) + 1
        return _folds.cv_idx_from_runs(*runs, num_folds, test_size)
    bucket_ids = _folds.trial_keys_codes(X, trial_id_columns)
    return sglm_pp.cv_idx_from_bucket_ids(bucket_ids, X, y=y, num_folds=num_folds,
                                          test_size=test_size)


def simple_cv_fit(X, y, cv_idx, glm_kwarg_lst, model_type='Normal', verbose=0, score_method='mse'):
    """backend/sglm_ez.py:347-389."""
    Xv = X if isinstance(X, LagFrame) else _host_matrix(X)
    yv = y.values if hasattr(y, "values") and not isinstance(y, np.ndarray) else y
    if getattr(yv, "dtype", None) is not None and not isinstance(yv.dtype, np.dtype):
        yv = np.asarray(pd.Series(yv).to_numpy(dtype=np.float64, na_value=np.nan))
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


def holdout_resplit_cv(X, y, id_df, glm_kwarg_lst, num_runs=3, id_cols=('nTrial',),
                       perc_holdout=0.2, num_folds=5, test_size=None, score_method='mse',
                       package_style=False):
    """Repeated holdout resplits batched on the resident design.

    The production notebooks loop ``for irun in range(num_runs)``: holdout split by trial id,
    folds on the setup rows, ``simple_cv_fit`` over the parameter list, then
    ``training_fit_holdout_score`` (02-create_features-p50-Lass-Rid-rerun-smpl.ipynb cell 12).
    Here the splits are drawn in that loop's RNG order (holdout, then folds, per run) and ALL
    runs' fold fits, setup refits and holdout scores are one batched MI355X solve.

    ``id_df`` holds the id columns aligned with the rows of X; ``package_style`` selects the
    package split functions (sglm.models.split_data: ``'__'`` keys, holdout without
    replacement) instead of the backend ones.  ``model_name`` is popped once from the kwargs
    and used for every run (a sequential loop over the same dicts would fall back to
    'Gaussian' after the first run, sglm_cv.py:288).  Returns, per run, a dict with
    ``holdout`` (bool array), ``cv_idx`` (setup-relative, as the loop sees them),
    ``best_score``, ``best_score_std``, ``best_params``, ``best_model``, ``full_cv_results``
    and the best refit's ``holdout_score`` (R^2 / D^2) and ``holdout_neg_mse_score``."""
    from sglm_hip import grid as _grid
    if package_style:
        from sglm.models import split_data as _sd
        hsplit, cvsplit = _sd.holdout_split_by_trial_id, _sd.cv_idx_by_trial_id
    else:
        hsplit, cvsplit = holdout_split_by_trial_id, cv_idx_by_trial_id
    id_df = pd.DataFrame(id_df).reset_index(drop=True)
    id_cols = list(id_cols)
    runs = []
    for _ in range(num_runs):
        hold = np.asarray(hsplit(id_df, id_cols=id_cols, perc_holdout=perc_holdout))
        setup = np.flatnonzero(~hold)
        cv_idx = cvsplit(id_df.iloc[setup].reset_index(drop=True),
                         trial_id_columns=id_cols, num_folds=num_folds, test_size=test_size)
        runs.append((hold, setup, cv_idx))
    params = []
    for glm_kwargs in glm_kwarg_lst:
        glm_kwargs = dict(glm_kwargs)
        mn = glm_kwargs.pop('model_name', 'Gaussian')
        roll = glm_kwargs.pop('roll', 0)
        params.append((mn, glm_kwargs, roll))
    objectives = [sglm_.GLM(mn, **kw).model.objective() for mn, kw, _ in params]
    rolls = [r for _, _, r in params]
    groups = [{"cv_idx": [(setup[tr], setup[te]) for tr, te in cv_idx],
               "objectives": objectives, "rolls": rolls, "refit_rows": setup,
               "holdout_rows": np.flatnonzero(hold)} for hold, setup, cv_idx in runs]
    Xv = X.design() if isinstance(X, LagFrame) else _host_matrix(X)
    yv = np.asarray(y.values if hasattr(y, "values") else y, dtype=np.float64).reshape(-1)
    res = _grid.run_multi(Xv, yv, groups, score_method=score_method)
    out = []
    for (hold, setup, cv_idx), rg in zip(runs, res):
        full = []
        for (mn, kw, roll), r in zip(params, rg):
            glm = sglm_.GLM(mn, **kw)
            glm._set_fitted(r["refit_coef"], r["refit_intercept"], max(r["n_iter"]))
            d = {k: r[k] for k in ("cv_coefs", "cv_intercepts", "cv_scores_train",
                                   "cv_scores_test", "cv_mean_score_train", "cv_mean_score",
                                   "cv_std_score", "cv_R2_score", "cv_mse_score")}
            d.update(glm_kwargs=kw, model=glm, holdout_score=r["refit_holdout_r2"],
                     holdout_neg_mse_score=r["refit_holdout_neg_mse"])
            full.append(d)
        key = 'cv_R2_score' if score_method == 'r2' else 'cv_mean_score'
        best = None
        for i, d in enumerate(full):                 # first strict max (sglm_cv.py:402-415)
            if best is None or d[key] > full[best][key]:
                best = i
        b = full[best]
        out.append({"holdout": hold, "cv_idx": cv_idx, "best_score": b[key],
                    "best_score_std": b["cv_std_score"], "best_params": b["glm_kwargs"],
                    "best_model": b["model"], "full_cv_results": full,
                    "holdout_score": b["holdout_score"],
                    "holdout_neg_mse_score": b["holdout_neg_mse_score"]})
    return out
