"""``sglm.models.split_data`` (sglm/sglm/models/split_data.py): holdout and CV splits with
the PACKAGE key scheme — trial keys ``len:str`` joined by ``'__' + len:str`` for extra id
columns (:36-41, :146-152; the backend joins with ``'_' + str``) — and holdout test groups
drawn WITHOUT replacement (:96; the backend draws with replacement).  Same global-RNG
consumption as the reference, so splits are bit-exact for the same seed."""
import numpy as np
import pandas as pd

from sglm_hip import folds as _folds


def holdout_split_by_trial_id(X, y=None, id_cols=['nTrial_filenum', 'iBlock'], strat_col=None,
                              strat_mode=None, perc_holdout=0.2):
    """split_data.py:5-101 — True where the row belongs to the holdout set."""
    assert len(X) > 0
    bucket_ids = _folds.trial_keys_codes(X, id_cols, package_style=True)
    num_bucket_ids = int(bucket_ids.max() + 1)
    if strat_col is not None:
        strat_df = X[[strat_col]].copy()
        strat_df['bucket_id'] = bucket_ids
        strat_groups = strat_df[strat_col].unique()
        distinct = [pd.Series(strat_df[strat_df[strat_col] == _]['bucket_id'].unique())
                    for _ in strat_groups]
        min_bucket_size = np.array([len(_) for _ in distinct]).min()
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
        test_ids = np.random.choice(num_bucket_ids, size=int(num_bucket_ids * perc_holdout),
                                    replace=False)
    return bucket_ids.isin(test_ids)


def holdout_splits(dfrel_setup, id_cols=['nTrial_filenum'], perc_holdout=0.2):
    """split_data.py:104-121 -> (setup frame, holdout frame, holdout mask)."""
    holdout = holdout_split_by_trial_id(dfrel_setup, id_cols=id_cols, perc_holdout=perc_holdout)
    return dfrel_setup.loc[~holdout], dfrel_setup.loc[holdout], holdout


def cv_idx_by_trial_id(X, y=None, trial_id_columns=[], num_folds=5, test_size=None):
    """split_data.py:124-157 (package key scheme)."""
    from sglm_hip.lagframe import LagFrame
    if not isinstance(X, LagFrame):
        X = pd.DataFrame(X)
    bucket_ids = _folds.trial_keys_codes(X, trial_id_columns, package_style=True)
    return cv_idx_from_bucket_ids(bucket_ids, X, y=y, num_folds=num_folds, test_size=test_size)


def cv_idx_from_bucket_ids(bucket_ids, X, y=None, num_folds=None, test_size=None):
    """split_data.py:160-188: GroupShuffleSplit on the bucket ids (LOO-sized default)."""
    return _folds.cv_idx_from_bucket_ids(bucket_ids, X, y=y, num_folds=num_folds,
                                         test_size=test_size)
