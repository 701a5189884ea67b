"""CPU restatement of the reference's CV fold generation — TEST INFRASTRUCTURE.

* ``bucket_ids_by_timeframe``  — backend/sglm_pp.py:218-234 (``arange(N) // (N // tpb)``).
* ``trial_bucket_codes``       — backend/sglm_ez.py:334-340 (key ``len(str(v)) + ':' + str(v)``,
                                  extra id columns joined with ``'_' + str(v)``), package twin
                                  sglm/sglm/models/split_data.py:146-152 (``'__' + len:str``),
                                  then pandas categorical codes (lexicographic key order).
* ``group_shuffle_split``      — backend/sglm_pp.py:236-264 -> sklearn ``GroupShuffleSplit``
                                  (sklearn/model_selection/_split.py:1925-1945, 2181-2187,
                                  2433-2505): ``np.unique`` inverse, per split
                                  ``rng.permutation(G)``; test = perm[:ceil(t G)],
                                  train = perm[n_test:]; rows = flatnonzero(isin(...)).
                                  ``random_state=None`` -> the global ``np.random`` state.

Pure numpy; pinned against sklearn's own GroupShuffleSplit in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import math

import numpy as np


def bucket_ids_by_timeframe(total_timesteps, timesteps_per_bucket=20):
    num_buckets = total_timesteps // timesteps_per_bucket
    return np.arange(total_timesteps) // num_buckets


def trial_bucket_codes(columns, package_style=False):
    """Group codes for ``cv_idx_by_trial_id`` given a list of 1-D id columns."""
    keys = None
    for i, col in enumerate(columns):
        s = [str(v) for v in col]
        if i == 0:
            keys = [f"{len(v)}:{v}" for v in s]
        elif package_style:
            keys = [k + "__" + f"{len(v)}:{v}" for k, v in zip(keys, s)]
        else:
            keys = [k + "_" + v for k, v in zip(keys, s)]
    uniq = sorted(set(keys))
    lookup = {k: i for i, k in enumerate(uniq)}
    return np.array([lookup[k] for k in keys], dtype=np.int64)


def _n_train_test(n_samples, test_size):
    if np.asarray(test_size).dtype.kind == "f":
        n_test = math.ceil(test_size * n_samples)
    else:
        n_test = int(test_size)
    return n_samples - n_test, n_test


def group_shuffle_split(groups, n_splits, test_size, rng=None):
    rng = np.random.mtrand._rand if rng is None else rng
    classes, gidx = np.unique(np.asarray(groups), return_inverse=True)
    n_train, n_test = _n_train_test(len(classes), test_size)
    out = []
    for _ in range(n_splits):
        perm = rng.permutation(len(classes))
        ind_test = perm[:n_test]
        ind_train = perm[n_test:n_test + n_train]
        out.append((np.flatnonzero(np.isin(gidx, ind_train)),
                    np.flatnonzero(np.isin(gidx, ind_test))))
    return out


def cv_idx_from_bucket_ids(bucket_ids, num_folds=None, test_size=None):
    bucket_ids = np.asarray(bucket_ids)
    if num_folds is None:
        num_folds = bucket_ids.max() + 1
    if test_size is None:
        test_size = 1 / num_folds
    return group_shuffle_split(bucket_ids, num_folds, test_size)
