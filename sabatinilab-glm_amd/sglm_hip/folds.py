"""CV fold generation (host numpy; integer work, bit-exact with the reference).

The reference draws its folds with sklearn ``GroupShuffleSplit`` on the GLOBAL numpy RNG
(backend/sglm_pp.py:236-264; sklearn/model_selection/_split.py:1925-1945, 2181-2187,
2433-2505).  This module restates that algorithm without sklearn so fold indices stay
bit-exact while the rest of the grid runs on the GPU:

    classes, gidx = unique(groups, return_inverse)
    n_test = ceil(test_size * G)  (float test_size) | int(test_size);  n_train = G - n_test
    per split: perm = rng.permutation(G); test = perm[:n_test]; train = perm[n_test:]
    rows = flatnonzero(isin(gidx, train/test))   (ascending)

Fold masks for the engine are multiplicity vectors (uint8), so user-supplied index lists
with repeats keep the weight that ``X[idx]`` copies would give them.
"""
from __future__ import annotations

import math

import numpy as np


def bucket_ids_by_timeframe(total_timesteps, timesteps_per_bucket=20):
    """backend/sglm_pp.py:218-234 (kept verbatim in behaviour, incl. the N//tpb divisor)."""
    num_buckets = total_timesteps // timesteps_per_bucket
    return np.arange(total_timesteps) // num_buckets


def _validate(n_samples, test_size):
    kind = np.asarray(test_size).dtype.kind
    if (kind == "i" and (test_size >= n_samples or test_size <= 0)) or \
            (kind == "f" and (test_size <= 0 or test_size >= 1)):
        raise ValueError(f"test_size={test_size} should be either positive and smaller than the "
                         f"number of samples {n_samples} or a float in the (0, 1) range")
    n_test = math.ceil(test_size * n_samples) if kind == "f" else int(test_size)
    n_train = n_samples - n_test
    if n_train <= 0:
        raise ValueError(f"With n_samples={n_samples}, test_size={test_size} and train_size=None, "
                         "the resulting train set will be empty. Adjust any of the "
                         "aforementioned parameters.")
    return n_train, n_test


def group_shuffle_split(groups, n_splits, test_size, random_state=None):
    if random_state is None:
        rng = np.random.mtrand._rand
    elif isinstance(random_state, np.random.RandomState):
        rng = random_state
    else:
        rng = np.random.RandomState(random_state)
    groups = np.asarray(groups)
    lo = int(groups.min()) if groups.size and groups.dtype.kind in "iu" else 0
    cnt = None
    if groups.size and groups.dtype.kind in "iu" and int(groups.max()) - lo < 4 * groups.size:
        # small-range integer ids (categorical codes): the same classes / inverse by counting
        g0 = groups.astype(np.int64)
        if lo:
            g0 -= lo
        cnt = np.bincount(g0)
        present = cnt > 0
        if present.all():                     # dense codes 0 .. G-1: the inverse is the code
            classes, gidx = np.arange(cnt.size) + lo, g0
        else:
            classes = np.flatnonzero(present) + lo
            gidx = (np.cumsum(present) - 1)[g0]
            cnt = cnt[present]
    else:
        classes, gidx = np.unique(groups, return_inverse=True)
    n_train, n_test = _validate(len(classes), test_size)
    G = len(classes)
    # the permutations in order (the RNG stream), then the row lists
    S = int(n_splits)
    side = np.zeros((max(S, 1), G), dtype=np.uint8)
    for k in range(S):
        perm = rng.permutation(G)
        side[k, perm[n_test:n_test + n_train]] = 1
        side[k, perm[:n_test]] = 2
    return _group_rows(np.ascontiguousarray(gidx, dtype=np.int64), side[:S], G, cnt)


def _group_rows(gidx, side, G, cnt=None):
    """Per split, (flatnonzero(side[gidx] == 1), flatnonzero(side[gidx] == 2)): the train / test
    row lists, built by the library's host code (sglm_host_group_rows, one thread per list)."""
    import ctypes
    from . import _lib
    from .engine import HOST_THREADS
    S, n = side.shape[0], gidx.size
    if S == 0:
        return []
    if cnt is None:
        cnt = np.bincount(gidx, minlength=G)[:G]
    lens = np.array([int(cnt[side[k] == v].sum()) for k in range(S) for v in (1, 2)],
                    dtype=np.int64)
    outs = [np.empty(int(L), dtype=np.int64) for L in lens]
    ptrs = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    side = np.ascontiguousarray(side)
    _lib.call("sglm_host_group_rows", gidx.ctypes.data, n, side.ctypes.data, S, G,
              ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, HOST_THREADS)
    return [(outs[2 * k], outs[2 * k + 1]) for k in range(S)]


def cv_idx_from_bucket_ids(bucket_ids, X=None, y=None, num_folds=None, test_size=None):
    """backend/sglm_pp.py:236-264 (X, y only validated for length by sklearn; unused)."""
    bucket_ids = np.asarray(bucket_ids)
    if num_folds is None:
        num_folds = bucket_ids.max() + 1
    if test_size is None:
        test_size = 1 / num_folds
    if X is not None and len(X) != len(bucket_ids):
        raise ValueError(f"Found input variables with inconsistent numbers of samples: "
                         f"[{len(X)}, {len(bucket_ids)}]")
    return group_shuffle_split(bucket_ids, num_folds, test_size)


def trial_key_runs(df, id_cols, package_style=False):
    """(code per run, run starts, run lengths) of the trial-key codes of ``trial_keys_codes``
    when the key is ONE numeric id column whose values never decrease (trial counters: each
    distinct value is one run of rows), else None.  The codes are the same ranks of the same
    key strings, kept per run instead of expanded per row."""
    if len(id_cols) != 1:
        return None
    c = df[id_cols[0]]
    if not (isinstance(c.dtype, np.dtype) and c.dtype.kind in "biuf"):
        return None
    v = c.to_numpy()
    if v.size < 2 or not bool(np.all(v[1:] >= v[:-1])):
        return None
    chg = np.empty(v.size, dtype=bool)
    chg[0] = True
    np.not_equal(v[1:], v[:-1], out=chg[1:])
    at = np.flatnonzero(chg)
    u = v[at]
    lens = np.diff(at, append=v.size).astype(np.int64)
    if c.dtype in (np.float64, np.int64) and u.size and u[0] >= 0 and \
            u[-1] < (1e7 if c.dtype == np.float64 else 1e9) and bool(np.all(u == np.floor(u))):
        # non-negative integral ids whose strings ("12" / "12.0") have at most 9 characters:
        # the key "<len>:<str>" orders by length (one digit), then lexicographically, i.e.
        # numerically -- the runs (increasing) are already in key order
        return np.arange(u.size, dtype=np.int64), at.astype(np.int64), lens
    if c.dtype in (np.float64, np.int64):
        strs = [str(x) for x in u.tolist()]
    else:
        su = pd_series(u, c.dtype)
        strs = list(su.apply(str) if package_style else su.astype(str))
    keys = [f"{len(sv)}:{sv}" for sv in strs]
    if len(set(keys)) != len(keys):
        return None
    order = np.argsort(np.asarray(keys, dtype=object), kind="stable")
    rank = np.empty(len(keys), dtype=np.int64)
    rank[order] = np.arange(len(keys))
    return rank, at.astype(np.int64), lens


def pd_series(values, dtype):
    import pandas as pd
    return pd.Series(values, dtype=dtype)


def cv_idx_from_runs(rank, starts, lens, num_folds, test_size=None, random_state=None):
    """cv_idx_from_bucket_ids for groups given as runs (trial_key_runs): the same
    GroupShuffleSplit permutations of the dense codes 0 .. G-1 (every run is its own group), the
    row lists written run by run by native threads (sglm_host_group_runs)."""
    import ctypes
    from . import _lib
    from .engine import HOST_THREADS
    if random_state is None:
        rng = np.random.mtrand._rand
    elif isinstance(random_state, np.random.RandomState):
        rng = random_state
    else:
        rng = np.random.RandomState(random_state)
    G = int(rank.size)
    if test_size is None:
        test_size = 1 / num_folds
    n_train, n_test = _validate(G, test_size)
    S = int(num_folds)
    side = np.zeros((max(S, 1), G), dtype=np.uint8)
    for k in range(S):
        perm = rng.permutation(G)
        side[k, perm[n_test:n_test + n_train]] = 1
        side[k, perm[:n_test]] = 2
    side = np.ascontiguousarray(side[:S])
    if S == 0:
        return []
    sr = side[:, rank]                                   # [S][runs]: the side of each run
    lens_l = np.stack([(lens[None, :] * (sr == 1)).sum(1), (lens[None, :] * (sr == 2)).sum(1)],
                      1).reshape(-1).astype(np.int64)
    outs = [np.empty(int(L), dtype=np.int64) for L in lens_l]
    ptrs = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    rank = np.ascontiguousarray(rank, dtype=np.int64)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    _lib.call("sglm_host_group_runs", starts.ctypes.data, lens.ctypes.data, rank.ctypes.data,
              int(rank.size), side.ctypes.data, S, G, ctypes.cast(ptrs, ctypes.c_void_p),
              lens_l.ctypes.data, HOST_THREADS)
    return [(outs[2 * k], outs[2 * k + 1]) for k in range(S)]


def trial_keys_codes(df, id_cols, package_style=False):
    """Categorical codes of the trial keys (backend/sglm_ez.py:334-340; package
    sglm/sglm/models/split_data.py:146-152 when ``package_style``).

    The keys are built as the reference builds them -- per id column the string of the value
    (``astype(str)`` / ``apply(str)``), prefixed with its length, joined with ``'_'`` (backend)
    or ``'__'`` (package) -- but only for the distinct id tuples: the codes are the ranks of
    those keys in lexicographic order (pandas' category order) taken back to the rows.  Numeric
    id columns only; anything else takes the row-wise string path."""
    import pandas as pd
    cols = [df[c] for c in id_cols]
    if cols and all(isinstance(c.dtype, np.dtype) and c.dtype.kind in "biuf" for c in cols):
        invs, strs = [], []
        runs = None
        for c in cols:
            v = c.to_numpy()
            if v.size > 1 and bool(np.all(v[1:] >= v[:-1])):
                # non-decreasing ids (trial counters): distinct values at the change points,
                # the inverse as run lengths (expanded only for a multi-column key)
                chg = np.empty(v.size, dtype=bool)
                chg[0] = True
                np.not_equal(v[1:], v[:-1], out=chg[1:])
                at = np.flatnonzero(chg)
                u = v[at]
                runs = np.diff(at, append=v.size)
                inv = runs if len(cols) == 1 else np.repeat(np.arange(at.size), runs)
            else:
                runs = None
                inv, u = pd.factorize(v, use_na_sentinel=False)          # hash, O(n)
            if c.dtype in (np.float64, np.int64):
                # Python's str of the float64 / int64 values: what Series.astype(str) and
                # .apply(str) print for these dtypes, a quarter of their time
                strs.append(np.array([str(x) for x in u.tolist()], dtype=object))
            else:
                su = pd.Series(u, dtype=c.dtype)
                strs.append(np.asarray((su.apply(str) if package_style else su.astype(str)),
                                       dtype=object))
            invs.append(inv if runs is not None else inv.astype(np.int64))
        if len(invs) == 1:
            tup, row_of = np.arange(strs[0].size)[:, None], invs[0]
        else:
            comb = invs[0]
            for inv, st in zip(invs[1:], strs[1:]):
                comb = comb * st.size + inv
            row_of, cu = pd.factorize(comb)
            tup = np.empty((cu.size, len(invs)), dtype=np.int64)
            rem = cu.astype(np.int64)
            for i in range(len(invs) - 1, -1, -1):
                tup[:, i] = rem % strs[i].size
                rem //= strs[i].size
        first = strs[0][tup[:, 0]]
        keys = [f"{len(sv)}:{sv}" for sv in first]
        for i in range(1, len(strs)):
            nxt = strs[i][tup[:, i]]
            keys = ([f"{k}__{len(sv)}:{sv}" for k, sv in zip(keys, nxt)] if package_style
                    else [f"{k}_{sv}" for k, sv in zip(keys, nxt)])
        keys = np.asarray(keys, dtype=object)
        order = np.argsort(keys, kind="stable")          # Python string order, as pandas
        rank = np.empty(keys.size, dtype=np.int64)
        rank[order] = np.arange(keys.size)
        # distinct tuples can share a key only if two values print alike: keep pandas' codes
        if len(set(keys.tolist())) == keys.size:
            dt = np.int8 if keys.size < 128 else (np.int16 if keys.size < 32768 else np.int32)
            if len(invs) == 1 and runs is not None:
                return pd.Series(np.repeat(rank.astype(dt), runs), index=df.index)
            return pd.Series(rank[row_of].astype(dt), index=df.index)
    bucket = None
    for i, idc in enumerate(id_cols):
        s = df[idc].astype(str) if not package_style else df[idc].apply(str)
        if i == 0:
            bucket = s.str.len().astype(str) + ":" + s
        elif package_style:
            bucket = bucket + "__" + s.str.len().apply(str) + ":" + s
        else:
            bucket = bucket + "_" + s
    return bucket.astype("category").cat.codes


def wrap_indices(idx, n):
    """int64 row indices with negative entries in [-n, 0) wrapped by + n, as the reference's
    numpy fancy indexing ``X[idx_train]`` (backend/sglm_cv.py:107-110) treats them; anything
    outside [-n, n) raises IndexError like numpy does."""
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    if idx.size and (idx.min() < -n or idx.max() >= n):
        bad = idx[(idx < -n) | (idx >= n)][0]
        raise IndexError(f"index {bad} is out of bounds for axis 0 with size {n}")
    return np.where(idx < 0, idx + n, idx)


def mask_from_idx(idx, n):
    """Multiplicity mask (uint8, length n) of one index list: 0/1 for strictly increasing
    indices, counts for repeats (holdout resampling)."""
    idx = wrap_indices(idx, n)
    if idx.size and (idx[0] < 0 or idx[-1] >= n or not np.all(idx[1:] > idx[:-1])):
        m = np.bincount(idx, minlength=n)[:n]              # repeats (holdout resampling)
        if m.max(initial=0) > 255:
            raise ValueError("an index repeats more than 255 times in one split")
        return m.astype(np.uint8)
    m = np.zeros(n, dtype=np.uint8)                         # strictly increasing: 0/1 mask
    m[idx] = 1
    return m


def masks_from_cv_idx(cv_idx, n):
    """Per split: (train multiplicity mask, test multiplicity mask) as uint8 arrays."""
    return [(mask_from_idx(tr, n), mask_from_idx(te, n)) for tr, te in cv_idx]
