"""Host logic and the C ABI without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def test_library_exports_every_header_symbol():
    from sglm_hip import _lib
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "sglm_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = re.findall(r"\b(sglm_[a-z0-9_]+)\s*\(", hdr)
    assert len(names) >= 15
    for name in names:
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, name
    assert lib.sglm_version() >= 1
    assert lib.sglm_xtr_work_bytes(2048, 120, 1_000_000) > 0
    assert lib.sglm_syrk_work_bytes(512, 1, 1) == 0


def test_engine_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import sglm
    from sglm_hip import _lib
    glm = sglm.GLM("Poisson", alpha=1.0)          # construction needs no GPU
    with pytest.raises(_lib.HipEngineUnavailable):
        glm.fit(np.ones((10, 2)), np.ones(10))


def test_product_folds_bit_exact_vs_sklearn(golden):
    from sglm_hip import folds
    g = golden("folds.npz")
    trial = np.arange(5000) // 100
    import pandas as pd
    df = pd.DataFrame({"nTrial": trial, "iBlock": trial // 7})
    for seed in (0, 3, 17):
        codes = folds.trial_keys_codes(df, ["nTrial"]).values
        assert np.array_equal(codes, g[f"f{seed}_codes"])
        np.random.seed(seed)
        for k, (tr, te) in enumerate(folds.cv_idx_from_bucket_ids(codes, num_folds=5)):
            assert np.array_equal(tr, g[f"f{seed}_k{k}_train"])
            assert np.array_equal(te, g[f"f{seed}_k{k}_test"])
    assert np.array_equal(folds.trial_keys_codes(df, ["nTrial", "iBlock"]).values,
                          g["codes_two_backend"])
    assert np.array_equal(folds.trial_keys_codes(df, ["nTrial", "iBlock"], package_style=True).values,
                          g["codes_two_package"])
    # the drop-in entry on a sorted trial column takes the run-based path (trial_key_runs ->
    # cv_idx_from_runs, native sglm_host_group_runs): the same sklearn folds
    import sglm_ez
    assert folds.trial_key_runs(df, ["nTrial"]) is not None
    for seed in (0, 3, 17):
        np.random.seed(seed)
        for k, (tr, te) in enumerate(sglm_ez.cv_idx_by_trial_id(df, trial_id_columns=["nTrial"],
                                                                 num_folds=5)):
            assert np.array_equal(tr, g[f"f{seed}_k{k}_train"])
            assert np.array_equal(te, g[f"f{seed}_k{k}_test"])
    np.random.seed(5)
    sp = folds.cv_idx_from_bucket_ids(folds.bucket_ids_by_timeframe(437, 20))
    assert len(sp) == int(g["tf_nsplits"])
    for k, (tr, te) in enumerate(sp):
        assert np.array_equal(tr, g[f"tf_k{k}_train"]) and np.array_equal(te, g[f"tf_k{k}_test"])


def test_sglm_ez_cv_idx_by_trial_id_matches_sklearn():
    """Drop-in sglm_ez.cv_idx_by_trial_id == sklearn GroupShuffleSplit (global RNG)."""
    import pandas as pd
    from sklearn.model_selection import GroupShuffleSplit
    import sglm_ez
    rng = np.random.default_rng(0)
    X = pd.DataFrame({"nTrial": rng.integers(0, 173, 3000), "x": rng.random(3000)})
    np.random.seed(11)
    got = sglm_ez.cv_idx_by_trial_id(X, trial_id_columns=["nTrial"], num_folds=7, test_size=0.3)
    key = X["nTrial"].astype(str).str.len().astype(str) + ":" + X["nTrial"].astype(str)
    np.random.seed(11)
    ref = list(GroupShuffleSplit(n_splits=7, test_size=0.3).split(X, None, key.astype("category").cat.codes))
    for (a, b), (c, d) in zip(got, ref):
        assert np.array_equal(a, c) and np.array_equal(b, d)


def test_masks_from_cv_idx_multiplicity():
    from sglm_hip import folds
    m = folds.masks_from_cv_idx([(np.array([0, 2, 2, 5]), np.array([1]))], 6)
    assert m[0][0].tolist() == [1, 0, 2, 0, 0, 1]
    assert m[0][1].tolist() == [0, 1, 0, 0, 0, 0]


def test_generate_mult_params_and_glm_dispatch():
    import sglm
    import sglm_cv
    from sglm_hip import estimators as est
    out = sglm_cv.generate_mult_params({"alpha": [0, 1], "l1_ratio": [0, 1]}, {"max_iter": 5})
    assert out[0] == {"max_iter": 5, "alpha": 0, "l1_ratio": 0}
    assert isinstance(sglm.GLM("Normal", alpha=0).model, est.LinearRegression)
    assert isinstance(sglm.GLM("Normal", alpha=1, l1_ratio=0).model, est.Ridge)
    assert isinstance(sglm.GLM("Normal", alpha=1, l1_ratio=1).model, est.Lasso)
    assert isinstance(sglm.GLM("Normal", alpha=1, l1_ratio=0.3).model, est.ElasticNet)
    m = sglm.GLM("Poisson", alpha=2.0).model
    assert isinstance(m, est.TweedieRegressor) and m.power == 1 and m.alpha == 2.0
    with pytest.raises(TypeError):
        sglm.GLM("Normal", alpha=0, reg_lambda=0)      # like sklearn (test_sglm.py:42)
    with pytest.raises(TypeError):
        sglm.GLM("Poisson", reg_lambda=0)
    o = sglm.GLM("Poisson", alpha=0.5).model.objective()
    assert o.lam(1000) == 500.0                          # mean-scaled objective
    assert sglm.GLM("Normal", alpha=3.0, l1_ratio=0).model.objective().lam(1000) == 3.0
    with pytest.raises(sglm.NotYetImplementedError):
        sglm.GLM("Logistic")


def test_timeshift_fill_bits():
    from sglm_hip.timeshift import fill_bits
    assert fill_bits(np.nan, np.float64) == int(np.array(np.nan).view(np.uint64))
    assert fill_bits(0, np.int16) == 0
    assert fill_bits(-1, np.int32) == 0xFFFFFFFF


def test_native_host_masks_vs_python():
    """sglm_host_masks (host code of the library, no GPU) against the Python mask builders:
    strictly increasing fold lists, fold lists with repeats (multiplicities), row lists with
    duplicates, every-row masks; nnz / sums; the error cases."""
    from sglm_hip import engine as E, folds, grid
    rng = np.random.default_rng(0)
    n, ld = 10_007, 10_048
    inc = np.sort(rng.choice(n, 6000, replace=False))
    rep = rng.integers(0, n, 9000)
    rows = rng.integers(0, n, 3000)
    specs = [(inc, True), (rep, True), (rows, False), (None, False), (inc[:0], True),
             (list(inc[:10]), False)]
    nnz, sums, M = E.host_masks(specs, n, ld)
    for f, (idx, mult) in enumerate(specs):
        want = grid._mask_array(idx, mult, n)
        np.testing.assert_array_equal(M[f, :n], want)
        assert not M[f, n:].any()
        assert nnz[f] == np.count_nonzero(want)
        assert sums[f] == want.sum(dtype=np.int64)
        assert sums[f] == grid._mask_count(idx, mult, n)
    np.testing.assert_array_equal(M[1, :n], folds.mask_from_idx(rep, n))
    with pytest.raises(ValueError, match="255"):
        E.host_masks([(np.zeros(256, np.int64), True)], n, ld)
    with pytest.raises(ValueError, match="outside"):
        E.host_masks([(np.array([3, n]), True)], n, ld)
    with pytest.raises(ValueError, match="outside"):
        E.host_masks([(np.array([-n - 1, 3]), False)], n, ld)


@pytest.mark.parametrize("layout", ["block", "columns", "block_subset"])
def test_host_pack_bits_cols(layout):
    """sglm_host_pack_bits_cols (host code, no GPU; the 0/1 event columns of a lagged frame
    cross PCIe as bit-planes): the row-major block path (a DataFrame of a C-order array) and the
    per-column path give np.packbits of (v == 1.0), and the 0/1 flag is cleared by NaN, 0.5
    and 2.0 but not by -0.0; row counts not a multiple of 32 or of the 2048-row chunks."""
    import pandas as pd
    from sglm_hip import _lib
    rng = np.random.default_rng(5)
    N, m = 70_001, 11
    E = (rng.random((N, m)) < 0.3).astype(np.float64)
    E[17, 2] = np.nan
    E[N - 1, 4] = 0.5
    E[4099, 6] = 2.0
    E[123, 8] = -0.0
    if layout == "columns":
        df = pd.DataFrame({f"e{a}": E[:, a].copy() for a in range(m)})
    else:
        df = pd.DataFrame(E, columns=[f"e{a}" for a in range(m)])
    cols = list(df.columns) if layout != "block_subset" else ["e3", "e5", "e4"]
    arrs = [df[c].to_numpy() for c in cols]
    k = len(arrs)
    nw = (N + 31) // 32
    bits = np.zeros(k * nw, np.uint32)
    binary = np.zeros(k, np.uint8)
    ones = np.zeros(k, np.int64)
    ptrs = (ctypes.c_void_p * k)(*[a.ctypes.data for a in arrs])
    strides = np.array([a.strides[0] // 8 for a in arrs], dtype=np.int64)
    _lib.call("sglm_host_pack_bits_cols", ctypes.cast(ptrs, ctypes.c_void_p),
              strides.ctypes.data, k, N, bits.ctypes.data, binary.ctypes.data,
              ones.ctypes.data, 4)
    V = np.stack(arrs)
    ref = np.packbits(V == 1.0, axis=1, bitorder="little")
    ref = np.ascontiguousarray(np.pad(ref, ((0, 0), (0, 4 * nw - ref.shape[1])))).view(np.uint32)
    np.testing.assert_array_equal(bits.reshape(k, nw), ref)
    want = [bool(np.all((v == 0.0) | (v == 1.0))) for v in V]
    np.testing.assert_array_equal(binary.astype(bool), want)
    np.testing.assert_array_equal(ones, (V == 1.0).sum(axis=1))


def test_negative_fold_indices_wrap_like_numpy():
    """X[idx_train] (backend/sglm_cv.py:107-110) wraps indices in [-n, 0); the native mask
    builder, the Python mask builders and the row counts do the same."""
    from sglm_hip import engine as E, folds, grid
    rng = np.random.default_rng(1)
    n, ld = 5_003, 5_120
    pos = np.sort(rng.choice(n, 2000, replace=False))
    neg = pos - n                                            # the same rows, negative
    mixed = np.where(rng.random(pos.size) < 0.5, pos, neg)   # unsorted once wrapped
    rep = rng.integers(-n, n, 4000)
    specs = [(neg, True), (mixed, True), (rep, True), (mixed, False)]
    nnz, sums, M = E.host_masks(specs, n, ld)
    want_rows = np.zeros(n, np.uint8)
    want_rows[pos] = 1
    for f, (idx, mult) in enumerate(specs):
        want = np.zeros(n, np.int64)
        np.add.at(want, np.asarray(idx) % n, 1)
        if not mult:
            want = (want > 0).astype(np.int64)
        np.testing.assert_array_equal(M[f, :n], want)
        np.testing.assert_array_equal(grid._mask_array(idx, mult, n), want)
        assert sums[f] == want.sum() == grid._mask_count(idx, mult, n)
        assert nnz[f] == np.count_nonzero(want)
    np.testing.assert_array_equal(M[0, :n], want_rows)
    np.testing.assert_array_equal(folds.mask_from_idx(neg, n), want_rows)
    with pytest.raises(IndexError):
        folds.wrap_indices([0, -n - 1], n)


def test_hessian_copies_resolve_to_formed_hessians():
    """engine._resolve_copies: an exact duplicate of a representative that is itself
    shared along its lambda chain reads the chain representative's Hessian, with the chain
    distance as its drift; order of the copy list does not matter."""
    from sglm_hip import engine as E
    # fit 3 duplicates 1 (same start); 1 is shared from 0 along the chain (dist .2); 5 from 1?
    src = {3: (1, 0.0), 1: (0, 0.2), 4: (2, 0.0), 6: (4, 0.0)}
    got = {k: (r, d) for k, r, d in E._resolve_copies(src, [0, 2, 7])}
    assert got == {3: (0, 0.2), 1: (0, 0.2), 4: (2, 0.0), 6: (2, 0.0)}
    with pytest.raises(RuntimeError):
        E._resolve_copies({1: (5, 0.0)}, [0])
    # uniq shares then fails back: a fit that is both formed and listed is its own source
    assert E._resolve_copies({}, [0, 1]) == []
    # the chain sharing of hess_finish: a chain 0 <- 1 <- 2 (greedy, summed distance)
    keep, shared = E._share_chains(np.array([0, 1, 2], np.int32), [[0, 1, 2]],
                                   np.array([0.1, 0.1]), 0.375)
    assert keep.tolist() == [0] and [(k, r) for k, r, _ in shared] == [(1, 0), (2, 0)]
    assert abs(shared[1][2] - 0.2) < 1e-12


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 100_000, 1_000_000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_row_slabs_cover_the_rows(n, world):
    """Row-sharded grids (sglm_hip/comm.py): the slabs of all ranks tile [0, n) in order,
    inner boundaries on 64-row blocks, sizes within one block of n / world."""
    from sglm_hip.comm import row_slab
    if n < world:
        with pytest.raises(ValueError):
            row_slab(n, 0, world)
        return
    sl = [row_slab(n, r, world) for r in range(world)]
    assert sl[0][0] == 0 and sl[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
    assert all(e > s for s, e in sl)
    if n >= 64 * world:
        assert all(b[0] % 64 == 0 for b in sl[1:])
    if n >= 64 * world:
        assert all(abs((e - s) - n / world) <= 64 for s, e in sl)


def test_group_rows_native_vs_numpy():
    """folds._group_rows (sglm_host_group_rows, host code) = flatnonzero(side[gidx] == 1 / 2)
    per split, for unsorted group indices and groups on neither side; a bad group index and a
    wrong list length are errors."""
    from sglm_hip import _lib, folds
    rng = np.random.default_rng(2)
    G, n = 997, 200_003
    gidx = rng.integers(0, G, n).astype(np.int64)
    side = rng.integers(0, 3, (4, G)).astype(np.uint8)
    got = folds._group_rows(gidx, side, G)
    for k, (tr, te) in enumerate(got):
        np.testing.assert_array_equal(tr, np.flatnonzero(side[k][gidx] == 1))
        np.testing.assert_array_equal(te, np.flatnonzero(side[k][gidx] == 2))
    bad = gidx.copy()
    bad[n // 2] = G
    with pytest.raises(Exception, match="outside"):
        folds._group_rows(bad, side, G)
    out = np.empty(3, dtype=np.int64)
    ptrs = (ctypes.c_void_p * 2)(out.ctypes.data, out.ctypes.data)
    lens = np.array([3, 3], dtype=np.int64)
    with pytest.raises(Exception, match="len"):
        _lib.call("sglm_host_group_rows", gidx.ctypes.data, n, side.ctypes.data, 1, G,
                  ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, 4)


@pytest.mark.parametrize("kind", ["dense", "gaps", "offset", "float"])
def test_group_shuffle_split_id_kinds_vs_sklearn(kind):
    """folds.group_shuffle_split on dense codes, integer ids with gaps, ids not starting at 0
    and float ids == sklearn GroupShuffleSplit on the same global RNG state."""
    from sklearn.model_selection import GroupShuffleSplit
    from sglm_hip import folds
    rng = np.random.default_rng(4)
    g = np.sort(rng.integers(0, 60, 5000))
    g = {"dense": np.unique(g, return_inverse=True)[1].astype(np.int16), "gaps": g * 3,
         "offset": g + 1000, "float": g.astype(np.float64) / 7}[kind]
    np.random.seed(9)
    got = folds.group_shuffle_split(g, 4, 0.25)
    np.random.seed(9)
    ref = list(GroupShuffleSplit(n_splits=4, test_size=0.25).split(g, None, g))
    for (a, b), (c, d) in zip(got, ref):
        assert np.array_equal(a, c) and np.array_equal(b, d)
