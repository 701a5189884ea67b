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
        E.host_masks([(np.array([-1, 3]), False)], n, ld)
