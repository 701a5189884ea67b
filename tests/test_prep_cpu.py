"""Session preprocessing (lynne_pp.preprocess_lynne): oracle vs the pandas formulation on CPU,
and the product's refusal to run without the GPU engine."""
import numpy as np
import pytest

from oracle import prep_ref
from oracle.prep_pandas import derived_columns
from sglm_hip.synth import session as synth_session


def _same(a, b):
    """Bit-level equality: NaN positions and the sign of zeros (-0.0 from the clamp) too."""
    a, b = np.asarray(a), np.asarray(b)
    return (a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b))
            and np.array_equal(np.nan_to_num(a, nan=7.0), np.nan_to_num(b, nan=7.0))
            and np.array_equal(np.signbit(a), np.signbit(b)))


@pytest.mark.parametrize("n,seed,k,rate", [
    (3000, 0, 7, 0.02), (3000, 15, 1, 0.02), (3000, 1, 0, 0.05), (2000, 2, -3, 0.03), (500, 3, 7, 0.2),
    (6, 4, 7, 0.5), (1, 5, 7, 0.5), (400, 6, 7, 0.0), (2500, 7, 25, 0.01),
])
def test_oracle_matches_pandas_semantics(n, seed, k, rate):
    _, cols = synth_session(n, seed, rate)
    ref = derived_columns(cols, k)
    got = prep_ref.preprocess_columns(cols, k)
    assert list(got) == list(prep_ref.OUT_COLS)
    for name in prep_ref.OUT_COLS:
        assert _same(got[name], ref[name]), name


def with_nans(cols, seed, frac=0.01, names=("r", "nr", "cpn", "lpx", "rpn", "ll")):
    """Float copies of the session columns with NaN at random rows of `names` (missing samples
    in the acquisition files): pandas' skipna sums/cumsums and NaN-key groupby paths."""
    rng = np.random.default_rng(seed)
    out = {c: np.asarray(v, dtype=np.float64).copy() for c, v in cols.items()}
    for c in names:
        out[c][rng.random(out[c].size) < frac] = np.nan
    return out


@pytest.mark.parametrize("n,seed,k,names", [
    (3000, 20, 7, ("r",)), (3000, 21, 1, ("r", "nr")), (2500, 22, 7, ("r", "nr", "cpn", "lpx", "rpn", "ll")),
    (2049, 23, -3, ("cpn", "rpx", "lpn")),
])
def test_oracle_matches_pandas_with_nan_inputs(n, seed, k, names):
    _, cols = synth_session(n, seed, 0.03)
    cols = with_nans(cols, seed, 0.02, names)
    ref = derived_columns(cols, k)
    got = prep_ref.preprocess_columns(cols, k)
    for name in prep_ref.OUT_COLS:
        assert _same(got[name], ref[name]), name


def test_oracle_columns_match_product_layout():
    import sglm_hip.prep as prep
    assert prep.IN_COLS == prep_ref.IN_COLS and prep.OUT_COLS == prep_ref.OUT_COLS
    hdr = open("include/sglm_hip.h").read()
    body = hdr[hdr.index("enum sglm_prep_out"):]
    body = body[:body.index("};")]
    names = [t.strip().split("=")[0].strip() for t in body.split("{")[1].split(",")]
    names = [t for t in names if t]
    assert names[-1] == "SGLM_PREP_NOUT" and len(names) - 1 == len(prep.OUT_COLS)
    for t, name in zip(names, prep.OUT_COLS):
        assert t == "SGLM_PREP_OUT_" + name.upper(), (t, name)


def test_preprocess_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import lynne_pp
    from sglm_hip._lib import HipEngineUnavailable
    df, _ = synth_session(100, 0)
    with pytest.raises(HipEngineUnavailable):
        lynne_pp.preprocess_lynne(df)
