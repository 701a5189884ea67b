"""Session preprocessing on the MI355X (sglm_prep_session through the C ABI) vs the CPU oracle
(oracle/prep_ref.py) and the pandas formulation (tests/prep_pandas.py).  Integer-valued event
columns -> bit-exact, NaN positions and signed zeros included."""
import numpy as np
import pandas as pd
import pytest

from oracle import prep_ref
from oracle.prep_pandas import derived_columns
from sglm_hip.synth import session as synth_session
from test_prep_cpu import _same, with_nans

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prep():
    import torch
    assert torch.cuda.is_available()
    from sglm_hip import prep as p
    return p


def _stack(cols):
    return np.stack([np.asarray(cols[c], dtype=np.float64) for c in prep_ref.IN_COLS])


@pytest.mark.parametrize("n,seed,k,rate", [
    (3000, 0, 7, 0.02), (3000, 15, 1, 0.02), (3000, 1, 0, 0.05), (2000, 2, -3, 0.03), (500, 3, 7, 0.2),
    (6, 4, 7, 0.5), (1, 5, 7, 0.5), (400, 6, 7, 0.0), (2500, 7, 25, 0.01),
    # scan chunk boundaries (2048 rows per chunk) with trials spanning chunks
    (2047, 8, 7, 0.002), (2048, 9, 7, 0.002), (2049, 10, 7, 0.002), (20000, 11, 7, 0.0005),
])
def test_session_columns_vs_oracle(prep, n, seed, k, rate):
    _, cols = synth_session(n, seed, rate)
    D = prep.session_columns(_stack(cols), k)
    ref = prep_ref.preprocess_columns(cols, k)
    for j, name in enumerate(prep_ref.OUT_COLS):
        assert _same(D[j], ref[name]), name


@pytest.mark.parametrize("n,seed,k,names", [
    (3000, 20, 7, ("r",)), (3000, 21, 1, ("r", "nr")),
    (2500, 22, 7, ("r", "nr", "cpn", "lpx", "rpn", "ll")), (2049, 23, -3, ("cpn", "rpx", "lpn")),
    (20000, 24, 7, ("r", "cpn")),
])
def test_session_columns_nan_inputs_vs_oracle(prep, n, seed, k, names):
    """NaN samples in the event / reward columns (the per-trial reward total of a
    NaN-r row must be the trial's skipna sum, as groupby('nTrial')['r'].transform(sum))."""
    _, cols = synth_session(n, seed, 0.03 if n < 10000 else 0.002)
    cols = with_nans(cols, seed, 0.02, names)
    D = prep.session_columns(_stack(cols), k)
    ref = prep_ref.preprocess_columns(cols, k)
    for j, name in enumerate(prep_ref.OUT_COLS):
        assert _same(D[j], ref[name]), name


def test_session_columns_empty(prep):
    D = prep.session_columns(np.zeros((9, 0)), 7)
    assert D.shape == (40, 0)


def test_session_columns_large_vs_pandas(prep):
    # > 1024 scan chunks: the carry kernel walks several chunks per thread
    n = 3_000_001
    _, cols = synth_session(n, 12, 0.001, with_extra=False)
    D = prep.session_columns(_stack(cols), 7)
    ref = derived_columns(cols, 7)
    for j, name in enumerate(prep_ref.OUT_COLS):
        assert _same(D[j], ref[name]), name
    nt = D[prep_ref.OUT_COLS.index("nTrial")]
    assert np.nanmax(nt) > 100 and np.all(np.diff(nt[~np.isnan(nt)]) >= 0)


def test_preprocess_lynne_frame(capsys):
    import lynne_pp
    df, cols = synth_session(5000, 13, 0.02)
    df["index"] = np.arange(len(df))           # dropped by the reference (lynne_pp.py:240-241)
    out = lynne_pp.preprocess_lynne(df, trial_shift_bounds=5)
    ref = derived_columns(cols, 5)
    renamed = [lynne_pp._RENAME.get(c, c) for c in df.columns
               if "Unnamed" not in c and c != "index"]
    assert list(out.columns) == renamed + list(prep_ref.OUT_COLS)
    assert all(out[c].dtype == np.float64 for c in out.columns)
    for c in renamed:
        src = [k for k in df.columns if lynne_pp._RENAME.get(k, k) == c][0]
        assert np.array_equal(out[c].to_numpy(), df[src].to_numpy(dtype=np.float64))
    for name in prep_ref.OUT_COLS:
        assert _same(out[name].to_numpy(), ref[name]), name
    iti = float(np.mean(ref["nTrial"] == ref["nEndTrial"]))
    assert f"Percent of Data in ITI: {iti}" in capsys.readouterr().out
    assert "index" not in out.columns and df.shape[1] == 13   # caller's frame untouched


def test_preprocess_lynne_overwrites_existing_columns():
    import lynne_pp
    df, cols = synth_session(3000, 14, 0.02)
    df.insert(2, "nTrial", -1.0)               # an existing column keeps its position
    out = lynne_pp.preprocess_lynne(df)
    assert list(out.columns).index("nTrial") == 1
    assert _same(out["nTrial"].to_numpy(), derived_columns(cols, 7)["nTrial"])
    with pytest.raises(KeyError):
        lynne_pp.preprocess_lynne(df.drop(columns=["reward"]))
