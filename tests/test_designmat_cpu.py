"""pp_design_mat.make_design_mat oracles on the CPU.

oracle/designmat_ref.py (explicit row / per-trial walks) is pinned to oracle/designmat_pandas.py
(the reference's lines as pandas operations: groupby cumcount / nth / first, map, get_dummies)
on synthetic sessions: column names and order, every value with its NaN positions.  The
reference holds no fixture for this function and its import is denied, so
parity is pinned to pandas semantics."""
import warnings

import numpy as np
import pandas as pd
import pytest

from oracle import designmat_pandas as P, designmat_ref as R

warnings.filterwarnings("ignore", category=FutureWarning)

ROW_COLS = ["nTrial", "nENL", "iBlock", "iSpout", "Cue", "ENL", "state_ENLP", "Consumption",
            "stateConsumption", "trial_clock", "Select", "ENLP", "z_grnR", "z_grnL"]


def as_f64(s):
    return s.to_numpy(dtype=np.float64, na_value=np.nan)


def run_both(ts, tr, **kw):
    pd_out = P.make_design_mat(ts.copy(), tr, verbose=False, **kw)
    cols = {c: ts[c].to_numpy(dtype=np.float64) for c in ROW_COLS}
    tcols = {c: tr[c].to_numpy(dtype=np.float64) for c in tr.columns}
    names, ref = R.design_columns(cols, tcols, photo=("z_grnR", "z_grnL"),
                                  **{k: v for k, v in kw.items()})
    return pd_out, names, ref


CASES = [
    dict(),
    dict(nth_licks=[1, 2]),
    dict(nth_licks=[2, 1, 3]),
    dict(nth_licks=[1, 1]),
    dict(nth_licks=[0]),
    dict(interactions={"Reward": ["Consumption", "Cue"]}),
    dict(interactions={"Reward": ["Consumption", "Cue"], "h2": ["Select", "ENLP"]}),
    dict(states=["Select", "Consumption"], interactions={"h2": ["Cons"]}),
]


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("kw", CASES)
def test_explicit_walk_oracle_equals_pandas_formulation(seed, kw):
    ts, tr = __import__("sglm_hip.synth", fromlist=["x"]).designmat_session(40, seed)
    kw = {k: (dict(v) if isinstance(v, dict) else v) for k, v in kw.items()}
    out, names, ref = run_both(ts, tr, **kw)
    assert list(out.columns) == names
    for c in names:
        np.testing.assert_array_equal(as_f64(out[c]), ref[c], err_msg=c)


def test_pandas_formulation_edge_semantics():
    """The pandas behaviours the device path must reproduce, on a hand-made session."""
    nan = np.nan
    ts = pd.DataFrame({
        "nTrial":      [nan, 1, 1, 1, 1, 2, 2, 2, nan, 2, 3, 3],
        "nENL":        [nan, 1, 1, 2, 2, 1, 1, 1, nan, 1, 1, 1],
        "iBlock":      [nan, 0, 0, 0, 0, 0, 0, 0, nan, 0, 0, 0],
        "iSpout":      [1, nan, 1, 1, 2, 1, nan, 1, 1, 1, nan, nan],
        "Cue":         [1, 1, 1, 0, 0, 0, 0, 0, 1, 0, 0, 0],
        "ENL":         [0, 0, 0, 1, 1, 1, 0, 0, 0, 0, 0, 0],
        "state_ENLP":  [1, 0, 0, 1, 1, 0, 0, 0, 1, 0, 0, 0],
        "Select":      [0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0],
        "Consumption": [0, 0, 0, 0, 1, 0, 1, 1, 0, 1, 1, 0],
        "ENLP":        [0, 0, 0, 1, 1, 0, 0, 0, 0, 0, 0, 0],
        "stateConsumption": [0, 0, 0, 0, 1, 1, 1, 1, 0, 1, 1, 1],
        "trial_clock": [nan, nan, 20, 40, 60, 0, 20, 40, 60, 80, 0, 20],
        "z_grnR": np.arange(12.0), "z_grnL": -np.arange(12.0)})
    tr = pd.DataFrame({"nTrial": [1, 2], "tSelection": [100.0, nan], "Reward": [1.0, nan],
                       "h2": [0.0, 1.0]})
    out, names, ref = run_both(ts, tr, interactions={"Reward": ["Consumption", "Cue"]})
    assert list(out.columns) == names
    for c in names:
        np.testing.assert_array_equal(as_f64(out[c]), ref[c], err_msg=c)
    # first non-null clock among the cue rows of trial 1 (row 1's clock is NaN): row 2's
    assert as_f64(out["hm_t_from_cue_onset"])[3] == 40 - 20
    # trial 2 has no cue row, trial 3 is not in the trial table: both flagged
    f = as_f64(out["flag"])
    assert np.isnan(f[0]) and f[1] == 0 and np.all(f[5:8] == 1) and np.all(f[10:] == 1)
    # the counters: NaN on NaN-trial rows that meet the condition, 0 elsewhere
    t = as_f64(out["time_from_enlp_onset"])
    assert np.isnan(t[0]) and t[3] == 0 and t[4] == 1 / 5000
