"""Drop-in for ``lynne_pp.py`` (import as ``import lynne_pp as lpp``): session preprocessing.

``preprocess_lynne(df, trial_shift_bounds=7)`` (lynne_pp.py:217-249) runs its arithmetic on
the MI355X in one call of ``sglm_prep_session``: trial segmentation (define_trial_starts_ends,
:20-44), reward flags (set_reward_flags, :113-125), port indicators (:127-158), side-agnostic
events (:160-180) and first-time events (get_first_time_events, :182-215).  The reference runs
these as pandas column operations and groupby passes; here they are row kernels and chunked
scans over float64 columns.  pandas bookkeeping stays on the host and follows the reference:
'Unnamed' columns dropped, the rename map, new columns appended in the reference's order
(existing columns of the same name overwritten in place), 'index' dropped, the whole frame
cast to float after the side-agnostic events, the 'Percent of Data in ITI' line printed.

Differences: event columns must be numeric (the reference would also accept the string
'False', replaced only after the trial segmentation); the per-trial sum of ``r`` is exact for
integer-valued rewards (the indicator columns the sessions hold) and otherwise summed in
chunk order.  The other lynne_pp helpers (detrend, get_is_not_iti, timeshift_vals,
get_first_entry_time) are outside this path.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from sglm_hip import prep as _prep

_RENAME = {"Ch1": "Ch1", "Ch2": "Ch2", "Ch5": "Ch5", "Ch6": "Ch6",
           "centerOcc": "cpo", "centerIn": "cpn", "centerOut": "cpx",
           "rightOcc": "rpo", "rightIn": "rpn", "rightOut": "rpx", "rightLick": "rl",
           "leftOcc": "lpo", "leftIn": "lpn", "leftOut": "lpx", "leftLick": "ll",
           "reward": "r", "noreward": "nr"}

# where each derived column appears in the reference's sequence of steps
_STEP_TRIALS = _prep.OUT_COLS[0:6]         # define_trial_starts_ends
_STEP_REWARD = _prep.OUT_COLS[6:8]         # set_reward_flags
_STEP_PORTS = _prep.OUT_COLS[8:16]         # set_port_entry_exit_rewarded_unrewarded_...
_STEP_SIDES = _prep.OUT_COLS[16:23]        # define_side_agnostic_events
_STEP_FIRST = _prep.OUT_COLS[23:40]        # get_first_time_events


def rename_columns(df: pd.DataFrame) -> pd.DataFrame:
    """lynne_pp.py:47-111: the session's long column names to the GLM's short ones."""
    return df.rename(_RENAME, axis=1)


def _assign(df: pd.DataFrame, names, cols) -> pd.DataFrame:
    new = [c for c in names if c not in df.columns]
    for c in names:
        if c in df.columns:
            df[c] = cols[c]
    if new:
        df = pd.concat([df, pd.DataFrame({c: cols[c] for c in new}, index=df.index)], axis=1)
    return df


def preprocess_lynne(df: pd.DataFrame, trial_shift_bounds: int = 7) -> pd.DataFrame:
    df = df[[c for c in df.columns if "Unnamed" not in c]]
    df = rename_columns(df)
    missing = [c for c in _prep.IN_COLS if c not in df.columns]
    if missing:
        raise KeyError(missing[0])
    X = np.empty((len(_prep.IN_COLS), len(df)), dtype=np.float64)
    for i, c in enumerate(_prep.IN_COLS):
        col = df[c]
        if not (pd.api.types.is_numeric_dtype(col) or pd.api.types.is_bool_dtype(col)):
            raise TypeError(f"column {c!r} must be numeric, got {col.dtype}")
        X[i] = col.to_numpy(dtype=np.float64)
    D = _prep.session_columns(X, int(trial_shift_bounds))
    cols = {name: D[j] for j, name in enumerate(_prep.OUT_COLS)}

    df = df.drop(columns=[c for c in ("event_col_a", "event_col_b", "event_col_c")
                          if c in df.columns]).copy()
    df = _assign(df, _STEP_TRIALS, cols)
    print("Percent of Data in ITI:", float(np.mean(cols["nTrial"] == cols["nEndTrial"])))
    df = _assign(df, _STEP_REWARD, cols)
    df = _assign(df, _STEP_PORTS, cols)
    df = _assign(df, _STEP_SIDES, cols)
    if "index" in df.columns:
        df = df.drop("index", axis=1)
    dfrel = df.copy()
    dfrel = dfrel.replace("False", 0).astype(float)
    dfrel = dfrel * 1
    dfrel = dfrel[[c for c in dfrel.columns if "Unnamed" not in c]]
    return _assign(dfrel, _STEP_FIRST, cols)
