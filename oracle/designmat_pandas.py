"""pandas formulation of pp_design_mat.make_design_mat -- TEST INFRASTRUCTURE ONLY.

The reference (/root/reference/pp_design_mat.py:6-205) builds the event design matrix of a
behaviour session with pandas column arithmetic, groupby cumcount / nth / first / sum and
Series.map lookups into the trial table.  This module states the same computation as
pandas operations (pandas' own semantics of groupby over a float key with NaN rows dropped,
cumcount, nth, first-non-null, map with missing keys, get_dummies), step by step with the
reference line each step follows.  It is the pin of oracle/designmat_ref.py (explicit
per-row / per-trial walks) in tests/test_designmat_cpu.py; the product never imports it.

The reference has no test or fixture for this function and its import is denied
(SURVEY.md §8(c)), so parity is "pinned to pandas semantics".

Deliberate deviation, shared with the product: the reference raises KeyError('flag') at
:196 when ``interactions`` is None/empty (the column is only created inside the
interactions branch, :189).  Here ``flag`` starts at 0 in that case, so the function is
usable without interactions; with interactions the behaviour is the reference's.
"""
from __future__ import annotations

import re

import numpy as np
import pandas as pd

ENL_SCALE = 50 * 100          # cumcount**2 / (50*100)   (pp_design_mat.py:171-172)
MS_PER_ROW = 1000 / 50        # (pp_design_mat.py:121)


def state_lick_name(state: str) -> str:
    """classify_lick_state's column name (:21)."""
    return f"{state[:3].lower()}_lick"


def lick_states(ts: pd.DataFrame, states) -> pd.DataFrame:
    """classify_lick_state (:6-23): one '<sta>_lick' column per state, state * Lick."""
    out = ts.copy()
    for st in states:
        out[state_lick_name(st)] = out[st] * out["Lick"]
    return out


def pull_nth_licks(ts: pd.DataFrame, lick_pos, state="Consumption",
                   keep_only_nth_lick=False) -> pd.DataFrame:
    """pull_lick_from_bout (:26-58): for each requested position (descending when several),
    the nth lick of the bout column within each nTrial moves to its own column."""
    bout = state_lick_name(state)
    order = sorted(lick_pos)[::-1] if len(lick_pos) > 1 else list(lick_pos)
    out = ts.copy()
    for nth in order:
        col = f"{bout}_{nth}"
        out[col] = 0
        licks = out.loc[out[bout] == 1].copy()
        picked = licks.groupby("nTrial", as_index=False).nth(nth - 1).index
        out.loc[picked, col] = 1
        out.loc[licks.groupby("nTrial", as_index=False).nth(nth - 1).index, bout] = 0
    if keep_only_nth_lick:
        out = out.drop(columns=[bout])
    return out


def interact(ts: pd.DataFrame, trials: pd.DataFrame, states, trial_type,
             as_dummy=True, drop_non_interaction=True) -> pd.DataFrame:
    """event_interactions_dummies (:61-105): the columns whose name matches any state's
    3-letter prefix, multiplied by every dummy of trials[trial_type] mapped onto the rows."""
    pattern = "|".join(s.lower()[:3] for s in states)
    picked = [c for c in ts.columns if re.search(pattern, str(c))]
    later = [c for c in ts.columns if c not in picked]
    out = ts[picked].copy()
    if not as_dummy:
        # the reference assigns this branch's frame to a misspelled name (:90), so the loop
        # below reads an undefined variable: NameError, kept
        raise NameError("name 'dummies' is not defined")
    dummies = pd.get_dummies(trials[trial_type], prefix=trial_type)
    for dc in dummies.columns:
        per_row = ts["nTrial"].map(dummies[dc])
        names = [f"{trial_type.lower()[:3]}_{dc.split('_')[-1]}_{c}" for c in picked]
        out[names] = out[picked].multiply(per_row, axis="index")
    if drop_non_interaction:
        out = out.drop(columns=picked)
    out[later] = ts[later].copy()
    return out


def heatmap_columns(ts: pd.DataFrame, trials: pd.DataFrame) -> pd.DataFrame:
    """add_heatmap_columns (:108-126)."""
    out = ts.copy()
    out["hm_t_cue_offset_to_sel"] = out["nTrial"].map(trials["tSelection"])
    first_cue = out.loc[out.Cue == 1].groupby("nTrial")["trial_clock"].first()
    out["hm_t_from_cue_onset"] = out["trial_clock"] - out["nTrial"].map(first_cue)
    first_cons = out.loc[out.Consumption == 1].groupby("nTrial")["trial_clock"].first()
    out["hm_t_from_cons_onset"] = out["trial_clock"] - out["nTrial"].map(first_cons)
    sums = out.groupby("nTrial", as_index=False).agg({"Consumption": "sum",
                                                       "stateConsumption": "sum"})
    sums["t_sel_to_cons"] = (sums.stateConsumption - sums.Consumption) * MS_PER_ROW
    out["hm_t_sel_to_cons"] = out["nTrial"].map(sums.set_index("nTrial")["t_sel_to_cons"])
    out["hm_t_cue_offset_to_cons"] = out["hm_t_sel_to_cons"] + out["hm_t_cue_offset_to_sel"]
    return out[[c for c in out.columns if str(c).startswith("hm")]]


def make_design_mat(timeseries: pd.DataFrame, trials: pd.DataFrame, states=None,
                    nth_licks=None, interactions=None, verbose=True) -> pd.DataFrame:
    """make_design_mat (:128-205).  Adds 'Lick' to the caller's ``timeseries`` (:160), as
    the reference does."""
    states = ["Select", "Consumption", "ENLP"] if states is None else states
    nth_licks = [1] if nth_licks is None else nth_licks
    tr = trials.set_index("nTrial").convert_dtypes()
    photo = [c for c in timeseries.columns if "z_grn" in c]
    hm = heatmap_columns(timeseries, tr)
    timeseries["Lick"] = (~np.isnan(timeseries.iSpout)).astype("int")
    ts = lick_states(timeseries, states)
    lick_cols = [c for c in ts.columns if "_lick" in c]
    ts["time_from_enl_onset"] = 0
    ts["time_from_enlp_onset"] = 0
    enl = (ts.ENL == 1) | (ts.Cue == 1)
    ts.loc[enl, "time_from_enl_onset"] = (
        ts.loc[enl].groupby("nTrial").cumcount() ** 2) / ENL_SCALE
    enlp = ts.state_ENLP == 1
    ts.loc[enlp, "time_from_enlp_onset"] = (
        ts.loc[enlp].groupby(["nTrial", "nENL"]).cumcount() ** 2) / ENL_SCALE
    onsets = ts.loc[ts.Cue == 1].groupby("nTrial", as_index=False).nth(0).index.values
    dm = ts[lick_cols + ["nTrial", "iBlock", "time_from_enl_onset", "time_from_enlp_onset"]
            + photo].copy()
    dm["cue"] = 0
    dm.loc[onsets, "cue"] = 1
    dm = pull_nth_licks(dm, nth_licks, keep_only_nth_lick=True)
    if interactions:
        dm["flag"] = 0
        for trial_type, st_ in interactions.items():
            dm["flag"] += dm["nTrial"].map(tr[trial_type].isna())
            dm = interact(dm, tr, states=st_, trial_type=trial_type)
    else:
        dm["flag"] = 0                  # reference: KeyError('flag') at :196 (fixed)
    dm[hm.columns] = hm
    dm["flag"] = dm["flag"].clip(0, 1)
    cue_like = [c for c in dm.columns if c.endswith("cue")]
    per_trial = dm.groupby("nTrial")[cue_like].sum().sum(axis=1)
    without = per_trial.loc[per_trial == 0].index.values
    if verbose:
        print(f"trials_without_dummies = {without!r}")
    dm.loc[dm.nTrial.isin(without), "flag"] = 1
    return dm
