"""Drop-in for the reference's ``pp_design_mat`` module (/root/reference/pp_design_mat.py):
the event design matrix of a behaviour session, with the per-row and per-trial work on the
MI355X (csrc/designmat.hip through sglm_hip/designmat.py).

Same functions, arguments and results as the reference (column names, order, index, values
and NaN positions; dtypes as pandas gives them where pandas yields a numpy dtype, float64 where
it yields object / nullable columns -- see sglm_hip/designmat.py).  Behaviour kept on purpose:
``make_design_mat`` adds the 'Lick' column to the caller's frame (:160) and prints
``trials_without_dummies`` (:202); ``event_interactions_dummies(as_dummy=False)`` raises the
reference's UnboundLocalError (the misspelt ``dummes``, :90).  Fixed on purpose:
``make_design_mat`` without ``interactions`` raised KeyError('flag') (:196); here 'flag'
starts at 0 and the cue check still applies.  There is no CPU fallback: without the library
or a ROCm device every function raises HipEngineUnavailable.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

from sglm_hip import designmat as _dm


def _col(df, c, dev="cuda"):
    import torch
    return torch.from_numpy(np.ascontiguousarray(
        df[c].to_numpy(dtype=np.float64, na_value=np.nan))).to(dev)


def _host(t):
    return t.cpu().numpy()


def _as_dtype(v, dt):
    if isinstance(dt, np.dtype) and dt.kind in "iub" and not np.all(np.isfinite(v)):
        return v
    return v.astype(dt) if isinstance(dt, np.dtype) else v


def classify_lick_state(timeseries, state):
    """pp_design_mat.py:6-23: '<sta>_lick' = state * Lick for each state."""
    _dm._require_gpu()
    t_ = timeseries.copy()
    lick = _col(t_, "Lick")
    outs, _ = _dm.licks(lick, False, [_col(t_, s) for s in state])
    for s, o in zip(state, outs):
        dt = np.result_type(t_[s].dtype, t_["Lick"].dtype)
        t_[f"{s[:3].lower()}_lick"] = _as_dtype(_host(o), dt)
    return t_


def pull_lick_from_bout(timeseries, lick_pos, state="Consumption", keep_only_nth_lick=False):
    """pp_design_mat.py:26-58: the nth lick of each trial's bout into its own column."""
    _dm._require_gpu()
    import torch
    bout_type = f"{state.lower()[:3]}_lick"
    if len(lick_pos) > 1:
        lick_pos = sorted(lick_pos)[::-1]
    t_ = timeseries.copy()
    if bout_type not in t_.columns:
        raise KeyError(bout_type)
    bout = _col(t_, bout_type)
    g = _dm.group_rows(_col(t_, "nTrial"))
    names, cols = [], []
    for nth in lick_pos:
        nm = "_".join([bout_type, str(nth)])
        if nm not in names:
            names.append(nm)
            cols.append(torch.empty(len(t_), dtype=torch.float64, device="cuda"))
        else:
            cols.append(cols[names.index(nm)])
    _dm.pull(bout, g, list(lick_pos), cols)
    for nm in names:
        t_[nm] = _host(cols[names.index(nm)]).astype(np.int64)
    t_[bout_type] = _as_dtype(_host(bout), t_[bout_type].dtype)
    if keep_only_nth_lick:
        t_.drop(columns=[bout_type], inplace=True)
    return t_


def event_interactions_dummies(timeseries, trials, states, trial_type, as_dummy=True,
                               drop_non_interaction=True):
    """pp_design_mat.py:61-105 (``trials`` indexed by nTrial, as make_design_mat passes it)."""
    import re
    _dm._require_gpu()
    import torch
    pat = "|".join(s.lower()[:3] for s in states)
    t_ = timeseries.filter(regex=pat)
    cols_to_interact = list(t_.columns)
    cols_for_later = [c for c in timeseries.columns if c not in t_.columns]
    if not as_dummy:
        raise UnboundLocalError("local variable 'dummies' referenced before assignment")
    labels, dvals = _dm._dummy_labels(trials[trial_type], trial_type)
    tt = _dm.TrialTable(trials.index.to_numpy(dtype=np.float64, na_value=np.nan), "cuda")
    tidx = tt.lookup(_col(timeseries, "nTrial"))
    unmapped = bool((tidx < 0).any().item())
    nsrc = len(cols_to_interact)
    if labels and nsrc:
        src = torch.stack([_col(t_, c) for c in cols_to_interact])
        vals = tt.values(dvals.T)
        out = torch.empty((len(labels) * nsrc, len(t_)), dtype=torch.float64, device="cuda")
        _dm.trial_map(tidx, src, [q for _ in labels for q in range(nsrc)], vals,
                      [d for d in range(len(labels)) for _ in range(nsrc)], out,
                      list(range(len(labels) * nsrc)))
        host = _host(out)
        for d, lab in enumerate(labels):
            for q, c in enumerate(cols_to_interact):
                dt = np.dtype(np.float64) if unmapped else np.result_type(t_[c].dtype, np.bool_)
                t_[f"{trial_type.lower()[:3]}_{lab}_{c}"] = _as_dtype(host[d * nsrc + q], dt)
    if drop_non_interaction:
        t_ = t_.drop(columns=cols_to_interact)
    t_[cols_for_later] = timeseries[cols_for_later].copy()
    return t_


def add_heatmap_columns(timeseries, trials):
    """pp_design_mat.py:108-126 (``trials`` indexed by nTrial)."""
    _dm._require_gpu()
    cols = {c: _col(timeseries, c) for c in ("nTrial", "trial_clock", "Cue", "Consumption",
                                             "stateConsumption")}
    g = _dm.group_rows(cols["nTrial"])
    tt = _dm.TrialTable(trials.index.to_numpy(dtype=np.float64, na_value=np.nan), "cuda")
    tidx = tt.lookup(cols["nTrial"])
    tsel = tt.values(trials["tSelection"].to_numpy(dtype=np.float64, na_value=np.nan))
    hm = _host(_dm.heatmap(cols, g, tidx, tsel[0]))
    names = [c for c in timeseries.columns if str(c).startswith("hm")]
    out = {c: timeseries[c] for c in names}
    for j, c in enumerate(_dm.HM_COLUMNS):
        if c not in names:
            names.append(c)
        out[c] = hm[j][: len(timeseries)]
    return pd.DataFrame(out, index=timeseries.index, columns=names)


def make_design_mat(timeseries, trials, states=None, nth_licks=None, interactions=None):
    """pp_design_mat.py:128-205."""
    if states is None:
        states = ["Select", "Consumption", "ENLP"]
    if nth_licks is None:
        nth_licks = [1]
    trials = trials.set_index("nTrial").convert_dtypes()
    res = _dm.design_matrix(timeseries, trials, states, nth_licks, interactions)
    timeseries["Lick"] = _host(res.lick).astype("int")          # the reference's side effect
    return _dm.to_frame(res, timeseries.index)
