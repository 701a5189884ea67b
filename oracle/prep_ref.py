"""CPU restatement of the session preprocessing — TEST INFRASTRUCTURE.

``lynne_pp.preprocess_lynne`` (lynne_pp.py:217-249) on float64 numpy columns, written as
explicit row / per-trial walks (not as the GPU's scans), so that the two formulations check
each other:

* ``trial_starts_ends`` — define_trial_starts_ends (lynne_pp.py:20-44)
* ``reward_flags``      — set_reward_flags (:113-125); groupby drops NaN trial keys
* ``port_indicators``   — set_port_entry_exit_rewarded_unrewarded_indicators (:127-158)
* ``side_agnostic``     — define_side_agnostic_events (:160-180)
* ``first_time_events`` — get_first_time_events (:182-215)
* ``preprocess_columns`` — the whole chain; returns {column name: float64 array} for the
                           derived columns, in the order the reference appends them.

Inputs are the renamed session columns (rename_columns, :95-111).  Pinning: the reference
has no test or fixture for this path and its import is denied here, so this
restatement is pinned by tests/test_prep_cpu.py against an independent pandas-operation
formulation of the same lines (Series.shift / bfill / ffill / cumsum, groupby transform /
cumsum, DataFrame.diff) on seeded sessions: "parity pinned to pandas semantics, reference
outputs unavailable".
"""
from __future__ import annotations

import numpy as np

IN_COLS = ("cpn", "lpx", "rpx", "lpn", "rpn", "r", "nr", "rl", "ll")
OUT_COLS = (
    "event_col", "trial_start_flag", "nTrial", "event_col_end", "trial_end_flag", "nEndTrial",
    "r_trial", "nr_trial",
    "rpxr", "rpxnr", "lpxr", "lpxnr", "rpnr", "rpnnr", "lpnr", "lpnnr",
    "spn", "spx", "spnr", "spnnr", "spxr", "spxnr", "sl",
    "nn", "xx",
    "ft_nn", "ft_xx", "ft_lpn", "ft_rpn", "ft_spn", "ft_lpx", "ft_rpx", "ft_spx", "ft_cpn",
    "ft_r_rpn", "ft_r_lpn", "ft_r_spn", "ft_nr_rpn", "ft_nr_lpn", "ft_nr_spn",
)


def _code(v, f):
    """x.replace(0, nan) * f."""
    out = np.where(v == 0, np.nan, v) * f
    return out


def _first_of(*cols):
    """a.combine_first(b).combine_first(c) ..."""
    out = cols[0].copy()
    for c in cols[1:]:
        m = np.isnan(out)
        out[m] = c[m]
    return out


def _shifted(cond, s):
    """bool Series.shift(s) * 1.0: value at t is cond[t - s], NaN outside the session."""
    n = len(cond)
    out = np.full(n, np.nan)
    for t in range(n):
        u = t - s
        if 0 <= u < n:
            out[t] = 1.0 if cond[u] else 0.0
    return out


def _cumsum_skipna(x):
    out = np.full(len(x), np.nan)
    acc = 0.0
    for t, v in enumerate(x):
        if not np.isnan(v):
            acc += v
            out[t] = acc
    return out


def trial_starts_ends(c, k):
    n = len(c["cpn"])
    ev = _first_of(_code(c["cpn"], 1.0), _code(c["lpx"], 2.0), _code(c["rpx"], 2.0))
    nxt = np.nan                                     # bfill: walk from the end
    for t in range(n - 1, -1, -1):
        if np.isnan(ev[t]):
            ev[t] = nxt
        else:
            nxt = ev[t]
    cond = np.zeros(n, bool)
    for t in range(n):
        after = ev[t + 1] if t + 1 < n else np.nan
        cond[t] = ev[t] == 1.0 and not after == 1.0
    start = _shifted(cond, -k)
    ntrial = _cumsum_skipna(start)
    ece = _first_of(_code(c["lpx"], 2.0), _code(c["rpx"], 2.0), _code(start, 1.0))
    last = np.nan                                    # ffill
    for t in range(n):
        if np.isnan(ece[t]):
            ece[t] = last
        else:
            last = ece[t]
    cond = np.zeros(n, bool)
    for t in range(n):
        before = ece[t - 1] if t >= 1 else np.nan
        cond[t] = ece[t] == 2.0 and not before == 2.0 and ntrial[t] > 0
    end = _shifted(cond, k)
    return {"event_col": ev, "trial_start_flag": start, "nTrial": ntrial,
            "event_col_end": ece, "trial_end_flag": end, "nEndTrial": _cumsum_skipna(end)}


def _trial_runs(ntrial):
    """(start, stop) row ranges of the trials (nTrial is nondecreasing where defined)."""
    runs = []
    t, n = 0, len(ntrial)
    while t < n:
        if np.isnan(ntrial[t]):
            t += 1
            continue
        u = t
        while u + 1 < n and ntrial[u + 1] == ntrial[t]:
            u += 1
        runs.append((t, u + 1))
        t = u + 1
    keys = [ntrial[a] for a, _ in runs]
    assert len(set(keys)) == len(keys), "trial numbers must form contiguous runs"
    return runs


def reward_flags(c, ntrial):
    n = len(ntrial)
    r_trial, nr_trial = np.zeros(n), np.zeros(n)
    for a, b in _trial_runs(ntrial):
        tot = np.nansum(c["r"][a:b])
        r_trial[a:b] = 1.0 if tot > 0 else 0.0
        nr_trial[a:b] = 1.0 if tot <= 0 else 0.0
    return {"r_trial": r_trial, "nr_trial": nr_trial}


def port_indicators(c):
    return {"rpxr": c["r"] * c["rpx"], "rpxnr": c["nr"] * c["rpx"],
            "lpxr": c["r"] * c["lpx"], "lpxnr": c["nr"] * c["lpx"],
            "rpnr": c["r"] * c["rpn"], "rpnnr": c["nr"] * c["rpn"],
            "lpnr": c["r"] * c["lpn"], "lpnnr": c["nr"] * c["lpn"]}


def side_agnostic(c, p):
    return {"spn": c["rpn"] + c["lpn"], "spx": c["rpx"] + c["lpx"],
            "spnr": p["rpnr"] + p["lpnr"], "spnnr": p["rpnnr"] + p["lpnnr"],
            "spxr": p["rpxr"] + p["lpxr"], "spxnr": p["rpxnr"] + p["lpxnr"],
            "sl": c["rl"] + c["ll"]}


def _first_transitions(x, ntrial):
    """((groupby(nTrial).cumsum() == 1) * 1).diff(), negatives multiplied by False."""
    n = len(x)
    cs = np.full(n, np.nan)
    for a, b in _trial_runs(ntrial):
        acc = 0.0
        for t in range(a, b):
            if not np.isnan(x[t]):
                acc += x[t]
                cs[t] = acc
    eq = (cs == 1.0).astype(np.int64)
    out = np.full(n, np.nan)
    for t in range(1, n):
        d = float(eq[t] - eq[t - 1])
        out[t] = d * float(d >= 0)
    return out


def first_time_events(c, s, ntrial):
    nn = np.nan_to_num(c["lpn"]) + np.nan_to_num(c["rpn"])
    xx = np.nan_to_num(c["lpx"]) + np.nan_to_num(c["rpx"])
    o = {"nn": nn, "xx": xx,
         "ft_nn": _first_transitions(nn, ntrial), "ft_xx": _first_transitions(xx, ntrial),
         "ft_lpn": nn * c["lpn"], "ft_rpn": nn * c["rpn"], "ft_spn": nn * s["spn"],
         "ft_lpx": xx * c["lpx"], "ft_rpx": xx * c["rpx"], "ft_spx": xx * s["spx"],
         "ft_cpn": _first_transitions(c["cpn"], ntrial)}
    for tag, w in (("r", c["r"]), ("nr", c["nr"])):
        for side in ("rpn", "lpn", "spn"):
            o[f"ft_{tag}_{side}"] = o[f"ft_{side}"] * w
    return o


def preprocess_columns(cols, trial_shift_bounds=7):
    """Derived columns of preprocess_lynne for the renamed float64 input columns."""
    c = {k: np.asarray(cols[k], dtype=np.float64) for k in IN_COLS}
    out = trial_starts_ends(c, trial_shift_bounds)
    out.update(reward_flags(c, out["nTrial"]))
    p = port_indicators(c)
    out.update(p)
    s = side_agnostic(c, p)
    out.update(s)
    out.update(first_time_events(c, s, out["nTrial"]))
    return {k: out[k] for k in OUT_COLS}
