"""Explicit-walk restatement of pp_design_mat.make_design_mat -- TEST INFRASTRUCTURE ONLY.

Column arithmetic of /root/reference/pp_design_mat.py:6-205 written as plain row loops and
per-trial dictionaries (no pandas groupby), float64 numpy columns in, a dict of float64
columns out.  Pinned to the pandas formulation (oracle/designmat_pandas.py) by
tests/test_designmat_cpu.py on synthetic sessions with NaN trial ids, trials without cues,
unmapped trial ids, licks before/after bouts and repeated nth positions.  Pure-Python loops:
small sessions only (<= ~50k rows).

Semantics restated (pandas' own, on a float key):
* groupby('nTrial') drops rows whose key is NaN; a group is every row with an equal key,
  wherever it sits; cumcount numbers a group's rows in row order from 0 (:171-172);
* groupby(...).nth(k) picks the k-th row of a group (k < 0 counts from the end) (:52-53, 175);
* groupby(...)['c'].first() is the first NON-NULL value of c in the group (:114, 117);
* Series.map(mapper) is NaN for keys absent from the mapper, and for NaN keys (:93, 112, 192).
"""
from __future__ import annotations

import math
import re

import numpy as np

ENL_SCALE = 5000.0
MS_PER_ROW = 20.0


def _isnan(v):
    return isinstance(v, float) and math.isnan(v)


def _key(v):
    return None if _isnan(v) else float(v)


def _groups(keys):
    """{key: [rows in order]} of the non-NaN keys (a tuple key is NaN if any part is)."""
    out = {}
    for i, k in enumerate(keys):
        if any(_isnan(x) for x in (k if isinstance(k, tuple) else (k,))):
            continue
        out.setdefault(k, []).append(i)
    return out


def _nth(rows, k):
    if k >= 0:
        return rows[k] if k < len(rows) else None
    return rows[len(rows) + k] if -k <= len(rows) else None


def _map(nt, table):
    """Series.map: per row the table value of its key, NaN when absent or the key is NaN."""
    return np.array([table.get(_key(v), np.nan) if not _isnan(v) else np.nan
                     for v in nt.tolist()], dtype=np.float64)


def design_columns(cols, trial_cols, states=("Select", "Consumption", "ENLP"), nth_licks=(1,),
                   interactions=None, photo=()):
    """cols: dict of float64 row columns (nTrial, nENL, iBlock, iSpout, Cue, ENL, state_ENLP,
    Consumption, stateConsumption, trial_clock, the states, photometry); trial_cols: dict of
    float64 trial columns with 'nTrial' and the mapped ones (NaN = missing).  Returns
    (ordered list of column names, dict name -> float64 column)."""
    n = len(cols["nTrial"])
    nt = np.asarray(cols["nTrial"], dtype=np.float64)
    tkeys = [float(v) for v in trial_cols["nTrial"]]

    def table(name):
        return {k: float(v) for k, v in zip(tkeys, trial_cols[name])}

    # add_heatmap_columns (:108-126)
    clock = cols["trial_clock"]
    g_all = _groups(nt.tolist())

    def first_clock(flagcol):
        out = {}
        for k, rows in g_all.items():
            vals = [clock[i] for i in rows if cols[flagcol][i] == 1 and not math.isnan(clock[i])]
            has = any(cols[flagcol][i] == 1 for i in rows)
            if has:
                out[k] = vals[0] if vals else np.nan
        return out
    fc, fcons = first_clock("Cue"), first_clock("Consumption")
    sel_to_cons = {}
    for k, rows in g_all.items():
        s_c = sum(cols["Consumption"][i] for i in rows if not math.isnan(cols["Consumption"][i]))
        s_s = sum(cols["stateConsumption"][i] for i in rows
                  if not math.isnan(cols["stateConsumption"][i]))
        sel_to_cons[k] = (s_s - s_c) * MS_PER_ROW
    hm = {}
    hm["hm_t_cue_offset_to_sel"] = _map(nt, table("tSelection"))
    hm["hm_t_from_cue_onset"] = clock - _map(nt, fc)
    hm["hm_t_from_cons_onset"] = clock - _map(nt, fcons)
    hm["hm_t_sel_to_cons"] = _map(nt, sel_to_cons)
    hm["hm_t_cue_offset_to_cons"] = hm["hm_t_sel_to_cons"] + hm["hm_t_cue_offset_to_sel"]

    # Lick, classify_lick_state (:160-163)
    lick = np.array([0.0 if math.isnan(v) else 1.0 for v in cols["iSpout"]])
    out, names = {}, []
    for s in states:
        nm = f"{s[:3].lower()}_lick"
        if nm not in out:
            names.append(nm)
        out[nm] = np.asarray(cols[s], dtype=np.float64) * lick
    # counters (:167-172)
    t_enl = np.zeros(n)
    t_enlp = np.zeros(n)
    for i in range(n):
        if cols["ENL"][i] == 1 or cols["Cue"][i] == 1:
            t_enl[i] = np.nan
        if cols["state_ENLP"][i] == 1:
            t_enlp[i] = np.nan
    for k, rows in g_all.items():
        c = 0
        for i in rows:
            if cols["ENL"][i] == 1 or cols["Cue"][i] == 1:
                t_enl[i] = float(c * c) / ENL_SCALE
                c += 1
    g2 = _groups(list(zip(nt.tolist(), np.asarray(cols["nENL"], float).tolist())))
    for k, rows in g2.items():
        c = 0
        for i in rows:
            if cols["state_ENLP"][i] == 1:
                t_enlp[i] = float(c * c) / ENL_SCALE
                c += 1
    # cue onsets (:175, 182-183)
    cue = np.zeros(n)
    for k, rows in g_all.items():
        r = [i for i in rows if cols["Cue"][i] == 1]
        if r:
            cue[r[0]] = 1.0
    for nm in ("nTrial", "iBlock"):
        names.append(nm)
        out[nm] = np.asarray(cols[nm], dtype=np.float64)
    names += ["time_from_enl_onset", "time_from_enlp_onset"] + list(photo) + ["cue"]
    out["time_from_enl_onset"], out["time_from_enlp_onset"], out["cue"] = t_enl, t_enlp, cue
    for p in photo:
        out[p] = np.asarray(cols[p], dtype=np.float64)
    # pull_lick_from_bout (:26-58), state 'Consumption', keep_only_nth_lick=True
    bout = "con_lick"
    if bout not in out:
        raise KeyError(bout)
    order = sorted(nth_licks)[::-1] if len(nth_licks) > 1 else list(nth_licks)
    for nth in order:
        nm = f"{bout}_{nth}"
        col = np.zeros(n)
        lk = out[bout]
        picked = []
        for k, rows in g_all.items():
            r = _nth([i for i in rows if lk[i] == 1], nth - 1)
            if r is not None:
                picked.append(r)
        for r in picked:
            col[r] = 1.0
            lk[r] = 0.0
        if nm not in out:
            names.append(nm)
        out[nm] = col
    names.remove(bout)
    del out[bout]
    # interactions (:187-193), event_interactions_dummies (:61-105)
    flag = np.zeros(n)
    if interactions:
        names.append("flag")
    for trial_type, st_ in (interactions or {}).items():
        isna = {k: float(math.isnan(v)) for k, v in zip(tkeys, trial_cols[trial_type])}
        flag = flag + _map(nt, isna)
        pat = "|".join(s.lower()[:3] for s in st_)
        picked = [c for c in names if re.search(pat, c)]
        later = [c for c in names if c not in picked]
        values = sorted({float(v) for v in trial_cols[trial_type] if not math.isnan(v)})
        # get_dummies labels of the convert_dtypes'd column: Int64 when every value is
        # integral ('1'), Float64 otherwise ('1.0', '0.5')
        integral = all(v.is_integer() for v in values)
        new = {}
        new_names = []
        for v in values:
            lab = str(int(v)) if integral else str(v)
            dmy = _map(nt, {k: float(x == v) for k, x in zip(tkeys, trial_cols[trial_type])
                            if not math.isnan(x)} | {k: 0.0 for k, x in
                                                     zip(tkeys, trial_cols[trial_type])
                                                     if math.isnan(x)})
            for c in picked:
                nm = f"{trial_type.lower()[:3]}_{lab}_{c}"
                new_names.append(nm)
                new[nm] = out[c] * dmy
        out.update(new)
        out["flag"] = flag
        for c in picked:
            del out[c]
        names = new_names + later
    if not interactions:
        names.append("flag")
    names += list(hm)
    out.update(hm)
    flag = np.where(np.isnan(flag), flag, np.clip(flag, 0, 1))
    cue_like = [c for c in names if c.endswith("cue")]
    for k, rows in g_all.items():
        tot = 0.0
        for c in cue_like:
            tot += sum(out[c][i] for i in rows if not math.isnan(out[c][i]))
        if tot == 0:
            for i in rows:
                flag[i] = 1.0
    out["flag"] = flag
    return names, out
