"""Second CPU formulation of lynne_pp.preprocess_lynne (lynne_pp.py:217-249) in pandas
Series operations — TEST INFRASTRUCTURE (tests/ and bench.py's cpu_baseline leg only).  It pins oracle/prep_ref.py (explicit row walks) to
pandas' own semantics of the operations the reference uses: Series.shift on a bool series
(NaN at the ends), bfill / ffill, NaN-skipping cumsum, groupby(...).transform('sum') and
groupby(...).cumsum() with NaN keys dropped, DataFrame.diff and the multiply-by-bool clamp.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

def derived_columns(c: dict, k: int) -> dict:
    """c: short name -> float64 array; returns derived name -> float64 array."""
    s = {name: pd.Series(np.asarray(v, dtype=np.float64)) for name, v in c.items()}
    nz = lambda x, f: x.mask(x == 0) * f                         # noqa: E731
    ev = nz(s["cpn"], 1.0).combine_first(nz(s["lpx"], 2.0)).combine_first(nz(s["rpx"], 2.0))
    ev = ev.bfill()
    start = (((ev == 1.0) & (ev.shift(-1) != 1.0)).shift(-k) * 1.0).astype(float)
    ntrial = start.cumsum()
    ece = nz(s["lpx"], 2.0).combine_first(nz(s["rpx"], 2.0)).combine_first(
        start.mask(start == 0.0)).ffill()
    end = (((ece == 2.0) & (ece.shift(1) != 2.0) & (ntrial > 0)).shift(k) * 1.0).astype(float)
    o = {"event_col": ev, "trial_start_flag": start, "nTrial": ntrial, "event_col_end": ece,
         "trial_end_flag": end, "nEndTrial": end.cumsum()}
    frame = pd.DataFrame({"nTrial": ntrial, "r": s["r"]})
    tot = frame.groupby("nTrial")["r"].transform("sum")
    o["r_trial"] = (tot > 0) * 1.0
    o["nr_trial"] = (tot <= 0) * 1.0
    for side in ("rpx", "lpx", "rpn", "lpn"):
        o[f"{side}r"] = s["r"] * s[side]
        o[f"{side}nr"] = s["nr"] * s[side]
    o["spn"], o["spx"] = s["rpn"] + s["lpn"], s["rpx"] + s["lpx"]
    for tag in ("nr", "nnr", "xr", "xnr"):
        o[f"sp{tag}"] = o[f"rp{tag}"] + o[f"lp{tag}"]
    o["sl"] = s["rl"] + s["ll"]
    both = pd.DataFrame({k2: s[k2] for k2 in ("lpn", "rpn", "lpx", "rpx")})
    o["nn"] = both[["lpn", "rpn"]].sum(axis=1)
    o["xx"] = both[["lpx", "rpx"]].sum(axis=1)
    parts = pd.DataFrame({"nTrial": ntrial, "nn": o["nn"], "xx": o["xx"], "cpn": s["cpn"]})
    cs = parts.groupby("nTrial")[["nn", "xx", "cpn"]].cumsum()
    steps = ((cs == 1) * 1).diff()
    steps = steps * (steps >= 0)
    for name in ("nn", "xx", "cpn"):
        o[f"ft_{name}"] = steps[name]
    o["ft_lpn"], o["ft_rpn"], o["ft_spn"] = o["nn"] * s["lpn"], o["nn"] * s["rpn"], o["nn"] * o["spn"]
    o["ft_lpx"], o["ft_rpx"], o["ft_spx"] = o["xx"] * s["lpx"], o["xx"] * s["rpx"], o["xx"] * o["spx"]
    for tag in ("r", "nr"):
        for side in ("rpn", "lpn", "spn"):
            o[f"ft_{tag}_{side}"] = o[f"ft_{side}"] * s[tag]
    return {name: np.asarray(v, dtype=np.float64) for name, v in o.items()}
