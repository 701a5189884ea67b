"""Where the drop-in NaN-row filter's time goes (development tool, on the box)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]
import bench
import torch
import sglm_ez
from sglm_hip import synth, lagframe
N, m, L, K, nlam = bench.CONFIGS["c4"]
s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
df, ev = bench.dropin_frame(s)
xcols = sglm_ez.add_timeshifts_to_col_list(ev, ev, neg_order=-L, pos_order=L - 1)
orig = lagframe.LagSource.device
T = {}
def timed_device(self, names):
    torch.cuda.synchronize(); t = time.perf_counter()
    r = orig(self, names)
    torch.cuda.synchronize(); T["device"] = T.get("device", 0) + time.perf_counter() - t
    return r
lagframe.LagSource.device = timed_device
orig_up = lagframe.LagSource.upload
def timed_upload(self, names):
    t = time.perf_counter()
    r = orig_up(self, names)
    T["upload"] = T.get("upload", 0) + time.perf_counter() - t
    return r
lagframe.LagSource.upload = timed_upload
orig_lnc = lagframe.LagFrame._lag_nan_counts
def timed_lnc(self, lag, out):
    t = time.perf_counter()
    r = orig_lnc(self, lag, out)
    T["lag_nan_counts"] = T.get("lag_nan_counts", 0) + time.perf_counter() - t
    return r
lagframe.LagFrame._lag_nan_counts = timed_lnc
for rep in range(4):
    T.clear()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    dfrel = sglm_ez.timeshift_cols(df, ev, neg_order=-L, pos_order=L - 1)
    t1 = time.perf_counter()
    sub = dfrel[["nTrial"] + xcols + ["y"]]
    t2 = time.perf_counter()
    na = sub.isna()
    t3 = time.perf_counter()
    cnt = na.sum(axis=1)
    torch.cuda.synchronize(); t4 = time.perf_counter()
    keep = cnt == 0
    t5 = time.perf_counter()
    out = dfrel[keep]
    torch.cuda.synchronize(); t6 = time.perf_counter()
    print({"timeshift": round(1e3*(t1-t0),2), "select": round(1e3*(t2-t1),2), "isna": round(1e3*(t3-t2),2),
           "sum": round(1e3*(t4-t3),2), "cmp": round(1e3*(t5-t4),2), "bool_rows": round(1e3*(t6-t5),2),
           "device_in_sum": round(1e3*T.get("device",0),2), "upload": round(1e3*T.get("upload",0),2),
           "lag_nan_counts": round(1e3*T.get("lag_nan_counts",0),2)})
