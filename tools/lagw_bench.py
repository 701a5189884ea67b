"""Standalone timing of the event-structured Gram (sglm_lag_gram_w) on the C4 design, 1 and 5
fits per launch, HIP events around the call (development tool): python tools/lagw_bench.py"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]
import numpy as np, torch
import bench
from sglm_hip import engine as E, synth, _lib
N, m, L, K, nlam = bench.CONFIGS["c4"]
s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
lg = E._lagw(d)
out = {}
for nf in (1, 5):
    fits = torch.arange(nf, dtype=torch.int32, device="cuda")
    W = torch.rand((nf, d.ld), device="cuda")
    H = torch.zeros((nf, d.P, d.P), device="cuda")
    wk = torch.empty(_lib.query("sglm_lag_gram_w_work_bytes", lg.n_raw, lg.K, nf, d.P), dtype=torch.uint8, device="cuda")
    probes = [int(x) for x in os.environ.get("LAGW_PROBES", "0").split(",")]
    for pr in probes:
        os.environ["SGLM_LAGW_PROBE"] = str(pr)
        ts = []
        for rep in range(int(os.environ.get('LAGW_REPS', '4'))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _lib.call("sglm_lag_gram_w", lg.R.data_ptr(), lg.occ.data_ptr(), lg.ev_off.data_ptr(), lg.m,
                      lg.n_raw, lg.shifts.data_ptr(), lg.bidx.data_ptr(), lg.K, lg.smin, lg.smax,
                      lg.layout, lg.row0, lg.n, W.data_ptr(), d.ld, fits.data_ptr(), nf,
                      H.data_ptr(), d.P, d.p, wk.data_ptr(), 0)
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[f"nf{nf}_probe{pr}"] = round(float(np.median(ts[1:])), 3)
        print(f"nf{nf}_probe{pr}", out[f"nf{nf}_probe{pr}"], flush=True)
print(json.dumps(out))
