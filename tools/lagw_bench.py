"""Standalone timing of the event-structured Gram (sglm_lag_gram_w) on the C4 design, 1, 2 and 5
fits per launch, HIP events around the call (development tool).

python tools/lagw_bench.py                      : median ms per call per fit count
LAGW_ENV=NAME=v1,v2 python tools/lagw_bench.py  : the same for each value of an environment
    switch the library reads per launch (alternating), and whether the variants' H agree
    bitwise with the half-occurrence split off (SGLM_LAGW_SPLIT=0) and to 1e-6 with it on."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sglm_hip import engine as E, synth, _lib  # noqa: E402

N, m, L, K, nlam = bench.CONFIGS["c4"]
s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
lg = E._lagw(d)
name, vals = (os.environ["LAGW_ENV"].split("=") if os.environ.get("LAGW_ENV")
              else ("SGLM_LAGW_NONE", "x"))
vals = vals.split(",")
reps = int(os.environ.get("LAGW_REPS", "6"))
out = {}
for nf in (1, 2, 5):
    fits = torch.arange(nf, dtype=torch.int32, device="cuda")
    W = torch.rand((nf, d.ld), device="cuda")
    H = torch.zeros((nf, d.P, d.P), device="cuda")
    wk = torch.empty(_lib.query("sglm_lag_gram_w_work_bytes", lg.n_raw, lg.K, nf, d.P),
                     dtype=torch.uint8, device="cuda")

    def call():
        _lib.call("sglm_lag_gram_w", lg.R.data_ptr(), lg.w_occ.data_ptr(),
                  lg.w_ev_off.data_ptr(), lg.m, lg.n_raw, lg.shifts.data_ptr(),
                  lg.bidx.data_ptr(), lg.K, lg.smin, lg.smax, lg.layout, lg.row0, lg.n,
                  W.data_ptr(), d.ld, fits.data_ptr(), nf, H.data_ptr(), d.P, d.p,
                  wk.data_ptr(), 0)

    ts = {v: [] for v in vals}
    for rep in range(reps):
        for v in (vals if rep % 2 == 0 else vals[::-1]):
            os.environ[name] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            ts[v].append(e0.elapsed_time(e1))
    for v in vals:
        out[f"nf{nf}_{name}={v}"] = round(float(np.median(ts[v][1:])), 3)
    if len(vals) > 1:
        up = torch.triu(torch.ones(d.P, d.P, dtype=torch.bool, device="cuda"))
        for split in ("0", "1"):
            os.environ["SGLM_LAGW_SPLIT"] = split
            hs = []
            for v in vals:
                os.environ[name] = v
                H.zero_()
                call()
                torch.cuda.synchronize()
                hs.append(H[:, up].clone())
            ok = all(torch.equal(hs[0], h) for h in hs[1:]) if split == "0" else all(
                float((hs[0] - h).abs().max() / hs[0].abs().max()) < 1e-6 for h in hs[1:])
            out[f"nf{nf}_H_{'bitwise' if split == '0' else 'close'}_split{split}"] = bool(ok)
        os.environ.pop("SGLM_LAGW_SPLIT", None)
    print(json.dumps({k: v for k, v in out.items() if k.startswith(f"nf{nf}_")}), flush=True)
print(json.dumps(out))
