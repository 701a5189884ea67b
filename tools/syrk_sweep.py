"""Gram v6 launch-size sweep (development tool): alg TFLOP/s of sglm_syrk_cbits for each
(fits, splits) pair at one mask size, plus the split the engine's heuristic picks."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    from sglm_hip import _lib, engine as E, synth
    rows = int(os.environ.get("SWEEP_ROWS", 1_000_000))
    keep = float(os.environ.get("SWEEP_KEEP", 0.8))
    s = synth.make(N=rows, m=50, L=20, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(1)
    nm = int(os.environ.get("SWEEP_MASKS", 1))       # distinct row masks, dealt to slots k % nm
    ms = [(rng.random(d.n) < keep).astype(np.uint8) for _ in range(nm)]
    prob = E.Problem(d, [np.zeros(d.n)], ms)
    cbs = [prob.compact(i) for i in range(nm)]
    cb = max(cbs, key=lambda c: c[1])
    Bmax = 30
    stride = max(64, (cb[1] + 63) // 64 * 64)
    g = torch.Generator(device="cuda").manual_seed(0)
    W = torch.zeros((Bmax, d.ld), dtype=torch.float32, device="cuda")
    W[:, : d.n] = 0.2 + torch.rand((Bmax, d.n), generator=g, device="cuda")
    wc = torch.zeros(Bmax * stride, dtype=torch.bfloat16, device="cuda")
    fits = torch.arange(Bmax, dtype=torch.int32, device="cuda")
    order = sorted(range(Bmax), key=lambda k: k % nm) if os.environ.get("SWEEP_SORT", "1") == "1" \
        else list(range(Bmax))
    desc = torch.tensor([[cbs[k % nm][0].data_ptr(), cbs[k % nm][1], wc.data_ptr() + 2 * k * stride,
                          0 if cbs[k % nm][2] is None else cbs[k % nm][2].data_ptr()]
                         for k in order], dtype=torch.int64).cuda()
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("sglm_gather_w", W.data_ptr(), d.ld, fits.data_ptr(), Bmax, desc.data_ptr(), cb[1], st)
    H = torch.zeros((Bmax, d.P, d.P), dtype=torch.float32, device="cuda")
    pa = d.p + 1
    nb = d.P // 128
    nsteps = (cb[1] + 63) // 64
    out = {"rows": int(cb[1]), "P": d.P, "p": d.p, "nsteps": nsteps, "masks": nm, "res": []}
    for B in [int(x) for x in os.environ.get("SWEEP_FITS", "1,2,3,4,6,8,12,16,30").split(",")]:
        pick = E.syrk6_splits(nb * (nb + 1) // 2 * B, nsteps, B, d.P)
        row = {"fits": B, "pick": pick, "tf": {}}
        for sp in [int(x) for x in os.environ.get("SWEEP_SPLITS", "1,2,3,4,6,8,12,16,24,32").split(",")]:
            if sp > max(1, nsteps // 8):
                break
            wb = _lib.query("sglm_syrk_work_bytes", d.P, B, sp)
            work = torch.empty(max(wb, 16), dtype=torch.uint8, device="cuda")
            ts = []
            for rep in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.call("sglm_syrk_cbits", desc.data_ptr(), d.P, fits.data_ptr(), B, sp,
                          H.data_ptr(), work.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    ts.append(e0.elapsed_time(e1) / 1e3)
            t = float(np.median(ts))
            row["tf"][sp] = round(B * cb[1] * pa * (pa + 1) / t / 1e12, 1)
            del work
        print(json.dumps(row), flush=True)
        out["res"].append(row)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
