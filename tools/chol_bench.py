"""Factorisation + explicit-inverse chain (sglm_chol_solve_inv, factor only) at the C4 size
(development tool): P = 2048, p = 2000, n representatives per call as the IRLS forms them.

python tools/chol_bench.py [--n 1 3] [--reps 20] : prints JSON {n: ms per call} timed with HIP
events on the launch stream (H restored from a copy before each call, outside the events), and
the host time of the call itself (the captured graph's launch).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1, 3])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--P", type=int, default=2048)
    ap.add_argument("--p", type=int, default=2000)
    ap.add_argument("--env", default=None,
                    help="NAME=v1,v2: time each value of an environment switch (alternating)")
    a = ap.parse_args()
    if a.env:
        name, vals = a.env.split("=")
        res = {}
        for r in range(3):
            for v in vals.split(","):
                os.environ[name] = v
                res.setdefault(v, []).append(run(a))
        print(json.dumps({v: {n: float(np.median([x[n]["ms_median"] for x in rs]))
                              for n in a.n} for v, rs in res.items()}))
        return
    print(json.dumps(run(a)))


def run(a):
    import torch
    from sglm_hip import _lib
    P, p = a.P, a.p
    rng = np.random.default_rng(0)
    out = {}
    for n in a.n:
        H = np.zeros((n, P, P), np.float32)
        for k in range(n):
            A = rng.normal(size=(p + 400, p + 1)).astype(np.float32)
            H[k, : p + 1, : p + 1] = A.T @ A / 100.0
        H0 = torch.from_numpy(H).cuda()
        Hd = torch.empty_like(H0)
        Md = torch.empty_like(H0)
        dsh = np.full((n, P), -1.0, np.float32)
        dsh[:, :p] = 0.5
        dsh[:, p] = 0.0
        dshd = torch.from_numpy(dsh).cuda()
        delta = torch.zeros((n, P), dtype=torch.float32, device="cuda")
        info = torch.zeros(n, dtype=torch.int32, device="cuda")
        frozen = torch.zeros((n, P), dtype=torch.uint8, device="cuda")
        cw = torch.empty(_lib.query("sglm_chol_work_bytes", P, n), dtype=torch.uint8,
                         device="cuda")
        fits = torch.arange(n, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        times, host = [], []
        for rep in range(a.reps + 3):
            Hd.copy_(H0)
            info.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            h0 = time.perf_counter()
            _lib.call("sglm_chol_solve_inv", Hd.data_ptr(), Md.data_ptr(), P, fits.data_ptr(),
                      None, None, n, n, None, 0, None, dshd.data_ptr(), delta.data_ptr(),
                      info.data_ptr(), frozen.data_ptr(), n, cw.data_ptr(), st)
            h1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            if rep >= 3:
                times.append(e0.elapsed_time(e1))
                host.append((h1 - h0) * 1e3)
        # accuracy of the inverse: |U M - I| on the free block of fit 0
        U = np.triu(Hd[0].cpu().numpy()[: p + 1, : p + 1].astype(np.float64))
        M = np.triu(Md[0].cpu().numpy()[: p + 1, : p + 1].astype(np.float64))
        err = float(np.abs(U @ M - np.eye(p + 1)).max())
        out[n] = {"ms_median": float(np.median(times)), "ms_min": float(np.min(times)),
                  "host_ms_median": float(np.median(host)),
                  "inv_err": err, "dropped": int(info.sum().item())}
    return out


if __name__ == "__main__":
    main()
