"""Probe the C5 multi-response elastic-net CV path at C4 scale (development tool).

python tools/c5_probe.py --responses 4 --alphas 20 : wall time, CD sweeps, phase split.
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
    ap.add_argument("--responses", type=int, default=4)
    ap.add_argument("--alphas", type=int, default=20)
    ap.add_argument("--rows", type=int, default=1_000_000)
    a = ap.parse_args()
    import pandas as pd
    import torch
    from sglm_hip import engine as E, enet, folds, synth
    s = synth.make(N=a.rows, m=50, L=20, family="gaussian", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(5)
    Y = np.stack([s.y + rng.normal(0, 1, s.N) for _ in range(a.responses)], 1)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    alphas = np.logspace(-4, 1, a.alphas)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = {}
    out = enet.cv_enet_path(d, Y, cv_idx, alphas, l1_ratio=0.5, stats=st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    nz = [int(np.sum(np.abs(out[0][j]["refit_coef"]) > 0)) for j in range(a.alphas)]
    print(json.dumps({"wall_s": dt, "stats": st, "fits_per_s": st["fits"] / dt,
                      "nonzeros_refit_r0": nz,
                      "sweeps_r0": [out[0][j]["n_iter"] for j in range(a.alphas)]}))


if __name__ == "__main__":
    main()
