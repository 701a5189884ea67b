"""Host/device phase breakdown of one C4 CV grid (development tool).

python tools/grid_phases.py [--config c4] : runs a warm-up grid, then one grid with a device
sync at every phase boundary and per-iteration IRLS phase timers, and prints JSON.
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
    ap.add_argument("--config", default="c4")
    a = ap.parse_args()
    import bench
    import pandas as pd
    import torch
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    N, m, L, K, nlam = bench.CONFIGS[a.config]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    st = E.IrlsStats(record=True, trace_phases=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(json.dumps({"wall_ms": wall * 1e3,
                      "phases_ms": {k: round(v * 1e3, 2) for k, v in st.phases.items()},
                      "fit_iters": st.fit_iters, "newton_iters": st.newton_iters}))


if __name__ == "__main__":
    main()
