"""Host (enqueue) time per phase of one C4 grid, no device syncs (development tool)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import pandas as pd
    import torch
    import bench
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    N, m, L, K, nlam = bench.CONFIGS["c4"]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    for _ in range(3):
        grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    for rep in range(3):
        st = E.IrlsStats(host_phases=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"wall_ms": round(wall, 2),
                          "host_phases_ms": {k: round(v * 1e3, 2) for k, v in st.phases.items()},
                          "sync_wait_ms": round(st.sync_wait_s * 1e3, 2)}))


if __name__ == "__main__":
    main()
