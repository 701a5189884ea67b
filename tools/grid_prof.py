"""Host profile (cProfile) of one C4 CV grid after warm-up (development tool): where the host
spends the grid, incl. the synchronisation waits.  Usage on the box: python tools/grid_prof.py"""
import cProfile
import os
import pstats
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
    N, m, L, K, nlam = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    for _ in range(4):
        grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    torch.cuda.synchronize()
    t = time.perf_counter()
    grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    torch.cuda.synchronize()
    print(f"grid {1e3 * (time.perf_counter() - t):.1f} ms")
    pr = cProfile.Profile()
    pr.enable()
    grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(50)


if __name__ == "__main__":
    main()
