"""Per-Newton-iteration log of the C4 grid (development tool): active fits, kept / aliased /
formed Hessians, stops, step sizes and per-fit contraction rates of the fits that continue.
python tools/iter_log.py [config]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import pandas as pd
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
    st = E.IrlsStats(iter_log=[])
    grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st)
    for row in st.iter_log:
        print(json.dumps(row))
    print(json.dumps({k: v for k, v in st.stops.items()}))


if __name__ == "__main__":
    main()
