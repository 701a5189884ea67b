"""The Gram launches of one C4 grid (development tool): per launch the fits, distinct row masks,
split-K factor, rows, time and algorithmic TFLOP/s.  Usage on the box: python tools/gram_launches.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    import bench
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    N, m, L, K, nlam = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    design = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    import pandas as pd
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    for _ in range(3):
        grid.run(design, s.y, cv_idx, objs, [0] * nlam)
    for rep in range(2):
        E.GRAM_LOG = []
        st = E.IrlsStats(record=True)
        grid.run(design, s.y, cv_idx, objs, [0] * nlam, stats=st)
        torch.cuda.synchronize()
        for (nact, nm, sp, rows), (e0, e1, _, fl) in zip(E.GRAM_LOG, st.syrk_events):
            ms = e0.elapsed_time(e1)
            print(json.dumps({"rep": rep, "fits": nact, "masks": nm, "splits": sp, "rows": rows,
                              "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
