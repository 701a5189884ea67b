set -e
O=gpurun_out/hp; mkdir -p $O
timeout -k 10 300 python - > $O/prof.txt 2>&1 <<'PY'
import sys, os, time, cProfile, pstats
sys.path[:0] = ['.', 'sabatinilab-glm_amd']
import numpy as np, pandas as pd, torch
import bench
from sglm_hip import engine as E, folds, grid, synth
from sglm_hip.estimators import Objective
N, m, L, K, nlam = bench.CONFIGS['c4']
s = synth.make(N=N, m=m, L=L, family='poisson', rho=0.02, seed=0)
d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
codes = folds.trial_keys_codes(pd.DataFrame({'nTrial': s.trial}), ['nTrial']).values
np.random.seed(3)
cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
objs = [Objective('irls', E.FAM_TWEEDIE_LOG, 1.0, float(al), 'n', True, 100) for al in np.logspace(-4, 1, nlam)]
for _ in range(3): grid.run(d, s.y, cv_idx, objs, [0]*nlam)
torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
t0 = time.perf_counter(); grid.run(d, s.y, cv_idx, objs, [0]*nlam); torch.cuda.synchronize()
print('wall', time.perf_counter() - t0)
pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(30)
PY
