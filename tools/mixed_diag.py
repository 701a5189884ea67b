"""Diagnostic: Poisson CV grid on the mixed golden design, engine knobs varied via env."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "sabatinilab-glm_amd"),
                os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..")]
import numpy as np
from test_oracle_golden import mixed_design
from oracle import glm_ref
from sglm_hip import grid, engine as E, folds as F
from sglm_hip.estimators import Objective
import pandas as pd

g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "mixed.npz"))
X = mixed_design(g)
y = g["mxpois_y"]
np.random.seed(30186)
codes = F.trial_keys_codes(pd.DataFrame({"nTrial": g["mx_trial"]}), ["nTrial"]).values
cv = F.cv_idx_from_bucket_ids(codes, num_folds=3, test_size=0.2)
obj = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, 1e-4, "n", False, 100)]
mode = sys.argv[1] if len(sys.argv) > 1 else "host"
if mode == "xonly":            # the 0/1 part only (continuous columns dropped)
    keep = np.setdiff1d(np.arange(X.shape[1]), g["mx_cpos"])
    X = X[:, keep]
st = E.IrlsStats()
r = grid.run(X, y, cv, obj, [0], stats=st)[0]
print("stops", st.stops, "newton", st.newton_iters)
print("converged", r["converged"], "n_iter", r["n_iter"])
for k, (tr, te) in enumerate(cv):
    c, _ = glm_ref.fit_tweedie_newton(X[tr], y[tr], 1e-4, 1.0, fit_intercept=False)
    e = np.max(np.abs(r["cv_coefs"][:, k] - c)) / np.max(np.abs(c))
    print("fold", k, "rel", e)
c, _ = glm_ref.fit_tweedie_newton(X, y, 1e-4, 1.0, fit_intercept=False)
print("refit rel", np.max(np.abs(r["refit_coef"] - c)) / np.max(np.abs(c)))
