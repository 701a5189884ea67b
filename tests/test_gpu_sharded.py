"""The sharded CV grid on the MI355X: each rank's share solved on the
device exactly as a rank of an N-GPU run solves it (grid.run(..., simulate=(rank, world)):
that rank's masks, responses and fits only), the shares merged and assembled as
grid.merge_results + grid.assemble do after the RCCL all-gather.

Against the unsharded run the merged result must hold every fit once and agree to 1e-5
relative.  Not bitwise: a rank's batch differs from the full batch, so its approximate-
Hessian decisions (reuse, lambda-neighbour sharing, two IRLS groups) take other paths to the
same minimiser, which both runs reach within their stopping tolerance."""
import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


@pytest.mark.parametrize("world", [2, 8])
def test_simulated_rank_shares_merge_to_the_unsharded_grid(engine, world):
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    lams = np.logspace(-4, 1, 20)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100) for a in lams]
    rolls = [0] * len(objs)
    full = grid.run(d, s.y, cv_idx, objs, rolls, score_method="r2")
    groups = [{"cv_idx": cv_idx, "objectives": objs, "rolls": rolls}]
    plan = grid.plan_fits(groups, s.N)
    merged, seen = {}, []
    for r in range(world):
        share = grid.run(d, s.y, cv_idx, objs, rolls, score_method="r2", simulate=(r, world))
        assert sorted(share) == grid.rank_share(plan, groups, r, world)
        seen += list(share)
        merged.update(share)
    assert sorted(seen) == list(range(len(objs) * 6))        # every fit on exactly one rank
    out = grid.assemble(groups, plan, merged, s.p)[0]
    for a, b in zip(out, full):
        assert a["converged"] and b["converged"]
        assert rel(a["cv_coefs"], b["cv_coefs"]) < 1e-5
        assert rel(a["cv_intercepts"], b["cv_intercepts"]) < 1e-5
        assert rel(a["refit_coef"], b["refit_coef"]) < 1e-5
        assert np.max(np.abs(a["cv_scores_test"] - b["cv_scores_test"])) < 1e-6
        assert abs(a["cv_R2_score"] - b["cv_R2_score"]) < 1e-6
