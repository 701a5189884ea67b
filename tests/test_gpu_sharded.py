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


@pytest.mark.parametrize("world,rank", [(4, 1), (8, 7)])
def test_row_slab_replay_follows_the_recorded_trajectory(engine, world, rank):
    """The row-sharded timing simulation (comm.SimComm, tools/rank_sim.py --mode rows): one
    rank's slab, fed the global sums of a recording of the unsharded grid and factoring only
    its round-robin share of the new factorisations (the other fits' directions replayed),
    must reproduce the recording bitwise -- the factor + inverse chain and the explicit-inverse
    solve of a fit do not depend on which other fits share the launch, and every host decision
    sees the recorded values.  Also pins the slab problem: masks cut to the slab, global
    counts."""
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.comm import SimComm, row_slab
    from sglm_hip.estimators import Objective
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    slab = row_slab(s.N, rank, world)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, slab=slab)
    assert d.slab == (slab[0], slab[1], s.N) and d.n == slab[1] - slab[0]
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100)
            for a in np.logspace(-4, 1, 20)]
    rolls = [0] * len(objs)
    prob = E.Problem.from_index_lists(d, s.y, [0], [(cv_idx[0][0], True), (None, False)])
    m0 = np.zeros(s.N, np.uint8)
    np.add.at(m0, cv_idx[0][0], 1)
    assert np.array_equal(prob.M[0, :d.n].cpu().numpy(), m0[slab[0]:slab[1]])
    assert int(prob.M[:, d.n:].sum()) == 0
    assert prob.mask_nnz(0) == np.count_nonzero(m0[slab[0]:slab[1]])
    assert prob.mask_count(0) == float(m0.sum()) and prob.mask_count(1) == float(s.N)
    assert np.array_equal(prob.Y[0, :d.n].cpu().numpy(), s.y[slab[0]:slab[1]].astype(np.float32))
    rec = SimComm.recorder()
    full = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    a = grid.run(full, s.y, cv_idx, objs, rolls, simulate=rec)
    assert len(rec.tape) > 0
    rp = rec.replay(rank, world)
    b = grid.run(d, s.y, cv_idx, objs, rolls, simulate=rp)
    assert rp._k == len(rec.tape)
    assert sorted(a) == sorted(b) == list(range(len(objs) * 6))
    for i in a:
        assert np.array_equal(a[i][0], b[i][0]) and a[i][1] == b[i][1] and a[i][2] == b[i][2]


def test_slab_multiplicity_sums_stay_local(engine):
    """A resampled fold list (rows with multiplicity 2, others missing) whose GLOBAL count
    equals the row count and whose slab rows are all present: the slab's own multiplicity sum
    differs from its row count, so the constant-weight (all-rows) first Gram is not taken on
    that slab (engine.irls ``mall``; min-reduced over the ranks in a row-sharded solve)."""
    from sglm_hip import engine as E, synth
    from sglm_hip.comm import row_slab
    s = synth.make(N=20_000, m=5, L=4, family="poisson", rho=0.05, seed=2)
    world, rank = 4, 1
    slab = row_slab(s.N, rank, world)
    nxt = row_slab(s.N, rank + 1, world)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, slab=slab)
    idx = np.sort(np.r_[np.setdiff1d(np.arange(s.N), [nxt[0]]), slab[0]])   # one dup, one gap
    prob = E.Problem.from_index_lists(d, s.y, [0], [(idx, True), (None, False)])
    assert prob.mask_count(0) == float(s.N) and prob.mask_nnz(0) == d.n
    assert prob.mask_local_count(0) == float(d.n + 1)
    assert prob.mask_local_count(1) == float(d.n)
