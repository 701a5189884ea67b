"""The sharded CV grid in a REAL process group on the GPU.

Two rank processes are started by torch.distributed.run (127.0.0.1 rendezvous) as children
of this test -- no rank touches the GPU before its process group exists -- and both run on
cuda:0 over gloo (a one-GPU rehearsal of the N-GPU run: the same product path as nccl, only
the transport differs; tests/dist_grid_worker.py).  Each rank solves its share of the C3-shape
grid (Poisson 100k x 500, 5 splits x 20 lambdas + refits) on the device; grid.run's
merge_results all-gathers the per-fit results and assembles the reference's per-parameter
dicts (backend/sglm_cv.py:188-200).  Rank 0's assembled grid must equal the unsharded grid
solved in this process to 1e-5 relative, with every fit solved on exactly one rank.

Row-sharded mode (opt-in, SGLM_SHARD=rows; the default shards by fits, sglm_hip/grid.py
SHARD_MODE, and sglm_hip/comm.py): each rank expands only its slab of
the rows and runs every fit on it; Grams, gradients, trial losses, scores and mask statistics
are all-reduced and the new factorisations dealt over the ranks.  Same bar against the
unsharded grid."""
import os
import socket
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


@pytest.mark.parametrize("world,mode", [(2, "fits"), (2, "rows"), (3, "rows")])
def test_process_group_grid_equals_unsharded(engine, tmp_path, world, mode):
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    out = tmp_path / "rank0.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port",
           str(_free_port()), os.path.join(ROOT, "tests", "dist_grid_worker.py"), str(out),
           "gloo", mode]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    got = np.load(out)
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    lams = np.logspace(-4, 1, 20)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100) for a in lams]
    full = grid.run(d, s.y, cv_idx, objs, [0] * len(objs), score_method="r2")
    shares = [got[f"share_{q}"] for q in range(world)]
    assert all(sh.size > 0 for sh in shares)
    if mode == "fits":
        assert sorted(np.concatenate(shares).tolist()) == list(range(120))
    else:
        assert all(sorted(sh.tolist()) == list(range(120)) for sh in shares)
    for j, b in enumerate(full):
        assert bool(got[f"{j}_conv"]) and b["converged"]
        assert rel(got[f"{j}_cv_coefs"], b["cv_coefs"]) < 1e-5, j
        assert rel(got[f"{j}_cv_intercepts"], b["cv_intercepts"]) < 1e-5, j
        assert rel(got[f"{j}_refit_coef"], b["refit_coef"]) < 1e-5, j
        assert np.max(np.abs(got[f"{j}_cv_scores_test"] - b["cv_scores_test"])) < 1e-6
        assert abs(float(got[f"{j}_r2"]) - b["cv_R2_score"]) < 1e-6
