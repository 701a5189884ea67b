"""One rank of a real multi-process sharded CV grid on the GPU (run by torch.distributed.run
from tests/test_gpu_dist.py; not collected by pytest).

Every rank: the C3-shape design (Poisson 100k x 500, 5 trial-id splits, 20 lambdas) built
from the same seeds, ``grid.run`` inside an initialised process group -- so the product's
own path runs: rank_share -> the rank's batched IRLS on the device -> the y-range all-reduce
-> grid.merge_results (all_gather_object) -> assemble.  Rank 0 writes the assembled result to
argv[1] (npz).  All ranks may share one GPU (rehearsal of the N-GPU run on one card).
argv[3] = "fits" (whole fits per rank, full design on every rank) or "rows" (every rank
expands only its row slab and runs every fit on it; sums over rows all-reduced, comm.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402


def main():
    out_path, backend = sys.argv[1], sys.argv[2]
    mode = sys.argv[3] if len(sys.argv) > 3 else "fits"
    import torch
    import torch.distributed as dist
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local % torch.cuda.device_count())
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group("gloo")
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    grid.SHARD_MODE = mode
    s = synth.make(N=100_000, m=25, L=10, family="poisson", rho=0.02, seed=0)
    slab = grid.rank_slab(s.N) if mode == "rows" else None
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, slab=slab)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=5)
    lams = np.logspace(-4, 1, 20)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(a), "n", True, 100) for a in lams]
    groups = [{"cv_idx": cv_idx, "objectives": objs, "rolls": [0] * len(objs)}]
    plan = grid.plan_fits(groups, s.N)
    mine = (list(range(len(plan[3]))) if mode == "rows"
            else grid.rank_share(plan, groups, dist.get_rank(), dist.get_world_size()))
    res = grid.run(d, s.y, cv_idx, objs, [0] * len(objs), score_method="r2")
    shares = [None] * dist.get_world_size()
    dist.all_gather_object(shares, mine)
    if dist.get_rank() == 0:
        arr = {}
        for j, r in enumerate(res):
            for key in ("cv_coefs", "cv_intercepts", "cv_scores_test", "cv_scores_train",
                        "refit_coef"):
                arr[f"{j}_{key}"] = np.asarray(r[key])
            arr[f"{j}_r2"] = np.float64(r["cv_R2_score"])
            arr[f"{j}_conv"] = np.bool_(r["converged"])
        for q, m in enumerate(shares):
            arr[f"share_{q}"] = np.asarray(m, dtype=np.int64)
        np.savez(out_path, **arr)
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
