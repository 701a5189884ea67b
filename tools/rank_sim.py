"""Per-rank cost of an N-GPU C4 grid, simulated on one GPU (development tool).

python tools/rank_sim.py --world 8 [--rank R | --all] [--plan mask_major|round_robin] :
solves one rank's share of the C4 grid (grid.shard_plan) after a warm-up, with device syncs
at phase boundaries, and prints the phase breakdown; --all times every rank and reports the
max over ranks (what an N-GPU grid's wall-clock follows).

--mode rows: the row-sharded grid (sglm_hip/comm.py).  One recording of the unsharded grid
keeps every collective's global value and every iteration's directions (SimComm.recorder);
each rank's slab design is then expanded alone and timed replaying it: the slab's own work,
its share of the factorisations, the collectives' results copied in.  The collectives are
NOT timed (no process group): their count and bytes per grid are reported.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--plan", default="mask_major")
    ap.add_argument("--mode", default="fits", choices=["fits", "rows"])
    a = ap.parse_args()
    import bench
    import pandas as pd
    import torch
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    N, m, L, K, nlam = bench.CONFIGS[a.config]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    grid.SHARD_PLAN = a.plan
    if a.mode == "rows":
        from sglm_hip.comm import SimComm, row_slab
        import gc
        rec = SimComm.recorder()
        grid.run(d, s.y, cv_idx, objs, [0] * nlam, simulate=rec)
        del d
        gc.collect()
        torch.cuda.empty_cache()
        per = []
        ranks = list(range(a.world)) if a.all else [a.rank]
        for r in ranks:
            dr = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N,
                                      slab=row_slab(s.N, r, a.world))
            for _ in range(int(os.environ.get("SIM_WARMUPS", "2"))):
                grid.run(dr, s.y, cv_idx, objs, [0] * nlam, simulate=rec.replay(r, a.world))
            gc.collect()
            st = E.IrlsStats(record=True)
            rp = rec.replay(r, a.world)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = grid.run(dr, s.y, cv_idx, objs, [0] * nlam, stats=st, simulate=rp)
            torch.cuda.synchronize()
            per.append({"rank": r, "rows": list(dr.slab), "wall_ms": round(
                (time.perf_counter() - t0) * 1e3, 2), "fits": len(res),
                "fit_iters": st.fit_iters, "newton_iters": st.newton_iters,
                "gram_fits": st.gram_fits, "gram_ms": round(sum(
                    e0.elapsed_time(e1) for e0, e1, _, _ in st.syrk_events), 2),
                "collectives": rp.calls, "collective_mb": round(rp.bytes / 2 ** 20, 1)})
            if r == ranks[0] and os.environ.get("SIM_CPROFILE"):
                import cProfile
                import pstats
                prof = cProfile.Profile()
                prof.enable()
                grid.run(dr, s.y, cv_idx, objs, [0] * nlam, simulate=rec.replay(r, a.world))
                torch.cuda.synchronize()
                prof.disable()
                ps = pstats.Stats(prof, stream=sys.stderr)
                ps.sort_stats("tottime").print_stats(45)
                ps.sort_stats("cumulative").print_stats(60)
            if r == ranks[0]:
                # phase breakdown of the first rank (device syncs at phase boundaries)
                st = E.IrlsStats(record=True, trace_phases=True)
                grid.run(dr, s.y, cv_idx, objs, [0] * nlam, stats=st,
                         simulate=rec.replay(r, a.world))
                per[-1]["phases_ms"] = {k: round(v * 1e3, 2) for k, v in st.phases.items()}
            del dr
            gc.collect()
            torch.cuda.empty_cache()
        print(json.dumps({"mode": "rows", "world": a.world, "per_rank": per,
                          "max_ms": max(q["wall_ms"] for q in per),
                          "note": "collectives not timed (one GPU, no process group)"}))
        return
    if a.all:
        per = []
        import gc
        for r in range(a.world):
            sim = (r, a.world)
            for _ in range(int(os.environ.get("SIM_WARMUPS", "2"))):
                grid.run(d, s.y, cv_idx, objs, [0] * nlam, simulate=sim)
            if os.environ.get("SIM_GC_FREEZE", "1") == "1":
                gc.collect()
                gc.freeze()
            # median of SIM_REPEATS timed runs: one run picks up host jitter of ~2 ms
            reps = []
            for _ in range(int(os.environ.get("SIM_REPEATS", "3"))):
                st = E.IrlsStats(record=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st, simulate=sim)
                torch.cuda.synchronize()
                reps.append(round((time.perf_counter() - t0) * 1e3, 2))
            per.append({"rank": r, "wall_ms": float(np.median(reps)), "repeats_ms": reps,
                        "fits": len(res), "fit_iters": st.fit_iters, "gram_fits": st.gram_fits})
        print(json.dumps({"plan": a.plan, "world": a.world, "per_rank": per,
                          "max_ms": max(q["wall_ms"] for q in per),
                          "wall_ms": "median per rank over SIM_REPEATS timed runs"}))
        return
    sim = (a.rank, a.world)
    for _ in range(int(os.environ.get("SIM_WARMUPS", "2"))):
        grid.run(d, s.y, cv_idx, objs, [0] * nlam, simulate=sim)
    import gc
    if os.environ.get("SIM_GC_FREEZE", "1") == "1":
        gc.collect()
        gc.freeze()                  # long-lived objects out of the collector's scans
    out = {"plain_repeats_ms": []}
    for rep in range(3):
        prof = None
        if rep == 0 and os.environ.get("SIM_CPROFILE"):
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        grid.run(d, s.y, cv_idx, objs, [0] * nlam, simulate=sim)
        torch.cuda.synchronize()
        out["plain_repeats_ms"].append(round((time.perf_counter() - t0) * 1e3, 2))
        if prof is not None:
            import pstats
            prof.disable()
            ps = pstats.Stats(prof, stream=sys.stderr)
            ps.sort_stats("tottime").print_stats(40)
            ps.sort_stats("cumulative").print_stats(50)
    st = E.IrlsStats(record=True, host_phases=True)
    grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st, simulate=sim)
    torch.cuda.synchronize()
    out["host_phases_ms"] = {k: round(v * 1e3, 2) for k, v in st.phases.items()}
    out["host_sync_wait_ms"] = round(st.sync_wait_s * 1e3, 2)
    for phases in (False, True):
        st = E.IrlsStats(record=True, trace_phases=phases)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st, simulate=sim)
        torch.cuda.synchronize()
        key = "traced" if phases else "plain"
        out[key] = {"wall_ms": (time.perf_counter() - t0) * 1e3, "fit_iters": st.fit_iters,
                    "gram_fits": st.gram_fits,
                    "gram_ms": [round(e0.elapsed_time(e1), 2) for e0, e1, _, _ in st.syrk_events]}
        if phases:
            out[key]["phases_ms"] = {k: round(v * 1e3, 2) for k, v in st.phases.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
