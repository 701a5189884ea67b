"""Benchmark: IRLS iterations/s and CV-grid wall-clock on the BASELINE.json north-star config.

Workload (configs[3], the config the metric is quoted on; it fits one MI355X): Poisson/log,
1M rows x 2000 time-shifted predictors (50 Bernoulli(0.02) events x 40 lags, synthetic per
SURVEY.md §8(d)), 5 GroupShuffleSplit splits x 20 lambdas + 20 full refits = 120 fits.
One step = one full CV grid (all 120 fits solved to convergence + scored).  With N ranks
the 120 fits are dealt round-robin (strong scaling: the grid is fixed); results are
all-gathered over RCCL once per grid.

value = fit-iterations (sum over fits of Newton/IRLS iterations, all ranks) / wall time.

Usage: python bench.py [--gpus N --steps K --warmup W] ; N > 1 under torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sabatinilab-glm_amd"))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0          # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    # name: (N rows, events m, L -> lags -L..L-1, n_splits, lambdas)
    "c4": (1_000_000, 50, 20, 5, 20),
    "c3": (100_000, 25, 10, 5, 20),
    "small": (50_000, 10, 5, 5, 4),
    # C5: 64 responses x C4 design, Gaussian elastic-net lambda path (l1_ratio 0.5, 20 alphas)
    "c5": (1_000_000, 50, 20, 5, 20),
    # session preprocessing (lynne_pp.preprocess_lynne): rows per session
    "prep": (16_000_000, 0, 0, 0, 0),
}
C5_RESPONSES = 64
PREP_SHIFT = 1     # er_refactored_from_scratch_cleanup.py:269 calls preprocess_lynne(df, trial_shift_bounds=1)
INIT_PASSES = 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-rows", type=int, default=200_000)
    ap.add_argument("--sklearn-rows", type=int, default=100_000)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for real runs; gloo to rehearse several ranks "
                         "on fewer GPUs")
    return ap.parse_args()


def dense_slice(s, rows):
    m = s.E.shape[1]
    X = np.empty((rows, s.p), dtype=np.float64)
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        X[:, bi * m:(bi + 1) * m] = s.E[r0 - sh:r0 - sh + rows]
    return X


def cpu_baseline(s, n_rows_unit, rows, fit_iters_per_grid, sk_rows):
    """Oracle (float64 numpy/LAPACK damped Newton) on a bounded slice of the same design, plus
    scikit-learn called directly with the estimator the reference selects
    (TweedieRegressor(power=1), backend/sglm.py:112-115): newton-cholesky (IRLS-equivalent)
    and the reference's default lbfgs."""
    from oracle import glm_ref
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    rows = min(rows, s.N)
    X = dense_slice(s, rows)
    y = s.y[:rows]
    t0 = time.perf_counter()
    _, _, iters = glm_ref.fit_tweedie_newton(X, y, 1e-2, 1.0, tol=1e-8, max_iter=50,
                                             return_iters=True)
    dt = time.perf_counter() - t0
    per_iter_unit = dt / max(iters, 1) * (n_rows_unit / rows)
    out = {"value": 1.0 / per_iter_unit, "unit": "IRLS fit-iterations/s (1M-row unit)",
           "cores": int(cores), "kind": "port",
           "sample": f"oracle fp64 damped Newton (numpy/LAPACK), Poisson alpha=1e-2, {rows}x{s.p} "
                     f"slice of the C4 design, {iters} iterations in {dt:.2f} s; per-iteration "
                     f"time scaled x{n_rows_unit / rows:.2f} to 1M rows",
           "grid_wall_s_extrapolated": fit_iters_per_grid * per_iter_unit}
    del X
    try:
        import platform
        from sklearn.linear_model import TweedieRegressor
        sk_rows = min(sk_rows, s.N)
        X = dense_slice(s, sk_rows)
        y = s.y[:sk_rows]
        model = platform.machine()
        try:
            with open("/proc/cpuinfo") as f:
                model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
        except Exception:  # pragma: no cover
            pass
        sk = {"rows": sk_rows, "cpu": model, "nproc": os.cpu_count()}
        for solver in ("newton-cholesky", "lbfgs"):
            m = TweedieRegressor(power=1.0, alpha=1e-2, link="log", solver=solver, tol=1e-4,
                                 max_iter=100)
            t0 = time.perf_counter()
            m.fit(X, y)
            dt = time.perf_counter() - t0
            it = int(m.n_iter_)
            sk[solver] = {"n_iter": it, "fit_s": dt,
                          "fit_s_1M_rows": dt * n_rows_unit / sk_rows,
                          "iters_per_s_1M_rows": it / dt * sk_rows / n_rows_unit}
        out["sklearn_direct"] = sk
    except Exception as e:  # pragma: no cover - sklearn is part of the image
        out["sklearn_direct"] = {"error": repr(e)}
    return out


def pmc_traffic():
    """HBM bytes per Gram launch from the newest committed PMC summary (profiles/*_pmc_traffic.json,
    written by tools/pmc_traffic.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    bench's grid; gfx950 corrections applied there).  PMC counters cannot be read in-process."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    dom = d.get("dominant") or {}
    if "syrk6_kernel" not in dom.get("kernel", ""):
        return None, None
    return dom["traffic_bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def bench_c5(a):
    """64 responses (independent y draws, same X as C4), elastic net
    l1_ratio 0.5 over 20 alphas, 5 splits + refit per (response, alpha) = 7680 fits, scored
    on the splits' test rows.  One rank (the path batches all responses on one GPU)."""
    import pandas as pd
    import torch
    from sglm_hip import engine as E, enet, folds, synth
    N, m, L, K, nlam = CONFIGS["c5"]
    R = C5_RESPONSES
    s = synth.make(N=N, m=m, L=L, family="gaussian", rho=0.02, seed=0)
    design = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    rng = np.random.default_rng(5)
    Y = np.stack([s.y + rng.normal(0, 1, s.N) for _ in range(R)], 1)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    alphas = np.logspace(-4, 1, nlam)
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    for _ in range(a.warmup):
        enet.cv_enet_path(design, Y, cv_idx, alphas, l1_ratio=0.5)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st = {}
        out = enet.cv_enet_path(design, Y, cv_idx, alphas, l1_ratio=0.5, stats=st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = (time.perf_counter() - t0) / a.steps
    fits_total = R * nlam * (K + 1)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64,
                         device="cuda" if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    if rank != 0:
        return
    cpu = None
    if not a.no_cpu and world == 1:
        from sklearn.linear_model import ElasticNet
        rows = min(a.sklearn_rows, s.N)
        X = dense_slice(s, rows)
        t1 = time.perf_counter()
        en = ElasticNet(alpha=float(alphas[nlam // 2]), l1_ratio=0.5, max_iter=1000).fit(X, Y[:rows, 0])
        dt = time.perf_counter() - t1
        per_fit_1m = dt * s.N / rows
        try:
            from threadpoolctl import threadpool_info
            cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
        except Exception:  # pragma: no cover
            cores = int(os.environ.get("OMP_NUM_THREADS", 1))
        cpu = {"value": 1.0 / per_fit_1m, "unit": "elastic-net fits/s (1M-row unit)",
               "cores": int(cores), "kind": "port",
               "sample": f"scikit-learn ElasticNet(alpha={alphas[nlam // 2]:.3g}, l1_ratio=0.5) "
                         f"on a {rows}x{s.p} slice, {en.n_iter_} CD epochs in {dt:.2f} s, "
                         f"scaled x{s.N / rows:.0f} to 1M rows",
               "grid_wall_s_extrapolated": per_fit_1m * fits_total}
    print(json.dumps({
        "metric": "elastic-net CV lambda-path fits/s (C5: 64 responses x 1M x 2000)",
        "value": fits_total / el, "unit": "fits/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64 (CD) / bf16-exact Gram",
        "data": "synthetic",
        "config": {"workload": f"Gaussian elastic net l1_ratio 0.5, {R} responses x {nlam} "
                               f"alphas x ({K} splits + refit) = {fits_total} fits on "
                               f"{s.N} x {s.p} timeshifted 0/1 predictors",
                   "config_name": "c5", "rank0": st,
                   "parallelism": f"responses round-robin over {world} rank(s)",
                   "refit_nonzeros_r0": [int(np.sum(np.abs(out[0][j]["refit_coef"]) > 0))
                                         for j in range(nlam)]},
        "roofline": None,
        "cpu_baseline": cpu}))


def bench_prep(a):
    """lynne_pp.preprocess_lynne's arithmetic (sglm_prep_session) on a
    16M-row synthetic session resident in HBM (9 float64 input columns -> 40 derived columns).
    One step = one session.  Sessions are independent: with N ranks each rank preprocesses
    its own session (weak scaling, no collective beyond the timing barrier)."""
    import torch
    import torch.distributed as dist
    from sglm_hip import prep, synth
    n = CONFIGS["prep"][0]
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    _, cols = synth.session(n, 100 + rank, 0.02, with_extra=False)
    Xh = np.stack([cols[c].astype(np.float64) for c in prep.IN_COLS])
    X = torch.from_numpy(Xh).cuda()
    out = torch.empty((len(prep.OUT_COLS), n), dtype=torch.float64, device="cuda")
    ws = prep.Workspace(n)
    for _ in range(max(1, a.warmup)):
        prep.session_columns_device(X, PREP_SHIFT, out, ws)
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        prep.session_columns_device(X, PREP_SHIFT, out, ws)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = (time.perf_counter() - t0) / a.steps
    call_ms = ev0.elapsed_time(ev1) / a.steps
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64,
                         device="cuda" if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0])
    if rank != 0:
        return
    # host DataFrame columns in, host columns out: the PCIe-inclusive rate (never `value`)
    t1 = time.perf_counter()
    prep.session_columns(Xh, PREP_SHIFT)
    pcie_s = time.perf_counter() - t1
    bytes_per_row = 8 * (len(prep.IN_COLS) + len(prep.OUT_COLS))
    achieved = bytes_per_row * n / (call_ms * 1e-3) / 1e9
    cpu = None
    if not a.no_cpu:
        from oracle import prep_pandas
        rows = 2_000_000
        sub = {c: v[:rows] for c, v in cols.items()}
        t2 = time.perf_counter()
        prep_pandas.derived_columns(sub, PREP_SHIFT)
        dt = time.perf_counter() - t2
        cpu = {"value": rows / dt, "unit": "session rows/s", "cores": 1, "kind": "port",
               "sample": f"oracle/prep_pandas.py (the reference's pandas operations: shift, "
                         f"bfill/ffill, cumsum, groupby transform/cumsum, diff) on the first "
                         f"{rows} rows of the same session, {dt:.2f} s"}
    print(json.dumps({
        "metric": "session preprocessing rows/s (lynne_pp.preprocess_lynne derived columns)",
        "value": n * world / el, "unit": "session rows/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"one {n}-row behaviour session per rank (9 float64 event "
                               f"columns -> 40 derived columns, trial_shift_bounds {PREP_SHIFT} as the drivers call it)",
                   "config_name": "prep", "rows": n,
                   "pcie_inclusive_rows_per_s": n / pcie_s,
                   "parallelism": f"one session per rank, {world} rank(s)"},
        "roofline": {"bound": "hbm", "kernel": "sglm_prep_session (whole call: 7 row kernels + "
                                               "9 chunked scans)",
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                     "algorithmic_bytes_per_row": bytes_per_row, "avg_call_ms": call_ms},
        "cpu_baseline": cpu}))


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())   # one rank per GPU; wraps only in rehearsals
    torch.cuda.set_device(dev)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    if a.config in ("c5", "prep"):
        (bench_c5 if a.config == "c5" else bench_prep)(a)
        if world > 1:
            dist.destroy_process_group()
        return
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective

    N, m, L, K, nlam = CONFIGS[a.config]
    t_setup = time.perf_counter()
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    design = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(__import__("pandas").DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    lams = np.logspace(-4, 1, nlam)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100) for al in lams]
    rolls = [0] * nlam
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    def step(stats=None):
        return grid.run(design, s.y, cv_idx, objs, rolls, stats=stats)

    # engine initialisation (part of setup, not a warmup step): the process's first two grids
    # pay one-time HIP runtime / allocator costs (the second grid of a fresh process measured
    # 20-30 ms slower than later ones on an 8-rank share), so two untimed passes run before the
    # W warmup steps
    for _ in range(INIT_PASSES):
        step()
    for _ in range(a.warmup):
        step()
    stats = E.IrlsStats(record=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step(stats)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # roofline of the dominant kernel (Gram) from HIP events on the launch stream
    ktime = sum(e0.elapsed_time(e1) for e0, e1, _, _ in stats.syrk_events) / 1e3
    kflop = sum(nact_flop for _, _, _, nact_flop in stats.syrk_events)
    nlaunch = len(stats.syrk_events)
    t = torch.tensor([elapsed, float(stats.fit_iters), ktime, kflop, float(nlaunch),
                      float(stats.gram_fits), stats.alg_flop, float(stats.reused)],
                     dtype=torch.float64, device="cuda" if a.dist_backend == "nccl" else "cpu")
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, fit_iters = float(mx[0]), float(sm[1])
        ktime, kflop, nlaunch = float(sm[2]), float(sm[3]), int(sm[4])
        gram_fits, alg_flop, reused = float(sm[5]), float(sm[6]), float(sm[7])
    else:
        fit_iters = float(stats.fit_iters)
        gram_fits, alg_flop = float(stats.gram_fits), stats.alg_flop
        reused = float(stats.reused)
    if rank == 0:
        pa = s.p + 1
        achieved = kflop / ktime / 1e12 if ktime > 0 else 0.0
        traffic, traffic_src = pmc_traffic()
        cpu = None
        if not a.no_cpu and world == 1:
            cpu = cpu_baseline(s, s.N, a.cpu_rows, fit_iters / a.steps, a.sklearn_rows)
        out = {
            "metric": "IRLS iters/sec on 1M×2000 design mat; CV-grid wall-clock (5-fold×20 λ)",
            "value": fit_iters / elapsed,
            "unit": "IRLS fit-iterations/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "workload": f"Poisson/log IRLS CV grid: {s.N} rows x {s.p} timeshifted predictors "
                            f"({m} events x {len(s.shifts)} lags), {K} GroupShuffleSplit splits x "
                            f"{nlam} lambdas + {nlam} refits = {nlam * (K + 1)} fits",
                "config_name": a.config,
                "n_rows": s.N, "p": s.p, "fits": nlam * (K + 1),
                "grid_wall_s": elapsed / a.steps,
                "fit_iters_per_grid": fit_iters / a.steps,
                "distinct_hessians_per_grid": gram_fits / a.steps,
                "kept_factor_fit_iters_per_grid": reused / a.steps,
                "hess_reuse_tol": E.HESS_REUSE_TOL,
                "init_passes_untimed": INIT_PASSES,
                "grid_roofline_frac": alg_flop / elapsed / (world * PEAK_BF16_TFLOPS * 1e12),
                "grid_roofline_note": "SURVEY.md 8(d): sum over fit-iterations of "
                                      "n p'(p'+1) + 4 n p' + p'^3/3 + 2 p'^2, / wall / "
                                      "(n_gpus x 2.5 PF)",
                "setup_s": setup_s,
                "parallelism": f"fits round-robin over {world} rank(s), RCCL all-gather of results",
            },
            "roofline": {
                "bound": "mfma",
                "kernel": "syrk6_kernel (X^T diag(w) X over row-compacted bit-planes, v_mfma_f32_32x32x16_bf16)",
                "achieved": achieved,
                "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_BF16_TFLOPS,
                "traffic": traffic,
                "traffic_unit": "bytes per launch (HBM/fabric, PMC)",
                "traffic_source": traffic_src,
                "algorithmic_flop_per_fit_iter": f"n_train*p'*(p'+1), p'={pa}",
                "launches": nlaunch,
                "avg_launch_ms": ktime / max(nlaunch, 1) * 1e3,
                "per_launch": [[n_, round(e0.elapsed_time(e1), 2), round(f_ / e0.elapsed_time(e1) / 1e9, 1)]
                               for e0, e1, n_, f_ in stats.syrk_events] if world == 1 else None,
            },
            "cpu_baseline": cpu,
        }
        conv = all(r["converged"] for r in res)
        out["config"]["all_converged"] = bool(conv)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
