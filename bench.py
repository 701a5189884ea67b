"""Benchmark: IRLS iterations/s and CV-grid wall-clock on the BASELINE.json north-star config.

Workload (configs[3], the config the metric is quoted on; it fits one MI355X): Poisson/log,
1M rows x 2000 time-shifted predictors (50 Bernoulli(0.02) events x 40 lags, synthetic per
SURVEY.md §8(d)), 5 GroupShuffleSplit splits x 20 lambdas + 20 full refits = 120 fits.
One step = one full CV grid (all 120 fits solved to convergence + scored).  With N ranks
the 120 fits are cut into mask-major, row-cost-balanced shards (grid.shard_plan; strong
scaling: the grid is fixed); results are all-gathered over RCCL once per grid.

value = CV-grid wall-clock (seconds per grid, max over ranks; lower is better).  The IRLS
rates ride along in `config`: all fit-iterations / s, and the Gram-forming ones (fit-iterations
whose own X^T W X was computed) / s.

Usage: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no launcher it starts
N rank processes itself (torch.distributed.run, 127.0.0.1) before touching the GPU.
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
# MI355X f64 vector FMA rate MEASURED on the box (tools/probe/f64_fma.hip: every CU full of
# independent v_fma_f64 chains, 61.3 TFLOP/s): MI355X_MICROARCH.md gives the f32 peaks only;
# AMD's spec sheet says 78.6 at the nominal clock
PEAK_F64_TFLOPS = 61.3

CONFIGS = {
    # name: (N rows, events m, L -> lags -L..L-1, n_splits, lambdas)
    "c4": (1_000_000, 50, 20, 5, 20),
    # C4 plus the production design's two unshifted continuous counters (cumcount^2 / 5000,
    # pp_design_mat.py:167-172): a mixed 0/1 + float64 design (csrc/mixed.hip)
    "c4mixed": (1_000_000, 50, 20, 5, 20),
    "c3": (100_000, 25, 10, 5, 20),
    "small": (50_000, 10, 5, 5, 4),
    # C5: 64 responses x C4 design, Gaussian elastic-net lambda path (l1_ratio 0.5, 20 alphas)
    "c5": (1_000_000, 50, 20, 5, 20),
    # session preprocessing (lynne_pp.preprocess_lynne): rows per session
    "prep": (16_000_000, 0, 0, 0, 0),
    # gen_signal_df.generate_signal_df: trials per session
    "signal": (0, 0, 0, 0, 0),
    # pp_design_mat.make_design_mat: trials per session
    "designmat": (0, 0, 0, 0, 0),
    # the reference's own logged OLS workload (02-create_features-lynne.ipynb cell 3, 483 s):
    # ~1.58M rows, 7 events x 41 lags = 287 predictors, 10 GroupShuffleSplit splits + refit +
    # holdout score, through the drop-in flow from a host frame
    "olsref": (1_581_817, 7, 20, 10, 1),
    # the production 50-split grid (er_refactored_from_scratch_cleanup.py:230-246, 421-452) at
    # the logged 1,900,992-row frame (02-create_features-lynne-f5.ipynb): 18 events x 41 lags
    "prod50": (1_900_992, 18, 20, 50, 1),
    # the multi-session production flow of sglm_cb_concat_make_design_mat.py:244-363 at the
    # logged frame size: 18 events x 41 lags + 2 counters + session dummies, 3 splits, OLS
    # without intercept
    "cbprod": (1_900_992, 18, 20, 3, 1),
}
DM_TRIALS = 100_000                 # ~9.8M rows at 50 Hz (a ~54 h session, or a day's sessions)
DM_CPU_TRIALS = 20_000              # the pandas sample (~2M rows, ~6 s)
DM_INTERACTIONS = {"Reward": ["Consumption", "Cue"], "h2": ["Select"]}
SIGNAL_TRIALS = 60_000
C5_RESPONSES = 64
PREP_SHIFT = 1     # er_refactored_from_scratch_cleanup.py:269 calls preprocess_lynne(df, trial_shift_bounds=1)
INIT_PASSES = 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 2; 20 for the millisecond-scale designmat step)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 1; 3 for "
                    "designmat)")
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the float64 Newton-distance spot check after the timed region "
                         "(its rocBLAS kernels stay out of a kernel-trace profile)")
    ap.add_argument("--cpu-full-fold", type=int, default=1,
                    help="1: the CPU baseline times one full-size split fit + refit (BASELINE.md "
                         "§2); 0: only the row sample")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in production-flow leg (dropin_grid_s)")
    ap.add_argument("--cpu-rows", type=int, default=100_000,
                    help="rows of the oracle Newton sample (secondary CPU figure)")
    ap.add_argument("--sklearn-rows", type=int, default=100_000,
                    help="rows of the reference-path (sklearn lbfgs fold loop) sample")
    ap.add_argument("--shard", default=None, choices=["fits", "rows"],
                    help="N > 1: whole fits per rank (default) or row slabs (sglm_hip/comm.py)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for real runs; gloo to rehearse several ranks "
                         "on fewer GPUs")
    a = ap.parse_args()
    short = a.config == "designmat"
    if a.steps is None:
        a.steps = 20 if short else 2
    if a.warmup is None:
        a.warmup = 3 if short else 1
    return a


def dense_slice(s, rows):
    m = s.E.shape[1]
    X = np.empty((rows, s.p), dtype=np.float64)
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        X[:, bi * m:(bi + 1) * m] = s.E[r0 - sh:r0 - sh + rows]
    return X


def _cpu_model():
    import platform
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:  # pragma: no cover
        return platform.machine()


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def cpu_reference_grid(s, cv_idx, lams, rows, lam_sample=(0, 10, 19), fold_threads=4):
    """The reference's CPU path on a row sample of the same design: for each sampled lambda,
    cv_glm_single_params' work (backend/sglm_cv.py:106-181) -- the 5 split fits on
    X[idx_train] copies dealt to 4 worker threads (:162-170), then the full refit -- with the
    estimator backend/sglm.py:112-115 selects, sklearn TweedieRegressor(power=1, alpha),
    default lbfgs / tol 1e-4 / max_iter 100.  sklearn is called directly: the reference
    modules' import is denied.  Extrapolated to the 1M-row, 20-lambda grid:
    x (20 / lambdas sampled) x (N / rows), labelled as such."""
    import threading
    from sklearn.linear_model import TweedieRegressor
    rows = min(rows, s.N)
    X = dense_slice(s, rows)
    y = s.y[:rows]
    # the splits restricted to the sample's rows (the same trial-id splits)
    sub = [(tr[tr < rows], te[te < rows]) for tr, te in cv_idx]
    per_lam = []
    iters = []
    t_all = time.perf_counter()
    for j in lam_sample:
        alpha = float(lams[j])
        t0 = time.perf_counter()
        tasks = list(range(len(sub)))
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    if not tasks:
                        return
                    k = tasks.pop(0)
                tr = sub[k][0]
                m = TweedieRegressor(power=1, alpha=alpha).fit(X[tr], y[tr])
                iters.append(int(m.n_iter_))
        ths = [threading.Thread(target=worker) for _ in range(fold_threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        m = TweedieRegressor(power=1, alpha=alpha).fit(X, y)       # the full refit
        iters.append(int(m.n_iter_))
        per_lam.append(time.perf_counter() - t0)
    sample_s = time.perf_counter() - t_all
    grid_s = float(np.mean(per_lam)) * len(lams) * (s.N / rows)
    return {"value": grid_s, "unit": "s per CV grid (extrapolated)", "cores": _blas_threads(),
            "kind": "reference",
            "sample": f"sklearn TweedieRegressor(power=1) lbfgs, reference fold loop (4 threads "
                      f"+ refit), first {rows} rows x {s.p}, lambdas {list(lam_sample)} in "
                      f"{sample_s:.1f} s (lbfgs iters {min(iters)}-{max(iters)}); "
                      f"x{len(lams) / len(lam_sample):.2f} lambdas x{s.N / rows:.0f} rows",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def cpu_reference_full(s, cv_idx, lams, js=(0, 10, 19)):
    """The BASELINE.md §2 CPU measurement at full size: for each sampled lambda index j, ONE
    split fit (split 0's train rows) and the full refit, sklearn TweedieRegressor(power=1,
    alpha) with its default lbfgs (backend/sglm.py:112-115) on dense float64 copies
    (X[idx_train] as the reference's fold loop makes them, backend/sglm_cv.py:107-110).  The
    strongest, middle and weakest penalties are sampled because lbfgs' iteration count moves
    with lambda.  Grid = mean over the sampled lambdas of (n_splits x split fit + refit) x the
    lambda count, labelled extrapolated.  Returns (seconds per grid, detail dict)."""
    from sklearn.linear_model import TweedieRegressor
    tr = np.asarray(cv_idx[0][0])
    X = dense_slice(s, s.N)
    Xtr = X[tr]
    ytr = s.y[tr]
    per = []
    for j in js:
        alpha = float(lams[j])
        t0 = time.perf_counter()
        m1 = TweedieRegressor(power=1, alpha=alpha).fit(Xtr, ytr)
        t_split = time.perf_counter() - t0
        t0 = time.perf_counter()
        m2 = TweedieRegressor(power=1, alpha=alpha).fit(X, s.y)
        t_refit = time.perf_counter() - t0
        per.append({"lambda_index": int(j), "lambda": alpha, "split_fit_s": round(t_split, 2),
                    "refit_s": round(t_refit, 2),
                    "lbfgs_iters": [int(m1.n_iter_), int(m2.n_iter_)]})
    del X, Xtr
    nspl = len(cv_idx)
    grid_s = float(np.mean([nspl * q["split_fit_s"] + q["refit_s"] for q in per])) * len(lams)
    return grid_s, {"lambdas": per, "rows": [int(tr.size), int(s.N)]}


def cpu_port_iter(s, n_rows_unit, rows):
    """Secondary: the float64 oracle's damped Newton (the IRLS restatement) per iteration,
    scaled to 1M rows."""
    from oracle import glm_ref
    rows = min(rows, s.N)
    X = dense_slice(s, rows)
    t0 = time.perf_counter()
    _, _, iters = glm_ref.fit_tweedie_newton(X, s.y[:rows], 1e-2, 1.0, tol=1e-8, max_iter=50,
                                             return_iters=True)
    dt = time.perf_counter() - t0
    return {"iters_per_s_1M_rows": max(iters, 1) / dt * rows / n_rows_unit, "rows": rows,
            "iters": int(iters), "s": round(dt, 2)}


def pmc_traffic(kernel="syrk6_kernel"):
    """HBM bytes per Gram launch from the newest committed PMC summary (profiles/*_pmc_traffic.json,
    written by tools/pmc_traffic.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    bench's grid; gfx950 corrections applied there).  PMC counters cannot be read in-process."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))[::-1]:
        with open(fn) as f:
            d = json.load(f)
        dom = d.get("dominant") or {}
        if kernel in dom.get("kernel", ""):
            return dom["traffic_bytes_per_launch"], os.path.relpath(fn, ROOT)
    return None, None


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
    # the responses resident in HBM before the timed region, like the design (the host copy
    # stays for the CPU baseline)
    Yd = torch.from_numpy(Y).cuda()
    for _ in range(a.warmup):
        enet.cv_enet_path(design, Yd, cv_idx, alphas, l1_ratio=0.5)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cd_ms = cd_flop = 0.0
    for _ in range(a.steps):
        st = {"record": True}
        out = enet.cv_enet_path(design, Yd, cv_idx, alphas, l1_ratio=0.5, stats=st)
        cd_ms += st.pop("cd_ms")
        cd_flop += st.pop("cd_flop")
        st.pop("record")
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
        cpu = cpu_reference_enet(s, Y, cv_idx, alphas, a.sklearn_rows, R, fits_total)
    achieved = cd_flop / (cd_ms * 1e-3) / 1e12
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
        "roofline": {"bound": "valu-f64", "kernel": "enet_cd_lane_kernel (cyclic coordinate "
                                                   "descent on the shared float64 Gram)",
                     "achieved": achieved, "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_F64_TFLOPS, "traffic": None,
                     "algorithmic_flop_per_sweep_per_fit": 2 * s.p * s.p,
                     "avg_launch_ms": cd_ms / a.steps,
                     "peak_source": "measured f64 FMA rate (tools/probe/f64_fma.hip, "
                                    "profiles/r04_f64_probe.json); MI355X_MICROARCH.md "
                                    "lists no f64 peak (AMD spec 78.6 at 2.4 GHz)",
                     "bound_note": "the coordinate steps are sequential (one barrier per "
                                   "coordinate): latency-bound; the Q row stream is an L2 hit "
                                   "for the workgroups of one (Q, alpha) on an XCD"},
        "cpu_baseline": cpu}))


def cpu_reference_enet(s, Y, cv_idx, alphas, rows, R, fits_total, lam_sample=(0, 10, 19),
                       fold_threads=4):
    """The reference's CPU path for one response on a row sample: cv_glm_single_params' fold
    loop (backend/sglm_cv.py:106-181; 5 split fits on X[idx_train] copies dealt to 4 threads,
    then the full refit) with the estimator backend/sglm.py:109-110 selects, sklearn
    ElasticNet(alpha, l1_ratio=0.5) at its defaults (max_iter 1000, tol 1e-4), called directly
    (the reference's import is denied).  Extrapolated to the C5 grid:
    x (alphas / sampled) x responses x (N / rows) (CD epochs are O(n p) with precompute=False),
    labelled as such."""
    import threading
    from sklearn.linear_model import ElasticNet
    rows = min(rows, s.N)
    X = dense_slice(s, rows)
    y = Y[:rows, 0]
    sub = [(tr[tr < rows], te[te < rows]) for tr, te in cv_idx]
    per_lam, iters = [], []
    t_all = time.perf_counter()
    for j in lam_sample:
        alpha = float(alphas[j])
        t0 = time.perf_counter()
        tasks = list(range(len(sub)))
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    if not tasks:
                        return
                    k = tasks.pop(0)
                m = ElasticNet(alpha=alpha, l1_ratio=0.5).fit(X[sub[k][0]], y[sub[k][0]])
                iters.append(int(m.n_iter_))
        ths = [threading.Thread(target=worker) for _ in range(fold_threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        m = ElasticNet(alpha=alpha, l1_ratio=0.5).fit(X, y)
        iters.append(int(m.n_iter_))
        per_lam.append(time.perf_counter() - t0)
    sample_s = time.perf_counter() - t_all
    grid_s = float(np.mean(per_lam)) * len(alphas) * R * (s.N / rows)
    return {"value": fits_total / grid_s, "unit": "elastic-net fits/s (extrapolated)",
            "cores": _blas_threads(), "kind": "reference",
            "sample": f"sklearn ElasticNet(l1_ratio=0.5) in the reference fold loop (4 threads "
                      f"+ refit), response 0, first {rows} rows x {s.p}, alphas "
                      f"{list(lam_sample)} in {sample_s:.1f} s (CD epochs {min(iters)}-"
                      f"{max(iters)}); x{len(alphas) / len(lam_sample):.2f} alphas x{R} "
                      f"responses x{s.N / rows:.0f} rows",
            "grid_wall_s_extrapolated": grid_s, "cpu": _cpu_model(), "nproc": os.cpu_count()}


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


def bench_signal(a):
    """gen_signal_df.generate_signal_df's per-sample work on the device
    (sglm_scatter_rows: the trial table aligned onto the signal, 31 columns; sglm_signal_trials:
    nTrial / nEndTrial / diffTrialNums and the duplication row map) for one synthetic session
    of SIGNAL_TRIALS trials, trial rows resident in HBM.  One step = one session; sessions are
    independent (weak scaling).  The drop-in's whole call (host pandas table steps + these
    kernels + the host row gather), host frames in and out, rides along in `config`."""
    import torch
    import torch.distributed as dist
    import pandas as pd
    from sglm.features import gen_signal_df as G
    from sglm_hip import signal, synth
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    sig, table = synth.signal_session(SIGNAL_TRIALS, 200 + rank)
    n = len(sig)
    # trial rows per index column as the drop-in builds them (host table steps, untimed here)
    df_t = G.generate_Ab_labels(table)
    for b in G.BASIS_AA_COLS:
        df_t[b] = (df_t["label"] == b).astype(np.float64)
    df_t[G.TABLE_INDEX_COLUMNS] = G.matlab_indexing_to_python(df_t[G.TABLE_INDEX_COLUMNS])
    df_t = G.replace_missed_center_out_indexes(df_t)
    pieces, nc = [], 0
    for col in G.TABLE_INDEX_COLUMNS:
        tr = df_t[G.get_is_relevant_trial(df_t["hasAllPhotometryData"], df_t[col])]
        pos = tr[col].to_numpy().astype(np.int64)
        keep = pos < n
        r = tr["wasRewarded"].to_numpy(dtype=np.float64)
        vals = [np.ones_like(r), r, 1.0 - r]
        if col in G._SIDE_COLS:
            vals += [tr[b].to_numpy(dtype=np.float64) for b in G.BASIS_AA_COLS]
        v = np.ascontiguousarray(np.stack(vals)[:, keep])
        pieces.append((nc, torch.from_numpy(pos[keep]).cuda(), torch.from_numpy(v).cuda()))
        nc += v.shape[0]
    out = torch.empty((nc, n), dtype=torch.float64, device="cuda")
    ws = signal.TrialWorkspace(n)
    ci_row, so_row = pieces[0][0], pieces[3][0]

    def step():
        for c0, rd, vd in pieces:
            signal.aligned_columns_device(n, rd, vd, out[c0:c0 + vd.shape[0]])
        signal.trial_runs_device(out[ci_row], out[so_row], -20, 20, ws)

    for _ in range(max(1, a.warmup)):
        step()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
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
    n_out = signal.n_out(n, -20, int(ws.ncopies.item()))
    nr = sum(int(rd.numel()) * (vd.shape[0] + 1) for _, rd, vd in pieces)
    # NaN fill of every aligned column, the trial rows scattered (values + row index), the two
    # flag columns read, three count columns written, the row map (int64 + u8) per output row
    algo = 8 * nc * n + 8 * nr + 16 * n + 24 * n + 9 * n_out
    achieved = algo / (call_ms * 1e-3) / 1e9
    t1 = time.perf_counter()
    full, _ = G.signal_frame(sig, table)
    e2e_s = time.perf_counter() - t1
    assert len(full) == n_out
    cpu = None
    if not a.no_cpu:
        from oracle import signal_ref
        trials = 3000
        ssig, stab = synth.signal_session(trials, 200 + rank)
        t2 = time.perf_counter()
        signal_ref.signal_frame(ssig, stab)
        dt = time.perf_counter() - t2
        cpu = {"value": len(ssig) / dt, "unit": "signal rows/s", "cores": 1, "kind": "port",
               "sample": f"oracle/signal_ref.py (the reference's pandas alignment, cumsum/shift "
                         f"and per-trial duplication loop) on a {trials}-trial session of "
                         f"{len(ssig)} rows, {dt:.2f} s"}
    print(json.dumps({
        "metric": "signal rows/s (gen_signal_df.generate_signal_df per-sample columns)",
        "value": n * world / el, "unit": "signal rows/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"one {SIGNAL_TRIALS}-trial session per rank ({n} signal rows, "
                               f"{nc} aligned columns, trial bounds -20 / +20, {n_out} output "
                               f"rows)",
                   "config_name": "signal", "rows": n,
                   "dropin_host_frames_rows_per_s": n / e2e_s,
                   "parallelism": f"one session per rank, {world} rank(s)"},
        "roofline": {"bound": "hbm", "kernel": "sglm_scatter_rows x5 + sglm_signal_trials "
                                               "(whole step: 17 launches)",
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                     "algorithmic_bytes_per_step": algo, "avg_call_ms": call_ms},
        "cpu_baseline": cpu}))


def bench_designmat(a):
    """pp_design_mat.make_design_mat (pp_design_mat.py:128-205) on a
    synthetic DM_TRIALS-trial session resident in HBM (float64 columns), interactions Reward x
    (Consumption, Cue) and h2 x Select, first licks of the consumption bouts.  One step = one
    session's design matrix (grouping, heatmap columns, licks, counters, pulls, interactions,
    flag) into one output block.  Sessions are independent: one per rank (weak scaling)."""
    import contextlib
    import io
    import torch
    import torch.distributed as dist
    import pp_design_mat
    from sglm_hip import designmat, synth
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    states = ["Select", "Consumption", "ENLP"]
    ts, tr = synth.designmat_session(DM_TRIALS, 300 + rank)
    n = len(ts)
    tri = tr.set_index("nTrial").convert_dtypes()
    cols, dts = designmat.upload(ts, states)

    def step():
        return designmat.design_matrix_device(cols, dts, n, tri, states, [1], DM_INTERACTIONS,
                                              verbose=False)
    for _ in range(max(1, a.warmup)):
        res = step()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        res = step()
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
    K = len(res.names)
    n_in = len([c for c in cols if c != "__order__"])
    algo_row = 8 * (n_in + K)                # every input column read once, the matrix written
    achieved = algo_row * n / el / 1e9
    # the drop-in with host frames in and out (PCIe + pandas frame assembly), never `value`
    t1 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        pp_design_mat.make_design_mat(ts.copy(), tr, interactions=DM_INTERACTIONS)
    e2e_s = time.perf_counter() - t1
    cpu = None
    if not a.no_cpu:
        import warnings
        from oracle import designmat_pandas
        sts, str_ = synth.designmat_session(DM_CPU_TRIALS, 300 + rank)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            t2 = time.perf_counter()
            designmat_pandas.make_design_mat(sts, str_, interactions=DM_INTERACTIONS,
                                             verbose=False)
            dt = time.perf_counter() - t2
        cpu = {"value": len(sts) / dt, "unit": "session rows/s", "cores": 1, "kind": "port",
               "sample": f"oracle/designmat_pandas.py (the reference's pandas operations: "
                         f"groupby cumcount / nth / first / sum, map, get_dummies) on a "
                         f"{DM_CPU_TRIALS}-trial session of {len(sts)} rows, {dt:.2f} s"}
    print(json.dumps({
        "metric": "design-matrix rows/s (pp_design_mat.make_design_mat)",
        "value": n * world / el, "unit": "session rows/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"one {DM_TRIALS}-trial session per rank ({n} rows, {n_in} "
                               f"float64 input columns -> {K} design columns; interactions "
                               f"{DM_INTERACTIONS}, nth_licks [1])",
                   "config_name": "designmat", "rows": n, "columns": res.names,
                   "dropin_host_frames_rows_per_s": n / e2e_s,
                   "event_ms_per_step": call_ms,
                   "parallelism": f"one session per rank, {world} rank(s)"},
        "roofline": {"bound": "hbm", "kernel": "design_matrix_device (whole step: 2 groupings, "
                                               "heatmap, licks, counters, pull, trial maps, flag)",
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                     "algorithmic_bytes_per_row": algo_row, "avg_step_ms": el * 1e3},
        "cpu_baseline": cpu}))


def ols_flow(df, ev, L, K, timings=None):
    """The reference's OLS production flow through the drop-in API
    (er_refactored_from_scratch_cleanup.py:421-452): sglm_ez.timeshift_cols (shifts 0,
    -L..-1, 1..L) -> the NaN-row filter -> holdout_split_by_trial_id (20 %) -> cv_idx_by_trial_id
    (K splits, test 20 %) -> simple_cv_fit (OLS, fit_intercept) -> training_fit_holdout_score.
    Returns (simple_cv_fit results, holdout R^2, setup frame)."""
    import contextlib
    import io
    import torch
    import sglm_ez
    ph = {} if timings is None else timings

    def mark(name, t):
        torch.cuda.synchronize()
        now = time.perf_counter()
        ph[name] = ph.get(name, 0.0) + now - t
        return now
    t = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):            # the reference prints as it goes
        dfrel = sglm_ez.timeshift_cols(df, ev, neg_order=-L, pos_order=L)
        xcols = sglm_ez.add_timeshifts_to_col_list(ev, ev, neg_order=-L, pos_order=L)
        t = mark("timeshift_cols", t)
        dfrel = dfrel[dfrel[["nTrial"] + xcols + ["y"]].isna().sum(axis=1) == 0]
        t = mark("nan_filter", t)
        np.random.seed(30186)
        hold = sglm_ez.holdout_split_by_trial_id(dfrel, id_cols=["nTrial"], perc_holdout=0.2)
        setup, holdout = dfrel.loc[~hold], dfrel.loc[hold]
        cv_idx = sglm_ez.cv_idx_by_trial_id(setup, trial_id_columns=["nTrial"], num_folds=K,
                                            test_size=0.2)
        t = mark("holdout_and_folds", t)
        kws = [{"alpha": 0.0, "l1_ratio": 0.0, "max_iter": 1000, "fit_intercept": True}]
        out = sglm_ez.simple_cv_fit(setup[xcols], setup["y"], cv_idx, kws, model_type="Normal",
                                    score_method="r2")
        t = mark("simple_cv_fit", t)
        _, hs, _ = sglm_ez.training_fit_holdout_score(setup[xcols], setup["y"], holdout[xcols],
                                                      holdout["y"], out[2])
        mark("training_fit_holdout_score", t)
    return out, hs, setup, xcols, cv_idx


def cpu_reference_ols(df, ev, L, setup, cv_idx, K):
    """The reference's CPU path sampled the BASELINE.md §2 way: sklearn LinearRegression (what
    GLM('Normal', alpha=0) selects, backend/sglm.py:96-101) on ONE full-size fold (its train rows
    of the dense float64 lag design) and on the full setup rows (the refit), called directly
    (the reference's import is denied); the workload = K fold fits + the refit
    + training_fit_holdout_score's second full fit, extrapolated from the two timings."""
    from sklearn.linear_model import LinearRegression
    E = df[ev].to_numpy(dtype=np.float64)
    y = df["y"].to_numpy()
    pos = setup.positions()
    shifts = [0] + list(range(-L, 0)) + list(range(1, L + 1))

    def dense(rows):
        X = np.empty((rows.size, len(shifts) * len(ev)))
        for bi, sh in enumerate(shifts):
            X[:, bi * len(ev):(bi + 1) * len(ev)] = E[rows - sh]
        return X
    tr = pos[np.asarray(cv_idx[0][0])]
    X = dense(tr)
    t0 = time.perf_counter()
    LinearRegression().fit(X, y[tr])
    t_fold = time.perf_counter() - t0
    del X
    X = dense(pos)
    t0 = time.perf_counter()
    LinearRegression().fit(X, y[pos])
    t_refit = time.perf_counter() - t0
    del X
    total = K * t_fold + 2 * t_refit
    return {"value": total, "unit": "s per workload (extrapolated)", "cores": _blas_threads(),
            "kind": "reference",
            "sample": f"sklearn LinearRegression (lstsq) on fold 0's {tr.size} train rows x "
                      f"{len(shifts) * len(ev)} ({t_fold:.1f} s) and on the {pos.size} setup "
                      f"rows ({t_refit:.1f} s); x{K} folds + 2 full fits",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def bench_ols(a):
    """The reference's OLS workloads end to end on one GPU: the logged notebook run (config
    olsref) and the 50-split production grid (prod50), from a host event frame through the
    drop-in API (ols_flow).  One step = the whole flow."""
    import torch
    from sglm_hip import synth
    N, m, L, K, _ = CONFIGS[a.config]
    df, ev, beta, b0 = synth.ols_frame(N, m, -L, L, seed=11)
    for _ in range(a.warmup):
        ols_flow(df, ev, L, K)
    torch.cuda.synchronize()
    ph = {}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out, hs, setup, xcols, cv_idx = ols_flow(df, ev, L, K, ph)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    best = out[3]
    coef = np.asarray(best.model.coef_)
    # the synthetic truth is known: the refit recovers it to the noise level
    truth_err = float(np.max(np.abs(coef - beta.reshape(-1))))
    cpu = None if a.no_cpu else cpu_reference_ols(df, ev, L, setup, cv_idx, K)
    p = len(xcols)
    print(json.dumps({
        "metric": "IRLS iters/sec on 1M\u00d72000 design mat; CV-grid wall-clock (5-fold\u00d720 \u03bb)",
        "value": el, "unit": "s per OLS workload (host frame -> fits -> holdout score)",
        "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": el * 1e3,
        "higher_is_better": False, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64 (exact 0/1 Gram in f32 integers, float64 factor / normal equations)",
        "data": "synthetic",
        "config": {"workload": f"Gaussian OLS (fit_intercept) {N} rows x {p} predictors "
                               f"({m} events x {2 * L + 1} lags), {K} GroupShuffleSplit splits + "
                               f"refit + holdout score, drop-in flow from a host frame",
                   "config_name": a.config, "setup_rows": int(setup.shape[0]),
                   "phases_ms": {k: v / a.steps * 1e3 for k, v in ph.items()},
                   # the host pandas lines before the shift (convert_dtypes / dropna /
                   # get_dummies on the raw frame) are the user's own pandas, not the path; the
                   # CPU baseline times the fits alone (folds + 2 full fits)
                   "flow_ms_after_host_prepare": (el - ph.get("prepare", 0.0) / a.steps) * 1e3,
                   "fits_ms": (ph.get("simple_cv_fit", 0.0)
                               + ph.get("training_fit_holdout_score", 0.0)) / a.steps * 1e3,
                   "best_cv_R2": float(out[0]), "holdout_R2": float(hs),
                   "refit_max_abs_err_vs_truth": truth_err,
                   "reference_logged_s": 483.2 if a.config == "olsref" else None,
                   "parallelism": "one GPU (the flow is one design; fits batched)"},
        "roofline": None,
        "cpu_baseline": cpu}))


CB_NOT_SFTD = ["time_from_enl_onset", "time_from_enlp_onset"]
CB_TRIAL_CONSTANTS = ["iBlock", "nTrial"]


def cb_flow(df0, X_cols, neg, pos, folds=3, timings=None, y_="grn"):
    """sglm_cb_concat_make_design_mat.py:244-363 replayed through the drop-in API: the frame
    convert_dtypes()'d (:244), the response's NaN rows dropped (:251), session dummies (:262),
    the event columns shifted (sglm_ez.timeshift_cols for the driver's own pandas CB_timeshifts
    -- the same columns and names, :50-74, 271-276; the lagged frame stays on the device), the
    flagged trials dropped (:281-283), the trial constants assigned back (:287), dropna (:294),
    holdout_split_by_trial_id 20 % (:305-311), cv_idx_by_trial_id (folds, test 20 %, :330-334),
    nTrial dropped (:343-344), simple_cv_fit OLS fit_intercept=False (:346-352) and
    training_fit_holdout_score (:357; the driver's function, :131-153).  Returns (simple_cv_fit
    results, holdout R^2, X_setup, y_setup, cv indices, column list)."""
    import contextlib
    import io
    import random
    import pandas as pd
    import torch
    import sglm_ez
    ph = {} if timings is None else timings

    def mark(name, t):
        torch.cuda.synchronize()
        now = time.perf_counter()
        ph[name] = ph.get(name, 0.0) + now - t
        return now
    t = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        df = df0.convert_dtypes()
        df_y = df.dropna(subset=y_).reset_index(drop=True)
        df_y = pd.get_dummies(df_y, columns=["session"])
        session_constants = [c for c in df_y.columns if "session" in c]
        t = mark("prepare", t)
        dfrel = sglm_ez.timeshift_cols(df_y, X_cols, neg_order=neg, pos_order=pos)
        X_cols_sftd = sglm_ez.add_timeshifts_to_col_list(X_cols, X_cols, neg_order=neg,
                                                         pos_order=pos)
        t = mark("timeshift_cols", t)
        dfrel = dfrel.loc[df_y["flag"] == 0]
        df_y = df_y.loc[df_y["flag"] == 0]
        dfrel[CB_TRIAL_CONSTANTS] = df_y[CB_TRIAL_CONSTANTS]
        assert np.all(dfrel.index == df_y.index)
        dfrel = dfrel.dropna()
        df_y = df_y.loc[df_y.index.isin(dfrel.index.values)]
        t = mark("flag_constants_dropna", t)
        X_cols_sftd = X_cols_sftd + ["nTrial"] + CB_NOT_SFTD + session_constants
        np.random.seed(30186)
        random.seed(30186)
        holdout = sglm_ez.holdout_split_by_trial_id(dfrel, id_cols=["nTrial"], perc_holdout=0.2)
        dfrel_holdout, dfrel_setup = dfrel.loc[holdout], dfrel.loc[~holdout]
        X_setup, X_holdout = dfrel_setup[X_cols_sftd].copy(), dfrel_holdout[X_cols_sftd].copy()
        y_setup, y_holdout = dfrel_setup[y_].copy(), dfrel_holdout[y_].copy()
        cv = sglm_ez.cv_idx_by_trial_id(X_setup, y=y_setup, trial_id_columns=["nTrial"],
                                        num_folds=folds, test_size=0.2)
        dfrel["holdout_mask"] = holdout
        X_setup = X_setup.drop(columns=["nTrial"])
        X_holdout = X_holdout.drop(columns=["nTrial"])
        t = mark("holdout_and_folds", t)
        hp = [{"alpha": 0.0, "l1_ratio": 0.0, "max_iter": 1000, "fit_intercept": False}]
        out = sglm_ez.simple_cv_fit(X_setup, y_setup, cv, hp, model_type="Normal", verbose=0,
                                    score_method="r2")
        t = mark("simple_cv_fit", t)
        _, hs, _ = sglm_ez.training_fit_holdout_score(X_setup, y_setup, X_holdout, y_holdout,
                                                      out[2])
        mark("training_fit_holdout_score", t)
    return out, hs, X_setup, y_setup, cv, [c for c in X_cols_sftd if c != "nTrial"]


def cpu_reference_cb(X_setup, y_setup, cv, folds):
    """The reference's CPU path for the cb flow sampled the BASELINE.md §2 way: sklearn
    LinearRegression(fit_intercept=False) (GLM('Normal', alpha=0, fit_intercept=False),
    backend/sglm.py:96-101) on ONE full-size fold's train rows of the materialised float64
    design and on the full setup rows (the refit); workload = folds x fold fit + 2 full fits
    (simple_cv_fit's refit and training_fit_holdout_score's), extrapolated."""
    from sklearn.linear_model import LinearRegression
    X = X_setup.to_numpy(dtype=np.float64)
    y = np.asarray(y_setup.to_numpy(dtype=np.float64, na_value=np.nan))
    tr = np.asarray(cv[0][0])
    Xtr = X[tr]
    t0 = time.perf_counter()
    LinearRegression(fit_intercept=False).fit(Xtr, y[tr])
    t_fold = time.perf_counter() - t0
    del Xtr
    t0 = time.perf_counter()
    LinearRegression(fit_intercept=False).fit(X, y)
    t_refit = time.perf_counter() - t0
    total = folds * t_fold + 2 * t_refit
    return {"value": total, "unit": "s per workload (extrapolated)", "cores": _blas_threads(),
            "kind": "reference",
            "sample": f"sklearn LinearRegression(fit_intercept=False) on fold 0's {tr.size} "
                      f"train rows x {X.shape[1]} ({t_fold:.1f} s) and on the {X.shape[0]} "
                      f"setup rows ({t_refit:.1f} s); x{folds} folds + 2 full fits",
            "cpu": _cpu_model(), "nproc": os.cpu_count()}


def bench_cb(a):
    """The multi-session production flow of sglm_cb_concat_make_design_mat.py (cb_flow) on one
    GPU at the logged production frame size: 1,900,992 rows, 18 events x 41 lags + the two
    counters + one dummy per session (4 sessions), 3 splits.  One step = the whole flow from the
    host frame."""
    import torch
    from sglm_hip import synth
    N, m, L, K, _ = CONFIGS[a.config]
    df, ev, beta, gamma, offs = synth.cb_frame(N, m, -L, L, sessions=4, seed=13)
    for _ in range(a.warmup):
        cb_flow(df, ev, -L, L, K)
    torch.cuda.synchronize()
    ph = {}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out, hs, X_setup, y_setup, cv, xcols = cb_flow(df, ev, -L, L, K, ph)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    coef = np.asarray(out[3].model.coef_)
    nl = len(ev) * (2 * L + 1)
    truth_err = float(np.max(np.abs(coef[:nl] - beta.reshape(-1))))
    cpu = None if a.no_cpu else cpu_reference_cb(X_setup, y_setup, cv, K)
    print(json.dumps({
        "metric": "IRLS iters/sec on 1M\u00d72000 design mat; CV-grid wall-clock (5-fold\u00d720 \u03bb)",
        "value": el, "unit": "s per production workload (host frame -> fits -> holdout score)",
        "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": el * 1e3,
        "higher_is_better": False, "scaling": "strong", "vs_baseline": None,
        "dtype": "f64 (exact 0/1 Gram in f32 integers + float64 continuous rows, float64 "
                 "normal equations)",
        "data": "synthetic",
        "config": {"workload": f"Gaussian OLS (fit_intercept=False) {N} rows x {len(xcols)} "
                               f"predictors ({m} events x {2 * L + 1} lags + 2 counters + "
                               f"{len(xcols) - nl - 2} session dummies), {K} splits + refit + "
                               f"holdout score, sglm_cb_concat_make_design_mat.py:244-363 from "
                               f"a host frame",
                   "config_name": a.config, "setup_rows": int(X_setup.shape[0]),
                   "phases_ms": {k: v / a.steps * 1e3 for k, v in ph.items()},
                   # the host pandas lines before the shift (convert_dtypes / dropna /
                   # get_dummies on the raw frame) are the user's own pandas, not the path; the
                   # CPU baseline times the fits alone (folds + 2 full fits)
                   "flow_ms_after_host_prepare": (el - ph.get("prepare", 0.0) / a.steps) * 1e3,
                   "fits_ms": (ph.get("simple_cv_fit", 0.0)
                               + ph.get("training_fit_holdout_score", 0.0)) / a.steps * 1e3,
                   "best_cv_R2": float(out[0]), "holdout_R2": float(hs),
                   "refit_lag_coef_max_abs_err_vs_truth": truth_err,
                   "parallelism": "one GPU (the flow is one design; fits batched)"},
        "roofline": None,
        "cpu_baseline": cpu}))


def spawn_ranks(a):
    """``--gpus N`` without a launcher: start N rank processes (torch.distributed.run, one per
    GPU, rendezvous on 127.0.0.1) as CHILDREN before anything touches the GPU, and exit with
    their status.  Under a launcher (WORLD_SIZE set) this returns and main() runs the rank."""
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def dropin_frame(s):
    """The host event DataFrame the reference's production flow starts from
    (er_refactored_from_scratch_cleanup.py:421-452): the N_raw rows of the 50 float64 event
    columns, nTrial, and the response (NaN on the rows the lag expansion cannot fill)."""
    import pandas as pd
    Nr, m = s.E.shape
    r0 = s.L - 1
    ev = [f"e{a}" for a in range(m)]
    df = pd.DataFrame(s.E.astype(np.float64), columns=ev)
    t = np.arange(Nr)
    df.insert(0, "nTrial", ((t - r0) // 100).astype(np.float64))
    y = np.full(Nr, np.nan)
    y[r0:r0 + s.N] = s.y
    df["y"] = y
    return df, ev


def dropin_grid(df, ev, L, K, lams):
    """The drop-in flow timed end to end: sglm_ez.timeshift_cols (lags -L..L-1) -> the NaN-row
    filter -> cv_idx_by_trial_id (seed 3) -> sglm_ez.simple_cv_fit over the 20 Poisson alphas.
    Returns (result dict, per-phase seconds)."""
    import contextlib
    import io
    import torch
    import sglm_ez
    ph = {}
    t = time.perf_counter()
    dfrel = sglm_ez.timeshift_cols(df, ev, neg_order=-L, pos_order=L - 1)
    xcols = sglm_ez.add_timeshifts_to_col_list(ev, ev, neg_order=-L, pos_order=L - 1)
    ph["timeshift_cols"] = time.perf_counter() - t
    t = time.perf_counter()
    dfrel = dfrel[dfrel[["nTrial"] + xcols + ["y"]].isna().sum(axis=1) == 0]
    ph["nan_filter"] = time.perf_counter() - t
    t = time.perf_counter()
    np.random.seed(3)
    cv_idx = sglm_ez.cv_idx_by_trial_id(dfrel, trial_id_columns=["nTrial"], num_folds=K)
    ph["folds"] = time.perf_counter() - t
    t = time.perf_counter()
    kws = [{"model_name": "Poisson", "alpha": float(al)} for al in lams]
    with contextlib.redirect_stdout(io.StringIO()):       # the reference prints per parameter
        out = sglm_ez.simple_cv_fit(dfrel[xcols], dfrel["y"], cv_idx, kws, model_type="Normal")
    torch.cuda.synchronize()
    ph["simple_cv_fit"] = time.perf_counter() - t
    return out[4], ph


def newton_distance(s, design, cv_idx, res, lams, checks, extra=None):
    """float64 Newton distance of a few fits of the last grid to the exact minimiser,
    max_j<p |(H^-1 g)_j| / max_j<p |beta_j| (the coefficients), from the exact design on the
    device (torch float64; outside the timed region)."""
    import torch
    m = s.E.shape[1]
    Ed = torch.from_numpy(s.E).cuda().to(torch.float64)
    kx = 0 if extra is None else extra.shape[0]
    p = s.p + kx
    Xd = torch.empty((s.N, p + 1), dtype=torch.float64, device="cuda")
    r0 = s.L - 1
    for bi, sh in enumerate(s.shifts):
        Xd[:, bi * m:(bi + 1) * m] = Ed[r0 - sh:r0 - sh + s.N]
    if kx:
        Xd[:, s.p:p] = torch.from_numpy(extra.T).cuda()
    Xd[:, p] = 1.0
    yd = torch.from_numpy(s.y).cuda()
    worst = 0.0
    for j, k in checks:
        r = res[j]
        if k < 0:
            coef, b, msk = r["refit_coef"], r["refit_intercept"], None
        else:
            coef, b, msk = r["cv_coefs"][:, k], r["cv_intercepts"][k], cv_idx[k][0]
        w = torch.ones(s.N, dtype=torch.float64, device="cuda")
        if msk is not None:
            w.zero_()
            w[torch.from_numpy(np.asarray(msk)).cuda()] = 1.0
        beta = torch.from_numpy(np.r_[coef, b]).cuda()
        mu = torch.exp(Xd @ beta)
        pen = torch.full((p + 1,), float(lams[j]) * float(w.sum()), dtype=torch.float64,
                         device="cuda")
        pen[-1] = 0.0
        g = Xd.t() @ (w * (mu - yd)) + pen * beta
        H = Xd.t() @ (Xd * (w * mu)[:, None])
        H.diagonal().add_(pen)
        step = torch.linalg.solve(H, g)
        worst = max(worst, float(step[:-1].abs().max()) / float(beta[:-1].abs().max()))
        del H
    del Xd
    torch.cuda.empty_cache()
    return worst


def main():
    a = parse()
    spawn_ranks(a)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    dev = local % max(1, torch.cuda.device_count())   # one rank per GPU; wraps only in rehearsals
    torch.cuda.set_device(dev)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    if a.config in ("c5", "prep", "signal", "designmat", "olsref", "prod50", "cbprod"):
        {"c5": bench_c5, "prep": bench_prep, "signal": bench_signal,
         "designmat": bench_designmat, "olsref": bench_ols, "prod50": bench_ols,
         "cbprod": bench_cb}[a.config](a)
        if world > 1:
            dist.destroy_process_group()
        return
    import ctypes
    from sglm_hip import _lib, engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective

    N, m, L, K, nlam = CONFIGS[a.config]
    t_setup = time.perf_counter()
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    # N > 1: each rank expands only its slab of the rows (row-sharded grid, comm.py), or the
    # whole design when the grid is sharded by fits (SGLM_SHARD=fits)
    if a.shard:
        grid.SHARD_MODE = a.shard
    rows_mode = world > 1 and grid.SHARD_MODE == "rows"
    slab = grid.rank_slab(s.N, rank, world) if rows_mode else None
    extra = synth.prod_counters(s.trial, seed=1) if a.config == "c4mixed" else None
    design = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N, slab=slab, extra=extra)
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
    # the structured Gram's kernel launches bracketed by HIP events inside the library (the
    # roofline divides by the kernel's own time, as rocprofv3 reports it)
    ktimer = E._lagw(design) is not None
    if ktimer:
        _lib.call("sglm_lag_gram_w_timing", 1, None, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step(stats)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # roofline of the dominant kernel (Gram) from HIP events on the launch stream: the whole
    # Gram call (the engine's events) and, for the structured Gram, the kernel alone
    ktime = sum(e0.elapsed_time(e1) for e0, e1, _, _ in stats.syrk_events) / 1e3
    kflop = sum(nact_flop for _, _, _, nact_flop in stats.syrk_events)
    nlaunch = len(stats.syrk_events)
    call_ms = ktime / max(nlaunch, 1) * 1e3
    if ktimer:
        kms, kn = ctypes.c_double(0.0), ctypes.c_int32(0)
        _lib.call("sglm_lag_gram_w_timing", 2, ctypes.byref(kms), ctypes.byref(kn))
        _lib.call("sglm_lag_gram_w_timing", 0, None, None)
        if kn.value > 0:
            ktime, nlaunch = kms.value / 1e3, kn.value
    alg_bytes = float(np.mean(stats.syrk_bytes)) if stats.syrk_bytes else None
    exec_flop = float(np.sum(stats.syrk_exec)) if stats.syrk_exec else None
    t = torch.tensor([elapsed, float(stats.fit_iters), ktime, kflop, float(nlaunch),
                      float(stats.gram_fits), stats.alg_flop, float(stats.reused),
                      float(stats.gram_fit_iters), float(stats.stops["stagnation"]),
                      float(stats.stops["line_search_failed"] + stats.stops["max_iter"]),
                      float(stats.aliased), float(stats.newton_iters), float(stats.shared),
                  float(stats.roundtrips), stats.sync_wait_s, stats.alg_flop_dense],
                     dtype=torch.float64, device="cuda" if a.dist_backend == "nccl" else "cpu")
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        t = sm
        if rows_mode:
            # every rank runs every fit: the fit / Newton / Gram counts and the algorithmic
            # flop are the same on all ranks (not disjoint shares); the Gram launches, their
            # time and flop and the host waits are per rank
            for q in (1, 5, 6, 7, 8, 9, 10, 11, 12, 13, 16):
                t[q] /= world
    fit_iters, ktime, kflop, nlaunch = float(t[1]), float(t[2]), float(t[3]), int(t[4])
    gram_fits, alg_flop, reused, gram_iters = float(t[5]), float(t[6]), float(t[7]), float(t[8])
    stag, failed = int(t[9]), int(t[10])
    aliased, newton_iters = float(t[11]), float(t[12])
    shared, roundtrips, sync_wait = float(t[13]), float(t[14]), float(t[15])
    alg_flop_dense = float(t[16])
    if rank == 0:
        grid_s = elapsed / a.steps
        achieved = kflop / ktime / 1e12 if ktime > 0 else 0.0
        # the Gram kernel that ran: the event-structured one when the design keeps its events
        gram_kernel = "lag_gram_w2_kernel" if E._lagw(design) is not None else "syrk6_kernel"
        traffic, traffic_src = pmc_traffic(gram_kernel)
        conv = all(r["converged"] for r in res)
        ndist = None
        if world == 1 and a.config in ("c4", "c4mixed") and not a.no_check:
            # float64 Newton distance of the lambda = 1e-4 split-0 fit and refit (parity spot
            # check of the timed grid's output; tests/test_gpu_fullsize.py checks every fit)
            ndist = newton_distance(s, design, cv_idx, res, lams, [(0, 0), (0, -1)], extra)
        dropin = None
        if world == 1 and a.config in ("c3", "c4") and not a.no_dropin:
            # the production flow through the drop-in API from a host event DataFrame (the
            # design stays on the device: sglm_hip.lagframe), one warm pass then timed passes
            df, ev = dropin_frame(s)
            dropin_grid(df, ev, L, K, lams)
            walls, phs = [], []
            for _ in range(3):
                torch.cuda.synchronize()
                t_d = time.perf_counter()
                dres, ph = dropin_grid(df, ev, L, K, lams)
                walls.append(time.perf_counter() - t_d)
                phs.append(ph)
            q = int(np.argmin(walls))
            diff = max(float(np.max(np.abs(r["model"].coef_ - g["refit_coef"])) /
                             max(float(np.max(np.abs(g["refit_coef"]))), 1e-30))
                       for r, g in zip(dres["full_cv_results"], res))
            dropin = {"dropin_grid_s": walls[q], "dropin_grid_s_runs": walls,
                      "dropin_over_grid": walls[q] / grid_s,
                      "dropin_phases_ms": {k: v * 1e3 for k, v in phs[q].items()},
                      "dropin_refit_coef_max_rel_vs_grid": diff,
                      "dropin_flow": "host event DataFrame (float64, N_raw rows) -> "
                                     "sglm_ez.timeshift_cols -> isna().sum(axis=1) == 0 row "
                                     "filter -> cv_idx_by_trial_id -> simple_cv_fit"}
        cpu = None
        if not a.no_cpu and world == 1 and extra is None:
            cpu = cpu_reference_grid(s, cv_idx, lams, a.sklearn_rows)
            if a.cpu_full_fold:
                # the planned measurement: one full-size split fit + refit,
                # x 120 fits; the row-sample extrapolation rides along
                full_s, det = cpu_reference_full(s, cv_idx, lams)
                cpu["row_sample_extrapolation_s"] = cpu["value"]
                cpu["row_sample"] = cpu["sample"]
                cpu["value"] = full_s
                lq = det["lambdas"]
                cpu["sample"] = ("sklearn TweedieRegressor(power=1) lbfgs at lambda index "
                                 + ", ".join(str(q["lambda_index"]) for q in lq)
                                 + f": the full-size split-0 train rows ({det['rows'][0]} x "
                                 f"{s.p}) and the full refit ({det['rows'][1]} rows); split fits "
                                 + "/".join(str(q["split_fit_s"]) for q in lq) + " s, refits "
                                 + "/".join(str(q["refit_s"]) for q in lq) + " s, lbfgs iters "
                                 + "/".join(f"{q['lbfgs_iters'][0]}+{q['lbfgs_iters'][1]}"
                                            for q in lq)
                                 + f"; mean of ({len(cv_idx)} x split + refit) x {len(lams)} "
                                 "lambdas")
                cpu["full_fold"] = det
            cpu["port_oracle_newton"] = cpu_port_iter(s, s.N, a.cpu_rows)
        out = {
            "metric": "IRLS iters/sec on 1M×2000 design mat; CV-grid wall-clock (5-fold×20 λ)",
            "value": grid_s,
            "unit": "s per CV grid (5 splits x 20 lambdas + 20 refits = 120 fits)",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": grid_s * 1e3,
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16 Hessian (w rounded to bf16, X exact 0/1) / exact-f32 gradient "
                     "(3 bf16 pieces, f64 slab sums) / f64 coefficients and line search",
            "data": "synthetic",
            "config": {
                "workload": f"Poisson CV grid {s.N}x{design.p} ({m} events x {len(s.shifts)} lags"
                            + (f" + {design.k} continuous counters" if design.k else "")
                            + f"), {K} splits x {nlam} lambdas + refits",
                "config_name": a.config,
                "irls_fit_iters_per_s": fit_iters / elapsed,
                "irls_fit_iters_counted": "fit-iterations incl. aliased / kept-factor ones "
                                          "(those forming their own Gram: "
                                          "gram_forming_fit_iters_per_s)",
                "gram_forming_fit_iters_per_s": gram_iters / elapsed,
                "fit_iters_per_grid": fit_iters / a.steps,
                "gram_forming_fit_iters_per_grid": gram_iters / a.steps,
                "kept_factor_fit_iters_per_grid": reused / a.steps,
                "aliased_fit_iters_per_grid": aliased / a.steps,
                "lambda_shared_fit_iters_per_grid": shared / a.steps,
                # host dependence of the number: round trips (stream synchronisations) per
                # grid, and the host's own time per grid (wall minus the time it sat blocked
                # in those synchronisations; summed over ranks when N > 1)
                "host_roundtrips_per_grid": roundtrips / a.steps / max(world, 1),
                "host_busy_ms_per_grid": (elapsed * (world if world > 1 else 1) - sync_wait)
                                         / a.steps / max(world, 1) * 1e3,
                "newton_iters_per_grid": newton_iters / a.steps,
                "computed_grams_per_grid": gram_fits / a.steps,
                # flop the grid's kernels executed (each Gram at the count of the kernel that
                # formed it: event-structured Grams at their structured products, the event
                # correlations at their histogram adds) / wall / peak
                "grid_roofline_frac": alg_flop / elapsed / (world * PEAK_BF16_TFLOPS * 1e12),
                "grid_roofline_frac_kind": "executed (structured Grams at their own count)",
                # the same grid with every computed Gram charged SURVEY.md §8(d)'s dense
                # n p'(p'+1): the work a dense Gram would have done (not executed here)
                "grid_dense_equiv_frac": alg_flop_dense / elapsed
                                         / (world * PEAK_BF16_TFLOPS * 1e12),
                "all_converged": bool(conv),
                "stagnation_or_failed_stops": stag + failed,
                "newton_dist_f64": ndist,
                **(dropin or {}),
                "setup_s": round(setup_s, 2),
                "parallelism": (f"row slabs over {world} ranks: RCCL all-reduce of the slab "
                                f"Grams, gradients, trial losses and directions" if rows_mode
                                else f"fit shards over {world} rank(s), RCCL all-gather of "
                                     f"results"),
            },
            "roofline": {
                "bound": "mfma",
                "kernel": gram_kernel,
                "achieved": achieved,
                "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_BF16_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_kind": "stored PMC (the committed rocprofv3 --pmc summary named in "
                                "traffic_source, per Gram launch of this grid; PMC counters "
                                "cannot be read inside this process)",
                # PMC bytes over the launch's algorithmic bytes (each compacted design once,
                # the bf16 weights, the upper-triangle f32 output): > 1 = re-read / slab bytes
                "algorithmic_bytes_per_launch": alg_bytes,
                "traffic_over_algorithmic": (traffic / alg_bytes) if (traffic and alg_bytes)
                                            else None,
                "launches": nlaunch,
                "avg_launch_ms": ktime / max(nlaunch, 1) * 1e3,
                "timed": ("the kernel alone (HIP events around each lag_gram_w2_kernel launch "
                          "inside the library, sglm_lag_gram_w_timing)" if ktimer else
                          "the Gram call (HIP events on its stream)"),
                "call_avg_ms": call_ms,
                # the event-structured Gram executes more MFMA work than its algorithmic
                # products (G entries that are no H entry, 32-row / 32-column padding)
                "executed_frac": (exec_flop / ktime / 1e12 / PEAK_BF16_TFLOPS
                                  if (exec_flop and ktime > 0 and world == 1) else None),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
