"""Batched (split x hyper-parameter) CV grid on the MI355X.

Restates the arithmetic of ``cv_glm_single_params`` / ``cv_glm_mult_params``
(backend/sglm_cv.py:42-206, 210-428) with GLM.fit_set (backend/sglm.py:254-312):

* every (param j, split k) cell is one fit on the train rows of split k with response
  ``np.roll(y, roll_j)`` (:95-96); every param adds one full-data refit on UN-rolled y
  (:180-181) — all of them in one batched IRLS over a single resident X (no
  ``X[idx_train, :]`` copies, :107-110);
* train/test scores are the GLM ``score`` of the chosen ``score_method`` ('mse' ->
  -mean((y - mu)^2), 'r2' -> R^2 or D^2), computed from device row sums
  (sglm_score_sums) plus float64 mask statistics;
* ``cv_R2_score`` pools the test residuals of all splits against per-split test means
  (calc_R2 over concatenations, :196), ``cv_mse_score`` = mean squared pooled residual.

Fits are independent, so with ``torch.distributed`` initialised the fit list is cut into
contiguous, row-cost-balanced chunks of a mask-major order (``shard_plan``: each rank holds
few masks, so it compacts and first-iterates few of them) and the per-fit results are
all-gathered (one RCCL collective over xGMI at the end).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import numpy as np

from . import engine as E
from . import folds as F
from .estimators import Objective


class _MaskStats:
    """float64 statistics of every (response, mask) pair that the scores and the y-range check
    need: count, mean, sum of squares about the mean, min y; per Tweedie power the summed
    loss constant and null deviance.  One pass of sglm_mask_stats over the device masks and
    responses per power (the reference computes them per fold on host copies,
    backend/sglm.py:150-184, 388-408)."""

    def __init__(self, prob: E.Problem, comm=None):
        import torch
        from . import _lib
        self.torch, self._lib = torch, _lib
        self.prob = prob
        self.comm = comm
        n, dev = prob.design.n, prob.design.device
        self.Yd = prob.y64_rows()                        # R x n float64 (device)
        self.F, self.R, self.n = prob.M.shape[0], self.Yd.shape[0], n
        if comm is None:
            self.Kd = self.Yd.mean(dim=1)                # per-response shift
        else:                                            # the global mean over all slabs
            tot = self.Yd.sum(dim=1)
            comm.sum_(tot)
            d = prob.design
            self.Kd = tot / float(d.n if d.slab is None else d.slab[2])
        self.K = self.Kd.cpu().numpy()
        self.work = torch.empty(_lib.query("sglm_mask_stats_work_bytes", self.F, self.R, n),
                                dtype=torch.uint8, device=dev)
        st = self._pass(-1.0)                             # [R][F][5]
        cnt = st[0, :, 0]
        a1, a2 = st[:, :, 1].T, st[:, :, 2].T             # F x R
        safe = np.where(cnt > 0, cnt, 1.0)[:, None]
        self.cnt = cnt
        self.sy = a1 + self.K[None, :] * cnt[:, None]
        self.mean = np.where(cnt[:, None] > 0, self.sy / safe, 0.0)
        self.sst = np.maximum(a2 - a1 * a1 / safe, 0.0) * (cnt[:, None] > 0)
        self.ymin = st[:, :, 4].T
        self.c = {}
        self._const = {}

    def _pass(self, power):
        torch, _lib, prob = self.torch, self._lib, self.prob
        out = torch.empty((self.R, self.F, 5), dtype=torch.float64, device=self.Yd.device)
        _lib.call("sglm_mask_stats", prob.M.data_ptr(), prob.M.shape[1], self.F,
                  self.Yd.data_ptr(), self.R, self.n, self.Kd.data_ptr(), float(power),
                  out.data_ptr(), self.work.data_ptr(), E._stream())
        if self.comm is not None:
            # counts, centred sums and loss constants add over the slabs; min y is a minimum
            sums, ymin = out[:, :, :4].contiguous(), out[:, :, 4].contiguous()
            self.comm.sum_(sums)
            self.comm.min_(ymin)
            out = torch.cat([sums, ymin[:, :, None]], dim=2)
        return out.cpu().numpy()

    def _consts(self, power):
        """Summed per-row loss constant of each (mask, response) for one Tweedie power."""
        if power not in self._const:
            self._const[power] = self._pass(float(power))[:, :, 3].T      # F x R
        return self._const[power]

    def get(self, r, m, power=None):
        key = (r, m, power)
        if key in self.c:
            return self.c[key]
        cnt = float(self.cnt[m])
        ym = float(self.mean[m, r])
        out = {"cnt": cnt, "mean": ym, "sst": float(self.sst[m, r]), "ymin": float(self.ymin[m, r])}
        if power is not None and cnt:
            out["const"] = float(self._consts(power)[m, r])
            sy = float(self.sy[m, r])
            if ym > 0:                   # sum of half_loss(y, log(mean)) in closed form
                if power == 1:
                    out["null"] = cnt * ym - math.log(ym) * sy
                elif power == 2:
                    out["null"] = cnt * math.log(ym) + sy / ym
                else:
                    out["null"] = (cnt * ym ** (2 - power) / (2 - power)
                                   - sy * ym ** (1 - power) / (1 - power))
            else:
                out["null"] = np.inf
        self.c[key] = out
        return out


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return dist
    except Exception:  # pragma: no cover
        pass
    return None


SHARD_PLAN = "mask_major"                    # or "round_robin" (comparison runs)
# "fits" (default): whole fits (cross-mask families) per rank with one all-gather of the
# results; "rows": a process group splits the rows of the grid (every rank runs every fit on
# its slab, sums all-reduced; comm.py).  Simulated C4 shares at 2 / 4 / 8 ranks are equal within
# 1 ms before the row mode's ~60 collectives per grid (profiles/r03_rank_shares*.json), so the
# mode without a data-path collective is the default and the row mode is opt-in
# (SGLM_SHARD=rows) -- it is balanced by construction and its floor is one slab's latency.
SHARD_MODE = os.environ.get("SGLM_SHARD", "fits")


def rank_slab(n: int, rank: Optional[int] = None, world: Optional[int] = None):
    """Rows [start, stop) of a rank's slab of an n-row design in a row-sharded grid (the
    current process group's rank / world by default)."""
    from .comm import row_slab
    if rank is None or world is None:
        d = _dist()
        rank, world = (d.get_rank(), d.get_world_size()) if d else (0, 1)
    return row_slab(n, rank, world)


def row_sharded(groups=None) -> bool:
    """True when a grid run now (process group of > 1 rank) splits rows, not fits."""
    if _dist() is None or SHARD_MODE != "rows":
        return False
    return groups is None or all(o.kind == "irls" for g in groups for o in g["objectives"])


def shard_indices(total: int, rank: int, world: int):
    """Round-robin deal of a list over ranks (item i -> rank i mod world)."""
    return [i for i in range(total) if i % world == rank]


def snake(j: int, count: int) -> int:
    """Position of parameter j in the order 0, count-1, 1, count-2, ...: neighbours in this
    order pair a weakly and a strongly penalised fit, so contiguous chunks of it mix fits
    that need many and few Newton iterations."""
    return 2 * j if j < (count + 1) // 2 else 2 * (count - 1 - j) + 1


def shard_plan(keys: Sequence[tuple], costs: Sequence[float], rank: int, world: int):
    """Indices of the fits rank ``rank`` of ``world`` solves: the fits sorted by ``keys``
    (mask-major), then cut into ``world`` contiguous chunks of near-equal summed cost (a fit
    goes to the chunk holding the midpoint of its cost interval).  Every fit lands on exactly
    one rank; a rank's fits share few row masks, so its first Newton iteration (all fits of
    one mask start from the same coefficients) and its per-mask bit-plane compaction cover
    few masks instead of all of them, as a round-robin deal would."""
    order = sorted(range(len(keys)), key=lambda i: keys[i])
    c = np.asarray([float(costs[i]) for i in order])
    total = c.sum()
    if world <= 1 or total <= 0:
        return sorted(order) if world <= 1 else shard_indices(len(keys), rank, world)
    mid = np.cumsum(c) - 0.5 * c
    owner = np.minimum((mid * world / total).astype(np.int64), world - 1)
    return sorted(order[q] for q in range(len(order)) if owner[q] == rank)


def merge_results(local: dict, dist=None) -> dict:
    """All-gather every rank's {fit index: result} and merge (one collective per grid)."""
    if dist is None:
        return local
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, local)
    out = {}
    for g in gathered:
        out.update(g)
    return out


def run(X, y, cv_idx, objectives: Sequence[Objective], rolls: Sequence[int],
        score_method: str = "mse", coef0=None, intercept0=None, stats=None, shard=True,
        simulate=None):
    """Return one result dict per objective (reference key set minus glm_kwargs/model).

    ``simulate=comm.SimComm`` (development only): one rank's slab of a row-sharded grid
    (or, with ``SimComm.recorder()`` and the full design, the recording it replays).
    ``simulate=(rank, world)`` (development only) solves just that rank's share without a
    process group and returns the raw per-fit results instead of the assembled dicts."""
    out = run_multi(X, y, [{"cv_idx": cv_idx, "objectives": objectives, "rolls": rolls}],
                    score_method, coef0, intercept0, stats, shard, simulate)
    return out if simulate is not None else out[0]


def plan_fits(groups: Sequence[dict], n: int, check: bool = True):
    """Host-side plan of a (multi-)grid, identical on every rank: the row-mask specs, per
    group its ([(train, test)] mask ids, refit mask, holdout mask), the masks' row counts, the
    fit table -- per group, (param j, split k) then refit (j, -1) as (group, j, k, fit mask,
    response, second score mask) -- and the sorted roll list (responses)."""
    specs, mkey = [], {}
    dedup = len(groups) > 1                  # one grid's masks are distinct by construction

    def add_spec(idx, multiplicity):
        """idx: row indices (None = every row); multiplicity: repeats count (fold lists)."""
        if dedup:                            # resplit grids share masks: dedup by content
            a = _mask_array(idx, multiplicity, n)
            k = a.tobytes()
            if k not in mkey:
                mkey[k] = len(specs)
                specs.append((idx, multiplicity, a))
            return mkey[k]
        specs.append((idx, multiplicity, None))
        return len(specs) - 1

    gm = []
    for g in groups:
        splits = [(add_spec(tr, True), add_spec(te, True)) for tr, te in g["cv_idx"]]
        refit = add_spec(g.get("refit_rows"), False)
        hold = g.get("holdout_rows")
        gm.append((splits, refit, -1 if hold is None else add_spec(hold, False)))
    counts = [_mask_count(sp[0], sp[1], n, check) for sp in specs]
    roll_list = sorted(set(int(r) for g in groups for r in g["rolls"]) | {0})
    ridx = {r: i for i, r in enumerate(roll_list)}
    table = []
    for gi, g in enumerate(groups):
        splits, refit, hold = gm[gi]
        for j, (obj, roll) in enumerate(zip(g["objectives"], g["rolls"])):
            for k, (tr, te) in enumerate(splits):
                table.append((gi, j, k, tr, ridx[int(roll)], te))
            table.append((gi, j, -1, refit, 0, hold))
    return specs, gm, counts, table, roll_list


def rank_share(plan, groups: Sequence[dict], rank: int, world: int):
    """Fit-table indices rank ``rank`` of ``world`` solves (mask-major cost-balanced chunks)."""
    specs, gm, counts, table, roll_list = plan
    if world > 1 and SHARD_PLAN == "round_robin":
        return shard_indices(len(table), rank, world)
    units = {}
    for i, t in enumerate(table):
        units.setdefault((t[0], t[1]), []).append(i)
    fam = (world > 1 and SHARD_PLAN == "mask_major" and E.HESS_XMASK_TOL > 0
           and len(units) >= world
           and all(o.kind == "irls" and o.family == E.FAM_TWEEDIE_LOG
                   for g in groups for o in g["objectives"]))
    if fam:
        # whole parameters (a penalty's split fits + refit: one cross-mask family, solved on
        # the refit's factor) per rank, in snake order of the penalty list, cut into
        # contiguous runs of near-equal count
        njs = [len(g["objectives"]) for g in groups]
        order = sorted(units, key=lambda u: (snake(u[1], njs[u[0]]), u[0]))
        cuts = np.linspace(0, len(order), world + 1).round().astype(int)
        return sorted(i for u in order[cuts[rank]:cuts[rank + 1]] for i in units[u])
    if world > 1:
        njs = [len(g["objectives"]) for g in groups]
        keys = [(t[3], t[4], snake(t[1], njs[t[0]]), t[0], t[1]) for t in table]
        costs = [counts[t[3]] for t in table]
        return shard_plan(keys, costs, rank, world)
    return list(range(len(table)))


def run_multi(X, y, groups: Sequence[dict], score_method: str = "mse", coef0=None,
              intercept0=None, stats=None, shard=True, simulate=None):
    """Several CV grids over ONE resident design, solved as one batch (SURVEY.md §8(f) 2:
    holdout resplits).  Each group: ``cv_idx`` (global row indices), ``objectives``,
    ``rolls``, optional ``refit_rows`` (the refit's rows; default all) and ``holdout_rows``
    (rows the refits are also scored on).  Returns one list of per-param dicts per group;
    with ``holdout_rows`` every dict also carries ``refit_holdout_r2`` (R^2 / D^2) and
    ``refit_holdout_neg_mse`` — what ``training_fit_holdout_score`` reports for that param."""
    import time
    tick = stats.mark if (stats is not None and (stats.trace_phases or stats.host_phases)) \
        else (lambda name, t: t)
    t0 = tick("-", time.perf_counter())
    from .comm import RowComm, SimComm, row_slab
    dist = _dist() if shard and simulate is None else None
    irls_only = all(o.kind == "irls" for g in groups for o in g["objectives"])
    comm = None
    if isinstance(simulate, SimComm):
        comm = simulate                          # one rank of a row-sharded solve, simulated
    elif (dist is not None and SHARD_MODE == "rows" and irls_only
          and not (isinstance(X, E.Design) and X.slab is None)):
        # host X is packed per slab here; a device Design must already be this rank's slab
        # (Design.from_events / from_host with slab=grid.rank_slab(n)) -- a full Design in a
        # process group is sharded by fits instead
        comm = RowComm(dist)
    if isinstance(X, E.Design):
        design = X
    else:
        design = E.Design.from_host(X, slab=None if comm is None else row_slab(
            np.asarray(X).shape[0], comm.rank, comm.world))
    if design.slab is not None and comm is None:
        raise ValueError("a slab design needs a row-sharded process group (or a SimComm)")
    if comm is not None and comm.world > 1 and (design.slab is None or row_slab(
            design.slab[2], comm.rank, comm.world) != tuple(design.slab[:2])):
        raise ValueError(f"design slab {design.slab} is not rank {comm.rank}/{comm.world}'s "
                         "row slab (grid.rank_slab)")
    n = design.n if design.slab is None else design.slab[2]
    p = design.p
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if y.shape[0] != n:
        raise ValueError(f"y has {y.shape[0]} rows, X has {n}")
    # one process builds every mask (no process group, or a row-sharded one): the mask builder
    # checks the fold indices; ranks that build only their own masks check all of them here so
    # that a bad index raises on every rank together
    single = dist is None or comm is not None
    plan = plan_fits(groups, n, check=not single)
    specs, gm, counts, table, roll_list = plan
    t0 = tick("grid_setup", t0)
    if comm is not None:
        # row-sharded: every rank runs every fit over its slab of the rows
        mine = list(range(len(table)))
    else:
        rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (simulate or (0, 1))
        mine = rank_share(plan, groups, rank, world)

    # only the masks (and responses) of this rank's fits are built and uploaded
    used = sorted({table[i][3] for i in mine} | {table[i][5] for i in mine if table[i][5] >= 0})
    local = {mid: q for q, mid in enumerate(used)}
    try:
        prob = E.Problem.from_index_lists(design, y, roll_list,
                                          [(specs[mid][0], specs[mid][1]) for mid in used])
    except ValueError as e:
        if single and "outside" in str(e):
            raise IndexError(str(e)) from None         # numpy's X[idx] error type
        raise
    t0 = tick("setup_problem", t0)
    ms = _MaskStats(prob, comm)
    for i in mine:                           # the IRLS setup reads these, not host passes
        _, _, _, m, r, _ = table[i]
        prob.seed_stats(r, local[m], float(ms.cnt[local[m]]), float(ms.sy[local[m], r]))
    # sklearn's y-range check of the log-link fits (y >= 0 on the fit's rows, positive mean;
    # glm.py:231-235), on this rank's fits from the device mask statistics; the verdict is
    # shared (one int all-reduce) so that every rank raises together
    bad = 0
    for i in mine:
        _, _, _, m, r, _ = table[i]
        if groups[table[i][0]]["objectives"][table[i][1]].family == E.FAM_TWEEDIE_LOG:
            st_ = ms.get(r, local[m])
            bad |= int(bool(st_["cnt"]) and (st_["ymin"] < 0 or st_["mean"] <= 0))
    if dist is not None and comm is None:
        import torch
        flag = torch.tensor([bad], dtype=torch.int32,
                            device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        bad = int(flag.item())
    if bad:
        raise ValueError("Some value(s) of y are out of the valid range of the loss "
                         "'HalfPoissonLoss'.")
    t0 = tick("setup_maskstats", t0)

    def objective(i):
        return groups[table[i][0]]["objectives"][table[i][1]]

    results = {}
    solve_groups = {}
    for i in mine:
        obj = objective(i)
        key = ("cd", 0.0) if obj.kind == "cd" else (obj.family, float(obj.power))
        solve_groups.setdefault(key, []).append(i)
    for key, idxs in solve_groups.items():
        reqs = []
        for i in idxs:
            _, _, _, m, r, _ = table[i]
            obj = objective(i)
            cnt = counts[m]
            reqs.append(E.FitReq(obj.family, obj.power, obj.lam(cnt), local[m], r,
                                 obj.fit_intercept, obj.max_iter,
                                 None if coef0 is None else np.asarray(coef0, float),
                                 None if intercept0 is None else float(intercept0)))
        t0 = tick("fit_table", t0)
        sets = np.array([[local[table[i][3]], local.get(table[i][5], -1)] for i in idxs],
                        dtype=np.int32)
        if key[0] == "cd":
            from . import cd
            res, eta = cd.enet_batch(prob, [objective(i) for i in idxs], reqs)
            sums = E.score_sums(prob, E.FAM_SQUARED, 0.0, eta, [table[i][4] for i in idxs],
                                sets)
        else:
            res, sums = E.irls_scored(prob, reqs, sets, stats=stats, comm=comm)
        t0 = tick("solve", t0)
        for q, i in enumerate(idxs):
            rr = res[q]
            _, _, k, m, r, mt = table[i]
            obj = objective(i)
            pw = obj.power if obj.family == E.FAM_TWEEDIE_LOG else None
            sc = {}
            if k < 0:
                if mt >= 0:
                    sth = ms.get(r, local[mt], pw)
                    sc["hold"] = (_score("r2", obj, sums[q][1], sth),
                                  _score("mse", obj, sums[q][1], sth))
            else:
                st_te = ms.get(r, local[mt], pw)
                sc["train"] = _score(score_method, obj, sums[q][0], ms.get(r, local[m], pw))
                sc["test"] = _score(score_method, obj, sums[q][1], st_te)
                sc["ss_res"] = float(sums[q][1][0])
                sc["sst"], sc["cnt_te"] = st_te["sst"], st_te["cnt"]
            results[i] = (rr.coef, rr.intercept, rr.n_iter, rr.converged, sc)
    t0 = tick("score_sums", t0)
    if simulate is not None:
        return results
    if comm is None:
        results = merge_results(results, dist)

    out_all = assemble(groups, plan, results, p)
    tick("assemble", t0)
    return out_all


def assemble(groups: Sequence[dict], plan, results: dict, p: int):
    """Per-param result dicts (reference key order, backend/sglm_cv.py:188-200) of every group
    from the merged per-fit results {table index: (coef, intercept, n_iter, converged, scores)}."""
    specs, gm, counts, table, roll_list = plan
    rows = {}                                   # (group, param) -> [(table index, split)]
    for i, t in enumerate(table):
        rows.setdefault((t[0], t[1]), []).append((i, t[2]))
    out_all = []
    for gi, g in enumerate(groups):
        K = len(gm[gi][0])
        out = []
        for j, obj in enumerate(g["objectives"]):
            cv_coefs = np.zeros((p, K))
            cv_b = np.zeros(K)
            s_tr = np.zeros(K)
            s_te = np.zeros(K)
            ss_res = ss_tot = n_te = 0.0
            n_iter = []
            conv = True
            refit = None
            hold_scores = None
            for i, k in rows.get((gi, j), ()):
                coef, b, it, cv_ok, sc = results[i]
                n_iter.append(it)
                conv &= cv_ok
                if k < 0:
                    refit = (coef, b)
                    hold_scores = sc.get("hold")
                    continue
                cv_coefs[:, k] = coef
                cv_b[k] = b
                s_tr[k] = sc["train"]
                s_te[k] = sc["test"]
                ss_res += sc["ss_res"]
                ss_tot += sc["sst"]
                n_te += sc["cnt_te"]
            d = {
                "cv_coefs": cv_coefs,
                "cv_intercepts": cv_b,
                "cv_scores_train": s_tr,
                "cv_scores_test": s_te,
                "cv_mean_score_train": np.mean(s_tr),
                "cv_mean_score": np.mean(s_te),
                "cv_std_score": np.std(s_te),
                "cv_R2_score": 0 if ss_tot == 0 else 1 - ss_res / ss_tot,
                "cv_mse_score": ss_res / n_te if n_te else np.nan,
                "refit_coef": refit[0],
                "refit_intercept": refit[1],
                "n_iter": n_iter,
                "converged": conv,
            }
            if hold_scores is not None:
                d["refit_holdout_r2"], d["refit_holdout_neg_mse"] = hold_scores
            out.append(d)
        out_all.append(out)
    return out_all


def _mask_array(idx, multiplicity, n):
    """uint8 mask of one spec: fold index lists count repeats (holdout resampling), row lists
    (refit / holdout rows) mark rows; None = every row."""
    if idx is None:
        return np.ones(n, np.uint8)
    if multiplicity:
        return F.mask_from_idx(idx, n)
    m = np.zeros(n, np.uint8)
    m[F.wrap_indices(idx, n)] = 1
    return m


def _mask_count(idx, multiplicity, n, check=True):
    """Row count of a spec (sum of multiplicities) without building the mask.  ``check`` =
    False leaves a fold list's range check to the mask builder (one process builds every mask
    of the grid: sglm_host_masks checks each index while it writes the row)."""
    if idx is None:
        return float(n)
    if multiplicity:
        # a fold list counts every entry: only the range check (numpy's IndexError), no wrap
        a = np.asarray(idx).reshape(-1)
        if check and a.size and (a.min() < -n or a.max() >= n):
            F.wrap_indices(a, n)                             # raises with numpy's message
        return float(a.size)
    return float(np.unique(F.wrap_indices(idx, n)).size)


def _score(method, obj: Objective, sums, st):
    s2, sl = sums
    cnt = st["cnt"]
    if cnt == 0:
        return np.nan
    if method != "r2":
        return -s2 / cnt
    if obj.family == E.FAM_SQUARED:
        if st["sst"] == 0:
            return 1.0 if s2 == 0 else 0.0
        return 1.0 - s2 / st["sst"]
    return 1.0 - (sl + st["const"]) / (st["null"] + st["const"])
