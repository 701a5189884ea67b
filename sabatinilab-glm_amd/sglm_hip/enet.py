"""Elastic net / Lasso on shared per-mask Grams (MI355X).

Replaces sklearn's cd_fast behind backend/sglm.py:106-110 (ElasticNet / Lasso):
  objective  1/(2n)|y - Xw - b|^2 + alpha rho |w|_1 + alpha (1 - rho)/2 |w|^2
  (sklearn/linear_model/_coordinate_descent.py:420-422), multiplied by n it is
  1/2 w^T Q w - q^T w + l1|w|_1 + l2/2|w|^2 on centred data, l1 = alpha rho n,
  l2 = alpha (1 - rho) n.

Everything that does not depend on the response or the penalty is formed once per row mask:
the exact Gram G_m = X^T diag(m) X (MFMA, W = mask: integer counts, exact for 0/1 designs)
and its centred float64 form Q_m (sglm_center_gram).  Per (response, mask) only
c = X^T (m * y) (MFMA gradient kernel); per fit only q = c_x - g c_p / n and the coordinate
descent (sglm_enet_cd_shared, one workgroup per fit, Q_m shared by index).

``cv_enet_path`` is the multi-response lambda path of SURVEY.md §8(d) C5: for every response
and every alpha, the K split fits and the full refit, scored on the split's test rows from
Gram algebra (|y - Xw - b|^2 over a mask = y'My - 2 beta'c_t + beta' G_t beta with the test
mask's Gram and X^T(m y)), so no linear predictor over n rows is ever formed.  The reference
runs one ``simple_cv_fit`` per response (er_refactored_from_scratch_cleanup.py:388), each
re-fitting sklearn ElasticNet on X[idx] copies (backend/sglm_cv.py:106-131).
"""
from __future__ import annotations

import math
from types import SimpleNamespace
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from . import engine as E
from . import folds as F

CD_TOL = 1e-10


class SharedGrams:
    """Exact Grams (augmented: ones column at p) of a problem's masks, formed on demand."""

    def __init__(self, prob: E.Problem):
        self.prob = prob
        self.d = prob.design
        self.slot = {}                   # mask -> row of self.H
        self.H = None
        self.Q = {}                      # (mask, center) -> row of Qt
        self.Qt = None

    def ensure(self, masks: Sequence[int]):
        need = [int(m) for m in dict.fromkeys(masks) if int(m) not in self.slot]
        if not need:
            return
        d, prob = self.d, self.prob
        old = self.H
        base = 0 if old is None else old.shape[0]
        H = torch.empty((base + len(need), d.P, d.P), dtype=torch.float32, device=d.device)
        if old is not None:
            H[:base].copy_(old)
        W = prob.M[need].to(torch.float32)                   # W = mask multiplicities
        ns = SimpleNamespace(W=W, H=H[base:], prob=prob, fit_mask=np.array(need), wc=None,
                             keep=None)
        E._syrk(d, ns, np.arange(len(need), dtype=np.int32), (d.n + 31) // 32,
                (d.P // 256) * (d.P // 256 + 1) // 2, None, E._stream(), exact=True)
        for i, m in enumerate(need):
            self.slot[m] = base + i
        self.H = H

    def complement(self, parts: dict):
        """Grams of masks that are the difference of two formed ones: parts[m] = (a, b) with
        mask m = mask a - mask b row by row, G_m = G_a - G_b -- exact (integer counts below
        2^24 in f32) when the design is 0/1."""
        need = [m for m in parts if m not in self.slot]
        if not need:
            return
        self.ensure([v for m in need for v in parts[m]])
        base = self.H.shape[0]
        H = torch.empty((base + len(need), self.d.P, self.d.P), dtype=torch.float32,
                        device=self.d.device)
        H[:base].copy_(self.H)
        for i, m in enumerate(need):
            a, b = parts[m]
            torch.sub(H[self.slot[a]], H[self.slot[b]], out=H[base + i])
            self.slot[m] = base + i
        self.H = H

    def centred(self, masks: Sequence[int], center: bool):
        """float64 Q (p x p) per (mask, center); returns the index of each requested mask."""
        self.ensure(masks)
        need = [m for m in dict.fromkeys(int(x) for x in masks) if (m, center) not in self.Q]
        if need:
            d = self.d
            base = 0 if self.Qt is None else self.Qt.shape[0]
            Qt = torch.empty((base + len(need), d.p, d.p), dtype=torch.float64, device=d.device)
            if self.Qt is not None:
                Qt[:base].copy_(self.Qt)
            g = torch.tensor([self.slot[m] for m in need], dtype=torch.int32, device=d.device)
            _lib.call("sglm_center_gram", E._p(self.H), d.P, d.p, E._p(g), len(need),
                      int(center), E._p(Qt[base:]), E._stream())
            for i, m in enumerate(need):
                self.Q[(m, center)] = base + i
            self.Qt = Qt
        return [self.Q[(int(m), center)] for m in masks]

    def sym(self, mask: int):
        """Full symmetric float64 augmented Gram (P x P) of one mask."""
        H = self.H[self.slot[int(mask)]].to(torch.float64)
        up = torch.triu(H)
        return up + torch.triu(H, 1).T


# base-256 digits of the fixed-point m*y in the exact X^T(m y) of 0/1 designs (5 digits: the
# quantisation step is 2^-38 of max|m y| per (response, mask), ~1e-13 of c)
XTY_DIGITS = E.XTV_DIGITS


def xty(prob: E.Problem, pairs: Sequence[tuple]) -> torch.Tensor:
    """c[(r, m)] = X^T (m * y_r) (float64 [len(pairs)][P]; c[p] = sum m y).

    0/1 (and mixed) designs: m*y (float64) is put on a fixed-point grid of 2^-(38 - e)
    (|m y| < 2^e) and split into XTY_DIGITS balanced base-256 digits; each digit plane is an
    integer vector with |digit| <= 128, so the MFMA gradient kernel (sglm_xtr_bits, row slabs
    <= 65,536 rows) sums it EXACTLY in f32 and float64, and c = sum_q 256^q X^T digit_q is
    float64-accurate (engine.xtv_digits) -- the reference's float64 ElasticNet sees X^T y to
    rounding (the f32-accumulated hi/lo passes left ~1e-8 of |c|, which is 2e-5 of alpha rho at
    alpha = 1e-4, C5).  Other designs: y as f32 high and low parts (two exact-product passes,
    f32 accumulation)."""
    d = prob.design
    out = torch.empty((len(pairs), d.P), dtype=torch.float64, device=d.device)
    if d.xbits is not None and E.XTR_BITS:
        return E.xtv_digits(d, prob.M, prob.y64_rows(), pairs, out)
    ylo = prob.y_lo()
    tmp = None if ylo is None else torch.empty((min(256, len(pairs)), d.P), dtype=torch.float64,
                                               device=d.device)
    chunk = 256
    for s in range(0, len(pairs), chunk):
        pr = pairs[s:s + chunk]
        R = torch.stack([prob.M[m].to(torch.float32) * prob.Y[r] for r, m in pr])
        d.xtr(R, len(pr), out[s:s + len(pr)])
        if ylo is not None:
            R = torch.stack([prob.M[m].to(torch.float32) * ylo[r] for r, m in pr])
            d.xtr(R, len(pr), tmp[:len(pr)])
            out[s:s + len(pr)] += tmp[:len(pr)]
    return out


def solve(prob: E.Problem, grams: SharedGrams, fits: Sequence[dict], c: torch.Tensor,
          cidx: Sequence[int], stats: Optional[dict] = None):
    """ElasticNet per fit dict {mask, alpha, l1_ratio, fit_intercept, max_iter} with
    c[cidx[f]] = X^T(m y) of its (response, mask).  Returns (w [B][p] f64, b [B] f64,
    sweeps [B] int, converged [B] bool) as host arrays."""
    p = prob.design.p
    if len(fits) == 0:
        return np.zeros((0, p)), np.zeros(0), np.zeros(0, int), np.zeros(0, bool)
    w, b, sw, conv = solve_arrays(
        prob, grams, np.array([int(f["mask"]) for f in fits]),
        np.array([float(f["alpha"]) for f in fits]), np.array([float(f["l1_ratio"]) for f in fits]),
        np.array([bool(f["fit_intercept"]) for f in fits]),
        max(int(f["max_iter"]) for f in fits), c, np.asarray(cidx), stats)
    return w.cpu().numpy(), b.cpu().numpy(), sw, conv


def solve_arrays(prob: E.Problem, grams: SharedGrams, masks: np.ndarray, alpha: np.ndarray,
                 l1_ratio: np.ndarray, fit_intercept: np.ndarray, max_iter: int,
                 c: torch.Tensor, cidx: np.ndarray, stats: Optional[dict] = None):
    """solve() on per-fit arrays; returns (w [B][p], b [B]) as float64 DEVICE tensors and
    (sweeps, converged) as host arrays."""
    d = prob.design
    p, dev = d.p, d.device
    B = int(masks.size)
    masks = masks.astype(np.int64)
    grams.ensure(np.unique(masks).tolist())
    cnt_m = np.array([float(prob.mask_count(m)) for m in range(int(masks.max()) + 1)])
    cnt = cnt_m[masks]
    q = torch.empty((B, p), dtype=torch.float64, device=dev)
    qidx = np.zeros(B, dtype=np.int32)
    cpv = torch.empty(B, dtype=torch.float64, device=dev)
    gv = torch.zeros((B, p), dtype=torch.float64, device=dev)
    for center in (True, False):
        sel = np.flatnonzero(fit_intercept == center)
        if not sel.size:
            continue
        um, inv = np.unique(masks[sel], return_inverse=True)
        qidx[sel] = np.asarray(grams.centred(um.tolist(), center), dtype=np.int32)[inv]
        sel_t = torch.from_numpy(sel.astype(np.int64)).to(dev)
        cc = c[torch.from_numpy(cidx[sel].astype(np.int64)).to(dev)]
        cpv[sel_t] = cc[:, p]
        if center:
            gslot = torch.from_numpy(np.array([grams.slot[int(m)] for m in um],
                                              dtype=np.int64)[inv]).to(dev)
            g = grams.H[:, :p, p][gslot].to(torch.float64)      # X^T m (upper: rows < p)
            n = torch.from_numpy(cnt[sel]).to(dev)
            gv[sel_t] = g
            q[sel_t] = cc[:, :p] - g * (cc[:, p] / n.clamp_min(1))[:, None]
        else:
            q[sel_t] = cc[:, :p]
    l1 = torch.from_numpy(alpha * l1_ratio * cnt).to(dev)
    l2 = torch.from_numpy(alpha * (1 - l1_ratio) * cnt).to(dev)
    w = torch.empty((B, p), dtype=torch.float64, device=dev)
    sw = torch.empty(B, dtype=torch.int32, device=dev)
    max_sweeps = int(max(int(max_iter), 10000))
    fpw = int(_lib.query("sglm_enet_cd_fits_per_wg", p))
    rec = stats is not None and stats.get("record")
    if rec:                          # the roofline times the CD kernel alone (bench.py)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    if fpw >= 2:
        # fits sharing a Q go to the same workgroups, fpw at a time (padding slots -1);
        # within a Q, fits of equal alpha (other responses) share workgroups: a workgroup
        # sweeps until its last fit converges, and equal penalties converge alike (the
        # near-empty large-alpha fits take one sweep instead of riding along with dense ones)
        order = np.lexsort((np.arange(B), alpha, qidx))           # by Q, then alpha, then index
        qs = qidx[order]
        starts = np.flatnonzero(np.r_[True, qs[1:] != qs[:-1]])
        ends = np.r_[starts[1:], B]
        nwg_q = (ends - starts + fpw - 1) // fpw
        wgf = np.full((int(nwg_q.sum()), fpw), -1, dtype=np.int32)
        wgq = np.repeat(qs[starts], nwg_q).astype(np.int32)
        row = 0
        for s0, e0, nw in zip(starts, ends, nwg_q):
            blk = np.full(nw * fpw, -1, dtype=np.int32)
            blk[: e0 - s0] = order[s0:e0]
            wgf[row:row + nw] = blk.reshape(nw, fpw)
            row += nw
        wgf_d = torch.from_numpy(wgf.reshape(-1)).to(dev)
        wgq_d = torch.from_numpy(wgq).to(dev)
        _lib.call("sglm_enet_cd_grouped", E._p(grams.Qt), p, E._p(wgf_d), int(wgq.size), fpw,
                  E._p(wgq_d), E._p(q), E._p(l1), E._p(l2), max_sweeps, CD_TOL, E._p(w),
                  E._p(sw), E._stream())
    else:
        qidx_d = torch.from_numpy(qidx).to(dev)
        _lib.call("sglm_enet_cd_shared", E._p(grams.Qt), p, E._p(qidx_d), B, E._p(q),
                  E._p(l1), E._p(l2), max_sweeps, CD_TOL, E._p(w), E._p(sw), E._stream())
    if rec:
        ev[1].record()
    fi = torch.from_numpy(np.asarray(fit_intercept, dtype=bool)).to(dev)
    n = torch.from_numpy(cnt).to(dev)
    b = torch.where(fi & (n > 0), (cpv - (gv * w).sum(1)) / n.clamp_min(1), 0.0)
    swh = sw.cpu().numpy()
    if rec:
        # algorithmic work of cyclic CD on a shared Q: every coordinate step reads one row of
        # Q and updates the running gradient, 2p flop, so 2p^2 per sweep per fit (float64)
        stats["cd_ms"] = stats.get("cd_ms", 0.0) + ev[0].elapsed_time(ev[1])
        stats["cd_flop"] = stats.get("cd_flop", 0.0) + 2.0 * p * p * float(np.sum(swh))
    return w, b, swh, swh < max_sweeps


def _mask_sum_y2(prob: E.Problem) -> np.ndarray:
    """[F][R] float64 sum over each mask of m y^2 (sglm_mask_stats with a zero shift)."""
    return _mask_sum_y2_dev(prob).cpu().numpy()


def _mask_sum_y2_dev(prob: E.Problem) -> torch.Tensor:
    """_mask_sum_y2 as a device tensor."""
    Y = prob.y64_rows()
    F_, R = prob.M.shape[0], Y.shape[0]
    n = prob.design.n
    K0 = torch.zeros(R, dtype=torch.float64, device=Y.device)
    out = torch.empty((R, F_, 5), dtype=torch.float64, device=Y.device)
    work = torch.empty(_lib.query("sglm_mask_stats_work_bytes", F_, R, n), dtype=torch.uint8,
                       device=Y.device)
    _lib.call("sglm_mask_stats", E._p(prob.M), prob.M.shape[1], F_, E._p(Y), R, n, E._p(K0),
              -1.0, E._p(out), E._p(work), E._stream())
    return out[:, :, 2].t()


def _test_is_complement(prob: E.Problem, K: int, full: int) -> bool:
    """Every test mask 2k+1 equals the full mask minus train mask 2k (0/1 designs only, Gram
    counts within f32's exact integers)."""
    d = prob.design
    if d.xbits is None or not E.XTR_BITS:
        return False
    M = prob.M[:, :d.n]
    if int(M[full].max()) * d.n >= (1 << 24):
        return False
    tr = M[0:2 * K:2].to(torch.int16)
    te = M[1:2 * K:2].to(torch.int16)
    return bool(((tr + te) == M[full].to(torch.int16)[None, :]).all())


def _assemble(w, b, sw, conv, ss, yyh, cnt, c_pm, R: int, A: int, K: int,
              score_method: str):
    """Per (response, alpha) result dicts from the flat fit arrays, fits ordered (r, j, k) with
    k = 0..K-1 the splits and k = K the refit (cv_enet_path's order); vectorised over all
    (r, j, k).  ss[f] = [train, test] residual sums of squares of split fit f, yyh[m, r] =
    sum over mask m of y_r^2, cnt[m] = rows of mask m (train 2k, test 2k+1), c_pm[r, m] =
    sum over mask m of y_r.  Scores as backend/sglm_cv.py:133-170: r2 = 1 - SS_res / SS_tot
    per split, mse = -SS_res / n; the pooled cv_R2 / cv_mse over the test rows of all splits."""
    p = w.shape[1]
    W5 = w.reshape(R, A, K + 1, p)
    B3 = b.reshape(R, A, K + 1)
    SW = np.asarray(sw).reshape(R, A, K + 1)
    CV = np.asarray(conv).reshape(R, A, K + 1)
    SS = np.asarray(ss).reshape(R, A, K + 1, 2)[:, :, :K, :]
    scores, sst_side, nm_side = [], [], []
    for side in (0, 1):
        mt = 2 * np.arange(K) + side
        nm = cnt[mt]                                               # [K]
        with np.errstate(divide="ignore", invalid="ignore"):
            ym = np.where(nm > 0, c_pm[:, mt] / np.where(nm > 0, nm, 1.0), 0.0)   # [R, K]
            sst = np.maximum(yyh[mt, :].T - nm * ym * ym, 0.0)     # [R, K]
            sres = SS[..., side]                                   # [R, A, K]
            if score_method == "r2":
                sc = np.where(sst[:, None, :] == 0, np.where(sres == 0, 1.0, 0.0),
                              1.0 - sres / sst[:, None, :])
            else:
                sc = -sres / nm
            sc = np.where(nm > 0, sc, np.nan)
        scores.append(sc)
        sst_side.append(sst)
        nm_side.append(nm)
    ss_res = SS[..., 1].sum(2)                                     # [R, A]
    ss_tot = sst_side[1].sum(1)                                    # [R]
    n_te = float(nm_side[1].sum())
    out = []
    for r in range(R):
        per = []
        for j in range(A):
            s_tr, s_te = scores[0][r, j], scores[1][r, j]
            sr, st = float(ss_res[r, j]), float(ss_tot[r])
            per.append({
                "cv_coefs": W5[r, j, :K].T.copy(), "cv_intercepts": B3[r, j, :K].copy(),
                "cv_scores_train": s_tr, "cv_scores_test": s_te,
                "cv_mean_score_train": np.mean(s_tr), "cv_mean_score": np.mean(s_te),
                "cv_std_score": np.std(s_te),
                "cv_R2_score": 0 if st == 0 else 1 - sr / st,
                "cv_mse_score": sr / n_te if n_te else np.nan,
                "refit_coef": W5[r, j, K].copy(), "refit_intercept": float(B3[r, j, K]),
                "n_iter": [int(v) for v in SW[r, j]], "converged": bool(CV[r, j].all()),
            })
        out.append(per)
    return out


def cv_enet_path(X, Y, cv_idx, alphas: Sequence[float], l1_ratio: float = 0.5,
                 fit_intercept: bool = True, max_iter: int = 1000, score_method: str = "mse",
                 stats: Optional[dict] = None, shard: bool = True):
    """Multi-response elastic-net CV path.  Returns ``out[r][j]``: the result dict of
    response r and alpha j with the keys of ``grid.run`` (cv_coefs p x K, cv_intercepts,
    cv_scores_train/test, cv_mean_score_train, cv_mean_score, cv_std_score, cv_R2_score,
    cv_mse_score, refit_coef, refit_intercept, n_iter, converged).

    With torch.distributed initialised the responses are dealt round-robin over the ranks
    (each rank forms the shared Grams of the masks itself) and the per-response results are
    all-gathered once (no data-path collective)."""
    # Y: host (n x R) float64, or a device tensor (kept resident: no upload per call)
    Y = Y.to(torch.float64) if torch.is_tensor(Y) else np.asarray(Y, dtype=np.float64)
    if Y.ndim == 1:
        Y = Y[:, None]
    from .grid import _dist
    dist = _dist() if shard else None
    if dist is not None:
        rank, world = dist.get_rank(), dist.get_world_size()
        mine = list(range(rank, Y.shape[1], world))
        local = {}
        if mine:
            st = {} if stats is not None else None
            res = cv_enet_path(X, Y[:, mine], cv_idx, alphas, l1_ratio, fit_intercept, max_iter,
                               score_method, st, shard=False)
            local = {r: v for r, v in zip(mine, res)}
            if stats is not None:
                stats.update(st)
        gathered = [None] * world
        dist.all_gather_object(gathered, local)
        merged = {}
        for g in gathered:
            merged.update(g)
        return [merged[r] for r in range(Y.shape[1])]
    design = X if isinstance(X, E.Design) else E.Design.from_host(X)
    n, p, dev = design.n, design.p, design.device
    if Y.shape[0] != n:
        raise ValueError(f"Y has {Y.shape[0]} rows, X has {n}")
    R, A, K = Y.shape[1], len(alphas), len(cv_idx)
    masks = []
    for tr, te in F.masks_from_cv_idx(cv_idx, n):
        masks += [tr, te]
    FULL = len(masks)
    masks.append(np.ones(n, np.uint8))
    prob = E.Problem(design, Y, masks)
    grams = SharedGrams(prob)
    pairs = [(r, m) for r in range(R) for m in range(len(masks))]
    if K and _test_is_complement(prob, K, FULL):
        # test mask = all rows - train mask (GroupShuffleSplit partitions the groups): the test
        # Grams and X^T(m y) are differences of the train and full ones, exact for 0/1 designs
        # (integer Gram counts; X^T(m y) float64-accurate), so only K + 1 masks are formed
        formed = [2 * k for k in range(K)] + [FULL]
        n_formed = len(formed)
        grams.ensure(formed)
        grams.complement({2 * k + 1: (FULL, 2 * k) for k in range(K)})
        bpairs = [(r, m) for r in range(R) for m in formed]
        cb = xty(prob, bpairs)
        bi = {pm: i for i, pm in enumerate(bpairs)}
        test = [i for i, (r, m) in enumerate(pairs) if m < FULL and m % 2]
        src = [bi[(r, FULL if (m < FULL and m % 2) else m)] for r, m in pairs]
        c = cb[torch.tensor(src, dtype=torch.int64, device=dev)]
        if test:
            c[torch.tensor(test, dtype=torch.int64, device=dev)] -= cb[torch.tensor(
                [bi[(pairs[i][0], pairs[i][1] - 1)] for i in test], dtype=torch.int64,
                device=dev)]
    else:
        n_formed = len(masks)
        grams.ensure(range(len(masks)))
        c = xty(prob, pairs)
    F_ = len(masks)
    # fits in (response, alpha, split) order, k = K the refit on the full mask; pairs are
    # (response, mask) in r-major order, so pair (r, m) sits at r * F_ + m
    nfit = R * A * (K + 1)
    rr = np.repeat(np.arange(R), A * (K + 1))
    jj = np.tile(np.repeat(np.arange(A), K + 1), R)
    kk = np.tile(np.arange(K + 1), R * A)
    fmask = np.where(kk == K, FULL, 2 * kk)
    al = np.asarray(alphas, dtype=np.float64)[jj]
    w_d, b_d, sw, conv = solve_arrays(prob, grams, fmask, al, np.full(nfit, float(l1_ratio)),
                                      np.full(nfit, bool(fit_intercept)), int(max_iter), c,
                                      rr * F_ + fmask, stats)
    pa = p + 1
    betad = torch.empty((nfit, pa), dtype=torch.float64, device=dev)
    betad[:, :p] = w_d
    betad[:, p] = b_d
    # the coefficients to the host while the scores run (one pinned staging copy)
    wb_h = E._pinned("enet_wb", nfit * pa, torch.float64)[: nfit * pa].view(nfit, pa)
    wb_h.copy_(betad, non_blocking=True)
    # ---- scores from Gram algebra: SS(mask) = y'My - 2 beta'c + beta' G beta (augmented),
    # sum m y^2 per (mask, response) from the mask-statistics kernel, the quadratic forms of
    # the split fits of one mask as one float64 GEMM against that mask's symmetric Gram
    yyd = _mask_sum_y2_dev(prob)                                 # F x R (device)
    cnt = np.array([float(prob.mask_count(m)) for m in range(F_)])
    ssd = torch.zeros((nfit, 2), dtype=torch.float64, device=dev)
    for k in range(K):
        rows = np.flatnonzero(kk == k)
        rows_d = torch.from_numpy(rows).to(dev)
        rr_d = torch.from_numpy(rr[rows]).to(dev)
        Bk = betad[rows_d]                                       # [nf, pa]
        for side, mt in ((0, 2 * k), (1, 2 * k + 1)):
            G = grams.sym(mt)[:pa, :pa]
            quad = ((Bk @ G) * Bk).sum(1)
            lin = (Bk * c[rr_d * F_ + mt, :pa]).sum(1)
            ssd[rows_d, side] = (yyd[mt, rr_d] - 2.0 * lin + quad).clamp_min(0.0)
    yyh = yyd.cpu().numpy()
    c_pm = c[:, p].cpu().numpy().reshape(R, F_)                  # sum m y per (r, m) pair
    ss = ssd.cpu().numpy()
    torch.cuda.current_stream().synchronize()                   # the pinned coefficients
    wb = wb_h.numpy()
    w, b = wb[:, :p], wb[:, p]
    out = _assemble(w, b, sw, conv, ss, yyh, cnt, c_pm, R, A, K, score_method)
    if stats is not None:
        stats.update({"fits": nfit, "grams": len(masks), "grams_formed": n_formed,
                      "xty_columns": len(pairs),
                      "cd_sweeps_total": int(np.sum(sw)), "cd_sweeps_max": int(np.max(sw))})
    return out
