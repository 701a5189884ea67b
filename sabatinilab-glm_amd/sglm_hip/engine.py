"""Batched IRLS engine on MI355X (host driver of libsglm_hip).

One call to :func:`irls` runs B independent fits — the (fold x lambda) cells of a CV grid,
or a single ``GLM.fit`` — against ONE resident design matrix.  Each fit differs only in
its row mask (train rows of its fold, as multiplicities), its response column (``roll``),
its penalty and its family.  The reference runs these as separate sklearn fits on copies
``X[idx_train, :]`` (backend/sglm_cv.py:106-131); here the copies never exist.

Per batched Newton iteration (all device work on the current torch stream):

  link_update   W = m * loss''(eta), R = m * loss'(eta)              (elementwise)
  xtr           g = X^T R  (f32 MFMA, float64 reduction) + lam * beta  (gradient)
  syrk          H = X^T diag(W) X  for the still-active fits          (bf16 MFMA)
  chol_solve    delta = -(H + lam I')^-1 g                           (per-fit Cholesky)
  gemv_eta      d_eta = X delta
  loss_trials   Armijo line search on sum m*loss(eta + t d_eta) + lam/2 |w + t d|^2
  eta_axpy      eta += t d_eta

The Hessian is only an approximation (bf16 operands, f32 factor); the gradient and the
objective are computed from exact X in f32/f64, so the fixed point is the exact minimiser
(inexact Newton, SURVEY.md §7 "Hard parts").  Gaussian (squared-loss) fits have a
Hessian that depends only on the mask: it is formed once per distinct mask and its factor
is reused by the refinement iterations.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib

try:
    import torch
except ImportError as e:  # pragma: no cover - torch is part of the image
    raise _lib.HipEngineUnavailable("PyTorch-ROCm is required for device memory") from e

FAM_SQUARED = 0
FAM_TWEEDIE_LOG = 1
X_BF16, X_F32 = 0, 1
COL_PAD = 256
ROW_PAD = 256
ARMIJO_SIGMA = 2.0 ** -11      # sklearn _newton_solver.py:214
# stopping rule: max|t d| <= STOP_TOL * max(max_j<p |w_j|, STOP_SCALE_FLOOR) on the
# coefficients, |t d| <= STOP_TOL on the intercept.  3e-6 (round 6; 1e-6 since round 3): the
# worst float64 Newton distance over the C4 grid's 120 fits is 3.1e-7 of max|coef| (1.1e-7 at
# 1e-6, 5.1e-6 at 1e-5), 30x inside the full-size test's 1e-5 and 300x inside the north star's
# Poisson 1e-4, for 590 -> 580 fit-iterations (C4 28.92 -> 28.31 ms; profiles/r06b_stop_tol.json)
STOP_TOL = float(__import__("os").environ.get("SGLM_STOP_TOL", "3e-6"))
STOP_SCALE_FLOOR = float(__import__("os").environ.get("SGLM_STOP_SCALE_FLOOR", "0.1"))
# round-2 rule, for comparison runs: max|t d| <= tol * (1 + max|w|), intercept included
STOP_LEGACY = __import__("os").environ.get("SGLM_STOP_RULE", "") == "legacy"
# second round of line-search step lengths (the first: 1, 1/2, 1/4, 1/8)
TV2 = np.array([0.0625, 0.03125, 0.015625, 0.0078125, 2.0 ** -10, 2.0 ** -14, 2.0 ** -20])
XTR_BITS = True                # X^T R on the MFMA from compacted bit-planes for 0/1 designs
# X^T R of a time-shifted 0/1 event design (Design.from_events) from the event occurrences
LAG_XTR = __import__("os").environ.get("SGLM_LAG_XTR", "0") == "1"
ETA_BITS = True                # eta on the MFMA from row-major bit-planes for 0/1 designs
ETA_FINAL_ALL = False          # recompute every fit's final eta (else only ETA_FINAL_ITERS+)
ETA_FINAL_ITERS = 8
# the Newton decisions (stage-1 Armijo, stopping rule) on the device (sglm_step_decide), the
# step and the next link enqueued before the host reads the iteration back.  Off by default:
# measured slower on the C4 grid (47.9 vs 46.8 ms, interleaved A/B on one box) -- the link then
# runs over every active fit, stopped ones included, and the host still waits for the next
# Hessian plan's readback behind it, so little host time leaves the critical path
DEV_DECIDE = __import__("os").environ.get("SGLM_DEV_DECIDE", "0") == "1"
# the Anderson correction as one kernel (sglm_aa_step) instead of ~20 torch operations
# (C4 grid 35.26 -> 34.69 ms, interleaved A/B with the event-structured Gram)
AA_KERNEL = __import__("os").environ.get("SGLM_AA_KERNEL", "1") == "1"
SYRK_CBITS = True              # ... and its row-compacted register-only form (v6) when fits
                               # carry masks (the default path for event designs)
# the Gram of a time-shifted 0/1 event design from its events (sglm_lag_gram_w: one matrix
# product per event over its occurrences, 2 rho of the dense Gram's products at event density
# rho) when the design keeps its event structure and the events are sparse enough
LAG_GRAM_W = __import__("os").environ.get("SGLM_LAG_GRAM_W", "1") == "1"
LAG_GRAM_W_MAX_RHO = 0.2        # above it the dense bit-plane Gram does fewer products
# ... also for mixed designs (their continuous rows / columns from _mix_hess after it)
# (c4mixed 49.4 -> 35.1 ms = 1.10x the C4 grid; tests/test_gpu_mixed.py green)
LAG_GRAM_W_MIXED = __import__("os").environ.get("SGLM_LAG_GRAM_W_MIXED", "1") == "1"
# Hessian reuse (log-link families): a fit keeps its last Hessian factor while the drift of
# its linear predictor since that Hessian was formed, D = sum of max_i |t d_eta_i| over the
# steps taken since, stays <= HESS_REUSE_TOL.  The IRLS weights then differ from the ones the
# factor holds by a factor in [e^-cD, e^cD] (c = max(1, |2 - power|)), which bounds the
# contraction of the inexact-Newton step by e^cD - 1; the fixed point (exact gradient) is
# unchanged.  0 disables reuse.
HESS_REUSE_TOL = float(__import__("os").environ.get("SGLM_HESS_REUSE_TOL", "0.375"))
# Hessian sharing: among fits of one (mask, response) that need a new Hessian, a fit whose
# predictor is within HESS_SHARE_TOL (max over its mask rows) of another's is factored from
# that fit's Gram, and starts its drift count at that distance (same bound as above).
HESS_SHARE_TOL = float(__import__("os").environ.get("SGLM_HESS_SHARE_TOL", "0.375"))
# Cross-mask Hessian sharing (log-link families): the fits of one penalty (alpha per row),
# response and intercept setting -- a lambda's CV split fits and its full-data refit -- differ
# only in their row masks.  A split fit k is solved on the factor of the member with the most
# rows ("representative") scaled by the row-count ratio, c_k (G_rep + alpha n_rep I') =
# c_k G_rep + alpha n_k I', while its predictor stays within XMASK_TOL (max over its rows) of
# the representative's; the generalized eigenvalues of (H_k, c_k H_rep) measured at the
# solutions of the C3 grid lie in [0.92, 1.10] (contraction <= 0.1).  A fit whose aliased
# step fails the line search or contracts slowly leaves the family for good.  0 disables.
HESS_XMASK_TOL = float(__import__("os").environ.get("SGLM_HESS_XMASK_TOL", "0.75"))
XMASK_SLOW = 0.7                # aliased-step contraction above which a fit leaves its family
# Newton solves on explicit factor inverses (sglm_chol_solve_inv: two full-chip GEMMs per
# iteration over every fit, grouped by factor) instead of per-fit triangular substitution
# chains; 0 restores sglm_chol_solve_mixed / sglm_chol_solve_alias.
SOLVE_INV = __import__("os").environ.get("SGLM_SOLVE_INV", "1") == "1"
# where the factorisation chain runs: "side" (its own stream, overlapping the gradient),
# "prio" (the same at high stream priority), "serial" (the main stream, before the gradient)
CHOL_STREAM = __import__("os").environ.get("SGLM_CHOL_STREAM", "side")
# secant (Anderson-1) correction of directions on an unchanged stale factor: the tail of a
# grid runs on kept / aliased factors converging linearly at 0.08-0.17 per iteration; the
# correction extrapolates along the secant (C4: 9 -> 7 Newton iterations, 636 -> 589
# fit-iterations, 51.4 -> 50.3 ms in one process; the fixed point is the exact gradient's)
ANDERSON = __import__("os").environ.get("SGLM_ANDERSON", "1") == "1"
# first iteration: link + gradient once per (mask, response, intercept) start key, the other
# fits' gradient rows copied (bitwise the same values; round 6)
GRAD_DEDUP = __import__("os").environ.get("SGLM_GRAD_DEDUP", "1") == "1"
# a batch of >= DEFER_INV_MIN new factorisations is solved on its fresh factors by substitution
# (sglm_chol_solve_alias) and its explicit inverses (the recursive-doubling levels, ~0.9 ms for
# 20 fits at P = 2048, until now on the critical path after the chain) are formed on the side
# stream behind it, beside the next main-stream work; 0 turns it off (round 6)
DEFER_INV_MIN = int(__import__("os").environ.get("SGLM_DEFER_INV_MIN", "0"))
# gradient enqueued before the Hessian decisions' device wait when no Hessian is planned
GRAD_FIRST = __import__("os").environ.get("SGLM_GRAD_FIRST", "1") == "1"
# gradient kernel that co-resides with the factorisation chain in iterations that form factors
XTR_COCHAIN = __import__("os").environ.get("SGLM_XTR_COCHAIN", "1") == "1"
# constant-weight Grams of lagged event designs from the event cross-correlations
LAG_GRAM = __import__("os").environ.get("SGLM_LAG_GRAM", "1") == "1"
# concurrent factorisation chains for a batch of >= CHOL_SPLIT_MIN new factorisations.  Round 3
# measured no gain (56.2 / 56.2 ms: the second chain started only as the first ended, beside a
# full-chip gradient); since the first iteration's gradient runs once per start key (GRAD_DEDUP)
# its 20-fit chain has the chip to itself, and two chains of 10 beat one of 20: C4 29.02 ->
# 28.83 ms, 13 of 14 interleaved rounds (profiles/r06b_ab_chol_split.json); every fit's
# arithmetic is the same in either split, so the factors are bitwise unchanged
CHOL_SPLIT = int(__import__("os").environ.get("SGLM_CHOL_SPLIT", "2"))
CHOL_SPLIT_MIN = int(__import__("os").environ.get("SGLM_CHOL_SPLIT_MIN", "12"))
# SGLM_GRAM_PIPE=1: Grams computed one source at a time with each group's factorisation chain
# started right behind its Gram -- measured slower: the per-group chains are latency-bound
# (~1.1 ms each at 1-3 fits against 2.6 ms for one chain of 20), so the side stream carried
# 28.6 instead of 12.1 ms per C4 grid and more of it was exposed (11.4 vs 7.1 ms).
# SGLM_GRAM_PIPE=0: one Gram launch, then one chain.
# SGLM_GRAM_PIPE=2: the sources in two batches -- one Gram launch and one chain per batch, the
# first batch's chain overlapping the second batch's Grams -- also measured slower (C4 grid
# 62.3 / 63.1 / 62.3 ms against 59.7 / 60.2 / 59.3 ms unpipelined, alternating on one box).
# Default 0.
GRAM_PIPE = int(__import__("os").environ.get("SGLM_GRAM_PIPE", "0") or 0)
# bit-planes of 0/1 event designs straight from the events (sglm_lag_bits; the dense bf16
# design only on first use)
LAG_BITS = __import__("os").environ.get("SGLM_LAG_BITS", "1") == "1"
# Rank decisions of unpenalised fits (float64 factor of the exact mask Gram, sglm_chol64_factor):
# a pivot whose Schur complement is <= tol * its diagonal is a dependent column.  The Gram of a
# 0/1 design is exact (integer counts in f32), so tol only has to clear float64 elimination
# noise (~1e-16 relative; a full-rank design would need cond(X^T X) > 1e9 to be truncated); the
# f32-accumulated Gram of a real-valued design carries ~1e-7 relative noise, so dependence there
# is judged at the f32 factor's former threshold.
RANK_TOL_EXACT = float(__import__("os").environ.get("SGLM_RANK_TOL_EXACT", "1e-9"))
RANK_TOL_F32 = float(__import__("os").environ.get("SGLM_RANK_TOL_F32", "1e-6"))
# Mixed 0/1 + continuous designs: a design whose non-binary columns are few keeps its 0/1
# columns as bit-planes (the bf16-MFMA Gram / gradient / predictor kernels) and holds the k
# continuous ones as a float64 block (csrc/mixed.hip), when k <= MIXED_MAX_K and the float64
# continuous Gram block (n * k(k+1)/2 products per Gram) stays within MIXED_BUDGET; otherwise
# the whole design is stored f32.
MIXED_MAX_K = int(__import__("os").environ.get("SGLM_MIXED_MAX_K", "256"))
MIXED_BUDGET = float(__import__("os").environ.get("SGLM_MIXED_BUDGET", "1e9"))
# R rows (fits x continuous columns) per weighted-Gram X^T (W C) launch of a mixed design
MIXED_WC_ROWS = 256
# base-256 digits of the fixed-point products in the exact X^T (m v) of 0/1 designs (xtv_digits)
XTV_DIGITS = 5


def mixed_ok(n: int, k: int) -> bool:
    """A design with k non-binary columns of n rows is stored mixed (see MIXED_MAX_K)."""
    return 0 < k <= MIXED_MAX_K and float(n) * k * (k + 1) / 2 <= MIXED_BUDGET


def _gram_groups(form, uniq, dup):
    """The fits that form a new Hessian this iteration grouped by the Gram they take it from,
    [(source, fits)] with the source first in its group, sources in ascending order; None when
    there is a single source or a formed fit's source is not among the computed Grams."""
    if len(uniq) < 2:
        return None
    src = {int(k): int(k) for k in uniq}
    for k, rk in dup:
        src[int(k)] = int(rk)
    groups = {int(r): [int(r)] for r in uniq}
    for k in form:
        k = int(k)
        r = src.get(k)
        if r is None or r not in groups:
            return None
        if k != r:
            groups[r].append(k)
    if sum(len(g) for g in groups.values()) != len(form):
        return None
    return [(r, np.asarray(groups[r], dtype=np.int64)) for r in sorted(groups)]


def _slab_info(slab, n: int):
    """(start, stop, n) of a row slab, checked against n rows."""
    s0, s1 = int(slab[0]), int(slab[1])
    if not 0 <= s0 < s1 <= int(n):
        raise ValueError(f"row slab {slab} outside 0..{n}")
    return s0, s1, int(n)


def require_gpu():
    """Raise unless the HIP engine can run (library present AND a ROCm device visible)."""
    _lib.load()
    if not torch.cuda.is_available():
        raise _lib.HipEngineUnavailable(
            "no ROCm GPU visible: the sglm HIP engine has no CPU fallback")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def pad_to(x, m):
    return (int(x) + m - 1) // m * m


# ------------------------------------------------------------------------------ design
class Design:
    """Design matrix resident in HBM, feature-major, with the ones column at index p.

    xb: bf16 [P, ld]  (Gram operand; exact for 0/1 event designs)
    xf: f32  [P, ld]  or None (only when X is not bf16-exact; used for eta and X^T r)
    """

    def __init__(self, n: int, p: int, device="cuda", zero=True, lazy_xb=None):
        require_gpu()
        self.n, self.p = int(n), int(p)
        self.P = pad_to(self.p + 1, COL_PAD)
        self.ld = pad_to(self.n + 1, ROW_PAD)     # >= 1 zero padding row (w = 0 there)
        # lazy_xb: a callable that fills a zeroed bf16 design when xb is first read (designs
        # whose bit-planes come straight from events never need the dense copy on the hot path)
        self._xb_fill = lazy_xb
        self._xb = None
        if lazy_xb is None:
            alloc = torch.zeros if zero else torch.empty
            self._xb = alloc((self.P, self.ld), dtype=torch.bfloat16, device=device)
        self.xf = None
        self.xbits = None      # uint32 bit-planes [P, ld/32] when the design is 0/1
        self.rbits = None      # row-major bit-planes [P/64][ld] x uint2 (MFMA eta) when 0/1
        self._cbits = None     # identity-row compacted planes [n/64][P] x uint2 (MFMA X^T R)
        self.lag = None        # LagStructure of a time-shifted 0/1 event design (from_events)
        # mixed designs: the k non-binary columns as float64 [k][ld] (zero rows >= n) at design
        # positions cpos (their bit-plane columns are zero; csrc/mixed.hip completes every
        # bit-plane product over them)
        self.cont = None
        self.cpos = None
        self._mix = None
        self.slab = None       # (start, stop, n_total): rows [start, stop) of an n_total-row
        #                        design (one rank's share of a row-sharded solve, comm.py)
        self.device = device

    @property
    def xb(self):
        """bf16 [P, ld] dense design (built on first use when the bit-planes came first)."""
        if self._xb is None:
            self._xb = torch.zeros((self.P, self.ld), dtype=torch.bfloat16, device=self.device)
            self._xb_fill(self._xb)
        return self._xb

    @xb.setter
    def xb(self, v):
        self._xb = v

    @property
    def xtype(self):
        return X_F32 if self.xf is not None else X_BF16

    @property
    def k(self) -> int:
        """Number of continuous (float64) columns of a mixed design (0 otherwise)."""
        return 0 if self.cont is None else int(self.cont.shape[0])

    def _set_cont(self, C, cpos):
        """Make this a mixed design: C = device float64 (k, >= n) continuous columns at design
        positions cpos (their bf16 / bit-plane columns must be zero)."""
        cpos = np.asarray(cpos, dtype=np.int64).reshape(-1)
        k = int(cpos.size)
        if k == 0:
            return
        if C.shape[0] != k or C.shape[1] < self.n:
            raise ValueError("continuous block shape does not match its positions")
        if np.any(cpos < 0) or np.any(cpos >= self.p) or np.unique(cpos).size != k:
            raise ValueError("continuous column positions out of range or repeated")
        self.cont = torch.zeros((k, self.ld), dtype=torch.float64, device=self.device)
        self.cont[:, :self.n] = C[:, :self.n]
        self.cpos = cpos
        cmap = np.full(self.P, -1, dtype=np.int32)
        cmap[cpos] = np.arange(k, dtype=np.int32)
        iu = np.triu_indices(k)
        pg = np.concatenate([iu[0], iu[1]]).astype(np.int32)
        px = np.concatenate([np.arange(k), np.full(k, k)]).astype(np.int32)
        dev = self.device
        self._mix = dict(cpos=torch.from_numpy(cpos.astype(np.int32)).to(dev),
                         cmap=torch.from_numpy(cmap).to(dev),
                         pg=torch.from_numpy(pg).to(dev), px=torch.from_numpy(px).to(dev))

    def mix_eta(self, beta, out, slots=None, nb=None):
        """out[slot] += C beta[slot][cpos] for the slots (all rows of beta when None)."""
        if self.cont is None:
            return
        nb = (beta.shape[0] if slots is None else int(slots.numel())) if nb is None else nb
        _lib.call("sglm_mixed_eta", _p(self.cont), self.ld, self.k, self.n, _p(self._mix["cpos"]),
                  _p(beta), self.P, _p(slots), int(nb), _p(out), out.shape[1], _stream())

    def mix_xtr(self, rmode, R, ldr, Bp, rsel, gslots, nq, g):
        """g[gslot_q][cpos] = C R_q (float64): the continuous coordinates of X^T R."""
        if self.cont is None or nq <= 0:
            return
        w = _work(_lib.query("sglm_mixed_work_bytes", int(nq), self.k, self.n), self.device,
                  "mixed")
        _lib.call("sglm_mixed_xtr", int(rmode), _p(R), int(ldr), int(Bp), _p(rsel), _p(gslots),
                  int(nq), _p(self.cont), self.ld, self.k, self.n, _p(self._mix["cpos"]), self.P,
                  _p(self._mix["px"]), _p(g), _p(w), _stream())

    def mix_gram_rows(self, W=None, wslots=None, M=None, mrows=None, upl=None):
        """float64 S [ns][k][P]: the Gram rows of the continuous columns, S[s][c][j] = sum_r
        wt_s(r) C[c][r] X[r][j].  Weighted (IRLS): wt_s = W[wslots[s]] (f32), the 0/1 columns
        from the bit-plane X^T (W C) kernel (f32-accurate products).  Exact (mask Grams): wt_s
        = M[mrows[s]] (uint8 multiplicities), the 0/1 columns from the exact digit-plane X^T (m C)
        (xtv_digits).  The continuous block itself in float64 (sglm_mixed_gram)."""
        k, P, n, ld, dev = self.k, self.P, self.n, self.ld, self.device
        exact = M is not None
        rows = np.asarray(mrows if exact else wslots, dtype=np.int64).reshape(-1)
        ns = int(rows.size)
        S = torch.empty((ns, k, P), dtype=torch.float64, device=dev)
        if ns == 0:
            return S
        rows_d = (upl(rows, np.int32) if upl is not None
                  else torch.from_numpy(rows.astype(np.int32)).to(dev))
        if exact:
            pairs = [(c, int(m)) for m in rows for c in range(k)]
            xtv_digits(self, M, self.cont, pairs, S.view(ns * k, P), mixed=False)
        else:
            per = max(1, MIXED_WC_ROWS // k)
            for s0 in range(0, ns, per):
                cnt = min(per, ns - s0)
                R = _work(cnt * k * ld * 4, dev, "mixed_wc")[: cnt * k * ld * 4].view(
                    torch.float32).view(cnt * k, ld)
                _lib.call("sglm_mixed_wc", _p(W), W.shape[1], _p(rows_d[s0:]), cnt,
                          _p(self.cont), ld, k, n, ld, _p(R), _stream())
                self.xtr(R, cnt * k, S[s0:s0 + cnt].view(cnt * k, P), mixed=False)
        w = _work(_lib.query("sglm_mixed_work_bytes", ns, k, n), dev, "mixed")
        src = M if exact else W
        _lib.call("sglm_mixed_gram", 1 if exact else 0, _p(src), src.shape[1], _p(rows_d), ns,
                  _p(self.cont), ld, k, n, _p(self._mix["cpos"]), P, _p(self._mix["pg"]), _p(S),
                  _p(w), _stream())
        return S

    def mix_to_h(self, S, slots, H, upl=None):
        """H[slots[s]]: the continuous rows and columns (f32) from S."""
        ns = int(S.shape[0])
        if ns == 0:
            return
        sl = np.asarray(slots, dtype=np.int32).reshape(-1)
        sl = upl(sl) if upl is not None else torch.from_numpy(sl).to(self.device)
        _lib.call("sglm_mixed_to_h", _p(S), ns, self.k, self.P, _p(self._mix["cpos"]), _p(sl),
                  _p(H), _stream())

    @property
    def xg(self):
        """Operand for the exact GEMV-class kernels."""
        return self.xf if self.xf is not None else self.xb

    @classmethod
    def from_host(cls, X, device="cuda", slab=None):
        """Pack a host (n x p) array / DataFrame (row-major) into HBM; ``slab`` = (start,
        stop) packs only those rows (a rank's share of a row-sharded solve)."""
        if hasattr(X, "values") and not isinstance(X, np.ndarray):
            X = X.values
        X = np.asarray(X)
        if X.ndim == 1:
            X = X.reshape(-1, 1)
        info = None
        if slab is not None:
            info = _slab_info(slab, X.shape[0])
            X = X[info[0]:info[1]]
        if X.dtype not in (np.float32, np.float64):
            X = X.astype(np.float64)
        X = np.ascontiguousarray(X)
        n, p = X.shape
        d = cls(n, p, device, zero=False)
        d._pack_chunked(X)
        d.slab = info
        return d

    def _pack_chunked(self, X: np.ndarray):
        """Upload a row-major host array in row chunks of <= UPLOAD_CHUNK_BYTES: each chunk is
        copied by HOST_THREADS threads into one of two pinned staging buffers (sglm_host_copy),
        moved by an asynchronous copy, and packed into the design's rows (sglm_pack_design_rows_cf,
        which also flags every column holding a value other than 0 / 1) -- no pageable multi-GB
        .to(device), and the host copy of chunk k + 1 overlaps the DMA and pack of chunk k.
        All-0/1: bit-planes.  A few non-binary columns (mixed_ok): those columns as a float64
        block (gathered from the host array by native threads), the rest as bit-planes.  Else the
        design is packed again with its f32 copy (the first chunk's flags catch a design with
        many non-binary columns before the rest is uploaded once for nothing)."""
        n, p = X.shape
        dev, is64 = self.device, X.dtype == np.float64
        item = X.itemsize
        rows = max(64, (UPLOAD_CHUNK_BYTES // max(1, p * item)) // 64 * 64)
        rows = min(rows, pad_to(max(n, 1), 64))
        tdt = torch.float64 if is64 else torch.float32
        hbuf = [_pinned(f"h2d{i}", rows * p, tdt) for i in range(2)]
        dbuf = [_work(rows * p * item, dev, f"h2d{i}") for i in range(2)]
        evs = [None, None]
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        colflag = torch.zeros(max(p, 1), dtype=torch.int32, device=dev)
        n64 = pad_to(n, 64)
        if n64 < self.ld:
            self.xb[:, n64:].zero_()
        st = _stream()

        def run(xf, r_from, r_to):
            for k, r0 in enumerate(range(r_from, r_to, rows)):
                c = min(rows, n - r0)
                b = k % 2
                if evs[b] is not None:
                    evs[b].synchronize()          # the DMA out of this staging buffer is done
                _lib.call("sglm_host_copy", hbuf[b].data_ptr(), X[r0:r0 + c].ctypes.data,
                          c * p * item, HOST_THREADS)
                dst = dbuf[b][: c * p * item]
                dst.copy_(hbuf[b][: c * p].view(torch.uint8), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                evs[b] = ev
                _lib.call("sglm_pack_design_rows_cf", dst.data_ptr(), int(is64), c, p, p, 1, 1,
                          _p(self.xb), _p(xf), self.ld, self.P, r0, _p(flag),
                          None if xf is not None else _p(colflag), st)
        if n == 0:
            return
        first = min(rows, n)
        run(None, 0, first)
        k_first = int((colflag[:p] != 0).sum().item()) if p else 0
        cont = None
        if k_first <= MIXED_MAX_K:
            run(None, first, n)
            cf = colflag[:p].cpu().numpy()
            cont = np.flatnonzero(cf)
            if cont.size and not mixed_ok(n, int(cont.size)):
                cont = None
        if cont is None:
            self.xf = torch.empty((self.P, self.ld), dtype=torch.float32, device=dev)
            if n64 < self.ld:
                self.xf[:, n64:].zero_()
            run(self.xf, 0, n)
            if bool(torch.isnan(self.xf).any()):
                raise ValueError("Input X contains NaN.")       # sklearn check_array's error
        else:
            if cont.size:
                self._gather_cont(X, cont)
                if bool(torch.isnan(self.cont).any()):
                    raise ValueError("Input X contains NaN.")
                self.xb[torch.from_numpy(cont).to(dev)] = 0        # their bit columns: zero
            self._pack_bits()
            if self.xbits is None:
                raise RuntimeError("mixed design: the 0/1 part did not pack as bit-planes")
        for ev in evs:
            if ev is not None:
                ev.synchronize()                      # the staging buffers are reusable

    def _gather_cont(self, X: np.ndarray, cont):
        """The float64 block of a mixed design from a host row-major array: columns ``cont``
        gathered by native threads into a pinned column-major stage, one asynchronous upload."""
        n, p = X.shape
        k = int(cont.size)
        item = X.itemsize
        stage = _pinned("cont", k * n, torch.float64 if item == 8 else torch.float32)
        ptrs = (ctypes.c_void_p * k)(*[X.ctypes.data + int(c) * item for c in cont])
        strides = np.full(k, p, dtype=np.int64)
        _lib.call("sglm_host_gather_cols", ctypes.cast(ptrs, ctypes.c_void_p),
                  strides.ctypes.data, k, n, item, stage.data_ptr(), HOST_THREADS)
        C = torch.empty((k, n), dtype=stage.dtype, device=self.device)
        C.view(-1).copy_(stage[: k * n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._set_cont(C.to(torch.float64), cont)
        ev.synchronize()                      # the pinned stage is reused by the next design

    @classmethod
    def from_lagged(cls, Ecm, cols, shifts, r0: int, n: int, rows=None, device="cuda",
                    ones=None):
        """A design whose column j is source column cols[j] lagged by shifts[j]:
        X[t, j] = Ecm[cols[j], row(t) - shifts[j]] with row(t) = r0 + t (rows None) or rows[t]
        (a device int64 row list).  Ecm: device float64 [m][N] source columns (NaN-free on
        every row read).  A contiguous, canonical shift-major (or event-major) 0/1 layout goes
        through from_events (LagStructure: event-correlation Gram and gradient); anything else
        is expanded / gathered column by column (sglm_timeshift_expand / _gather)."""
        require_gpu()
        cols = np.asarray(cols, dtype=np.int64)
        shifts = np.asarray(shifts, dtype=np.int64)
        m = int(Ecm.shape[0])
        if rows is None:
            for major in (False, True):
                lay = _canonical_lags(cols, shifts, m, major)
                if lay is not None:
                    ev, sl = lay
                    E = Ecm[torch.from_numpy(ev).to(Ecm.device)].t()
                    # ones: per source row of Ecm its count of 1 cells when every source is
                    # known 0/1 (the host pack's flags): no device checks or counts to wait on
                    hint = None if ones is None else int(np.asarray(ones, np.int64)[ev].sum())
                    return cls.from_events(E, sl, r0, n, device=device, event_major=major,
                                           nnz=hint)
            # a canonical lag block followed by unshifted columns -- the production design's
            # counters and session dummies after the event lags (sglm_cb_concat_make_design_
            # mat.py:286, 310): the lag block from its events (LagStructure: structured Gram and
            # correlation start), the others as the float64 block of a mixed design
            L0 = _lag_block_split(cols, shifts)
            if L0 is not None and mixed_ok(n, int(cols.size) - L0):
                for major in (False, True):
                    lay = _canonical_lags(cols[:L0], shifts[:L0], m, major)
                    if lay is None:
                        continue
                    ev, sl = lay
                    E = Ecm[torch.from_numpy(ev).to(Ecm.device)]
                    if not bool(((E == 0) | (E == 1)).all()):
                        break
                    extra = Ecm[torch.from_numpy(cols[L0:]).to(Ecm.device), r0:r0 + n]
                    hint = None if ones is None else int(np.asarray(ones, np.int64)[ev].sum())
                    return cls.from_events(E.t(), sl, r0, n, device=device, event_major=major,
                                           nnz=hint, extra=extra)
        p = int(cols.size)
        d = cls(n, p, device, zero=True)
        c_d = torch.from_numpy(cols.astype(np.int32)).to(device)
        s_d = torch.from_numpy(shifts.astype(np.int32)).to(device)
        N = int(Ecm.shape[1])
        Eb = Ecm.to(torch.bfloat16).contiguous()
        binsrc = ((Ecm == 0) | (Ecm == 1)).all(dim=1).cpu().numpy()

        def expand(src, out, elem, cd=c_d, sd=s_d, ncol=p):
            if rows is None:
                _lib.call("sglm_timeshift_expand", _p(src), N, 1, N, _p(cd), _p(sd), ncol,
                          _p(out), n, 1, d.ld, int(r0), elem, 0, _stream())
            else:
                _lib.call("sglm_timeshift_gather", _p(src), N, 1, N, _p(cd), _p(sd), ncol,
                          _p(out), n, 1, d.ld, _p(rows), elem, 0, _stream())
        expand(Eb, d.xb, 2)
        d.xb[p, :n] = 1.0
        # design columns lagged from a source with values other than 0 / 1
        contc = np.flatnonzero(~binsrc[cols]) if p else np.zeros(0, np.int64)
        if contc.size == 0:
            d._pack_bits()
        elif mixed_ok(n, int(contc.size)):
            # mixed: those columns as a float64 block lagged from the float64 sources, the rest
            # as bit-planes
            k = int(contc.size)
            C = torch.zeros((k, d.ld), dtype=torch.float64, device=device)
            cc = torch.from_numpy(cols[contc].astype(np.int32)).to(device)
            sc = torch.from_numpy(shifts[contc].astype(np.int32)).to(device)
            expand(Ecm.contiguous(), C, 8, cc, sc, k)
            d.xb[torch.from_numpy(contc).to(device)] = 0
            d._pack_bits()
            if d.xbits is None:
                raise RuntimeError("mixed design: the 0/1 part did not pack as bit-planes")
            d._set_cont(C, contc)
        else:
            Ef = Ecm.to(torch.float32).contiguous()
            d.xf = torch.zeros((d.P, d.ld), dtype=torch.float32, device=device)
            expand(Ef, d.xf, 4)
            d.xf[p, :n] = 1.0
        return d

    @classmethod
    def from_lagged_bits(cls, B, N_raw: int, cols, shifts, r0: int, n: int, ones):
        """from_lagged for 0/1 sources given as device bit rows B (int32 [m][ceil(N_raw/32)],
        bit r & 31 of word r >> 5 = source row r; lagframe.LagSource.bits) with their counts of 1
        cells: the canonical shift-major / event-major layout of contiguous rows goes straight to
        the bit-plane design (from_event_bits); None for any other layout."""
        require_gpu()
        cols = np.asarray(cols, dtype=np.int64)
        shifts = np.asarray(shifts, dtype=np.int64)
        for major in (False, True):
            lay = _canonical_lags(cols, shifts, int(B.shape[0]), major)
            if lay is not None:
                ev, sl = lay
                eb = B[torch.from_numpy(ev).to(B.device)].contiguous()
                hint = int(np.asarray(ones, np.int64)[ev].sum())
                return cls.from_event_bits(eb, int(N_raw), sl, int(r0), int(n),
                                           device="cuda", event_major=major, nnz=hint)
        return None

    @classmethod
    def from_event_bits(cls, ebits, N_raw: int, shifts: Sequence[int], row0: int, n: int,
                        device="cuda", event_major=False, nnz=None):
        """from_events for 0/1 events given as device bit rows ebits (int32 [m][nwords], bit
        v & 31 of word v >> 5 = event row v): the lag bit-planes (sglm_lag_bits), the
        LagStructure (occurrences unpacked from the bits) and a dense bf16 copy only on first
        use."""
        require_gpu()
        m = int(ebits.shape[0])
        nwords = int(ebits.shape[1])
        K = len(shifts)
        p = K * m
        if event_major:
            cols = np.repeat(np.arange(m), K)
            sh = np.tile(np.asarray(shifts), m)
        else:
            cols = np.tile(np.arange(m), K)
            sh = np.repeat(np.asarray(shifts), m)
        cols_d = torch.tensor(cols, dtype=torch.int32, device=device)
        sh_d = torch.tensor(sh, dtype=torch.int32, device=device)

        def fill(xb):
            Eb = _unpack_bits(ebits, N_raw).to(torch.bfloat16).contiguous()   # (m, N_raw)
            _lib.call("sglm_timeshift_expand", _p(Eb), N_raw, 1, N_raw, _p(cols_d), _p(sh_d), p,
                      _p(xb), n, 1, xb.shape[1], row0, 2, 0, _stream())
            xb[p, :n] = 1.0
        d = cls(n, p, device, lazy_xb=fill)
        d.xbits = torch.empty((d.P, d.ld // 32), dtype=torch.int32, device=device)
        d.rbits = torch.empty((d.P // 64) * d.ld * 2, dtype=torch.int32, device=device)
        _lib.call("sglm_lag_bits", _p(ebits), nwords, _p(cols_d), _p(sh_d), p, row0, n,
                  d.ld, d.P, _p(d.xbits), _p(d.rbits), _stream())
        d.lag = LagStructure.build(None, shifts, row0, n, event_major, ebits=ebits, nnz=nnz,
                                   n_raw=N_raw)
        return d

    @classmethod
    def from_device(cls, Xt, device="cuda"):
        """Pack a device torch tensor (n x p, f32/f64, any strides); a few non-binary columns
        make a mixed design (see MIXED_MAX_K)."""
        n, p = Xt.shape
        if Xt.dtype not in (torch.float32, torch.float64):
            Xt = Xt.to(torch.float64)
        # sklearn's check (as the host upload path and the lagged frame raise it): a NaN would
        # otherwise sit in the float64 block or the f32 copy and give NaN coefficients
        if bool(torch.isnan(Xt).any()):
            raise ValueError("Input X contains NaN.")
        nonbin = np.flatnonzero((~((Xt == 0) | (Xt == 1)).all(dim=0)).cpu().numpy())
        if nonbin.size and mixed_ok(n, int(nonbin.size)):
            d = cls(n, p, device, zero=True)
            Xb = Xt.clone()
            nb_d = torch.from_numpy(nonbin).to(Xt.device)
            Xb[:, nb_d] = 0
            d._pack(Xb, is_f64=Xb.dtype == torch.float64, rs=Xb.stride(0), cs=Xb.stride(1))
            if d.xbits is None:
                raise RuntimeError("mixed design: the 0/1 part did not pack as bit-planes")
            d._set_cont(Xt[:, nb_d].t().to(torch.float64), nonbin)
            return d
        d = cls(n, p, device, zero=False)
        d._pack(Xt, is_f64=Xt.dtype == torch.float64, rs=Xt.stride(0), cs=Xt.stride(1))
        return d

    def _pack(self, src, is_f64, rs, cs):
        flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.call("sglm_pack_design", _p(src), int(is_f64), self.n, self.p, rs, cs, 1,
                  _p(self.xb), None, self.ld, self.P, _p(flag), _stream())
        if int(flag.item()):
            self.xf = torch.empty((self.P, self.ld), dtype=torch.float32, device=self.device)
            flag.zero_()
            _lib.call("sglm_pack_design", _p(src), int(is_f64), self.n, self.p, rs, cs, 1,
                      _p(self.xb), _p(self.xf), self.ld, self.P, _p(flag), _stream())
        else:
            self._pack_bits()

    def _pack_bits(self):
        """Bit-plane copies for 0/1 designs (column-packed for the Gram, row-major for eta);
        dropped again if X is not binary."""
        bits = torch.empty((self.P, self.ld // 32), dtype=torch.int32, device=self.device)
        flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.call("sglm_pack_bits", _p(self.xb), self.ld, self.P, _p(bits), _p(flag), _stream())
        if int(flag.item()):
            self.xbits = self.rbits = None
            return
        self.xbits = bits
        self.rbits = torch.empty((self.P // 64) * self.ld * 2, dtype=torch.int32,
                                 device=self.device)
        _lib.call("sglm_pack_bits_t", _p(self.xb), self.ld, self.P, _p(self.rbits), _p(flag),
                  _stream())

    @classmethod
    def from_events(cls, E, shifts: Sequence[int], row0: int, n: int, device="cuda",
                    event_major=False, slab=None, nnz=None, extra=None):
        """Expand base events E (N_raw x m) into lag columns directly on the device.

        Output column (shift block b, event a) = E[t + row0 - shifts[b], a] for rows
        t < n — the shift-major layout of sglm_ez.timeshift_cols (backend/sglm_ez.py:
        102-123) after the NaN-row drop (row0 = max positive shift), or event-major when
        ``event_major`` (setup_model_fit.timeshift_vals_by_dict, lag order as given).
        Source rows outside E can only occur if row0/n exceed the valid window; they are
        filled with 0.  ``slab`` = (start, stop): only rows [start, stop) of the n-row design
        (a rank's share of a row-sharded solve, comm.py).  ``extra``: float64 (k, n) continuous
        columns (unshifted, one value per design row -- the production design's cumcount^2 /
        5000 counters, pp_design_mat.py:167-172) placed after the lag columns: a mixed design.
        """
        require_gpu()
        info = None
        if slab is not None:
            info = _slab_info(slab, n)
            row0, n = row0 + info[0], info[1] - info[0]
            if extra is not None:
                extra = extra[:, info[0]:info[1]]
        if extra is not None:
            extra = torch.as_tensor(extra, dtype=torch.float64).to(device)
            if extra.ndim != 2 or extra.shape[1] != n:
                raise ValueError(f"extra columns must be (k, {n})")
            if bool(torch.isnan(extra).any()):
                raise ValueError("Input X contains NaN.")
        if isinstance(E, np.ndarray):
            E = torch.from_numpy(np.ascontiguousarray(E, dtype=np.float32))
        E = E.to(device=device, dtype=torch.float32)
        N_raw, m = E.shape
        K = len(shifts)
        pl = K * m                                          # lag columns
        kx = 0 if extra is None else int(extra.shape[0])
        p = pl + kx
        Eb = E.t().contiguous().to(torch.bfloat16)          # feature-major bf16 (m, N_raw)
        if event_major:
            cols = np.repeat(np.arange(m), K)
            sh = np.tile(np.asarray(shifts), m)
        else:
            cols = np.tile(np.arange(m), K)
            sh = np.repeat(np.asarray(shifts), m)
        cols_d = torch.tensor(cols, dtype=torch.int32, device=device)
        sh_d = torch.tensor(sh, dtype=torch.int32, device=device)

        def fill(xb):
            _lib.call("sglm_timeshift_expand", _p(Eb), N_raw, 1, N_raw, _p(cols_d), _p(sh_d), pl,
                      _p(xb), n, 1, xb.shape[1], row0, 2, 0, _stream())
            xb[p, :n] = 1.0

        # nnz (the events' count of 1 cells) is given only for events known to be 0/1
        if LAG_BITS and (nnz is not None or bool(((E == 0) | (E == 1)).all())):
            # 0/1 events: the bit-planes straight from the events' occurrence bitmaps (no dense
            # 4-GB-at-C4 design to write and pack twice); the dense copy is built on first use
            d = cls(n, p, device, lazy_xb=fill)
            nwords = (N_raw + 31) // 32
            ebits = torch.empty((m, nwords), dtype=torch.int32, device=device)
            _lib.call("sglm_event_bits", _p(Eb), N_raw, m, N_raw, _p(ebits), nwords, _stream())
            d.xbits = torch.empty((d.P, d.ld // 32), dtype=torch.int32, device=device)
            d.rbits = torch.empty((d.P // 64) * d.ld * 2, dtype=torch.int32, device=device)
            lb, lc, ls = ebits, cols_d, sh_d
            if kx:
                # the continuous columns' bit columns: zero (an all-zero event row, shift 0)
                lb = torch.cat([ebits, torch.zeros((1, nwords), dtype=torch.int32,
                                                   device=device)])
                lc = torch.cat([cols_d, torch.full((kx,), m, dtype=torch.int32, device=device)])
                ls = torch.cat([sh_d, torch.zeros(kx, dtype=torch.int32, device=device)])
            _lib.call("sglm_lag_bits", _p(lb), nwords, _p(lc), _p(ls), p, row0, n,
                      d.ld, d.P, _p(d.xbits), _p(d.rbits), _stream())
            d.lag = LagStructure.build(E, shifts, row0, n, event_major, ebits=ebits, nnz=nnz)
            if kx:
                d._set_cont(extra, np.arange(pl, p))
            d.slab = info
            return d
        d = cls(n, p, device, zero=True)
        fill(d.xb)
        exact = bool(torch.equal(Eb.float(), E.t()))
        if exact:
            d._pack_bits()
            if d.xbits is not None and bool(((E == 0) | (E == 1)).all()):
                d.lag = LagStructure.build(E, shifts, row0, n, event_major)
        if not exact:
            if kx:
                raise NotImplementedError("extra continuous columns need 0/1 events")
            Ef = E.t().contiguous()
            d.xf = torch.zeros((d.P, d.ld), dtype=torch.float32, device=device)
            _lib.call("sglm_timeshift_expand", _p(Ef), N_raw, 1, N_raw, _p(cols_d), _p(sh_d),
                      p, _p(d.xf), n, 1, d.ld, row0, 4, 0, _stream())
            d.xf[p, :n] = 1.0
        elif kx:
            if d.xbits is None:
                raise NotImplementedError("extra continuous columns need 0/1 events")
            d._set_cont(extra, np.arange(pl, p))
        d.slab = info
        return d

    def cbits_full(self):
        """Compacted bit-planes of all n rows (Gram v6 layout, K = rows): the A operand of
        the MFMA gradient and the Gram of full-data fits.  Built once per design."""
        if self._cbits is None and self.xbits is not None:
            self._cbits = torch.empty(max(1, (self.n + 63) // 64) * self.P * 2,
                                      dtype=torch.int32, device=self.device)
            if self.rbits is not None:
                _lib.call("sglm_compact_rbits", _p(self.rbits), self.ld, self.P, None, self.n,
                          _p(self._cbits), _stream())
            else:
                _lib.call("sglm_compact_bits", _p(self.xbits), self.ld, self.P, None, self.n,
                          _p(self._cbits), _stream())
        return self._cbits

    def xtr(self, R, B, g_out, work=None, mixed=True):
        """g_out[k] (float64) = X^T R[k] for k < B (R: [B][ld] f32 device); ``mixed`` = False
        leaves a mixed design's continuous coordinates as the bit-plane kernel wrote them (0)."""
        st = _stream()
        if self.xbits is not None and XTR_BITS:
            w = _work(_lib.query("sglm_xtr_bits_work_bytes", self.P, B, self.ld), self.device,
                      "xtr")
            _lib.call("sglm_xtr_bits", _p(self.cbits_full()), self.ld, self.P, self.n, _p(R), B,
                      _p(g_out), _p(w), st)
        else:
            w = _work(_lib.query("sglm_xtr_work_bytes", self.P, B, self.n), self.device, "xtr")
            _lib.call("sglm_xtr", _p(self.xg), self.xtype, self.ld, self.P, self.n, _p(R), B,
                      _p(g_out), _p(w), st)
        if mixed:
            self.mix_xtr(0, R, R.shape[1], 0, None, None, B, g_out)

    def xtr_int_ok(self) -> bool:
        """sglm_xtr_bits_int applies: a 0/1 design with P % 512 == 0 and ld < 2^26."""
        return (self.xbits is not None and XTR_BITS and self.P % 512 == 0
                and 64 * self.ld < (1 << 32))

    def xtr_int(self, D, B, g_out, mixed=True):
        """g_out[k] (float64) = X^T D[k] for k < B, D: bf16 [ceil(B/32)*32][ld] device tensor of
        integers |d| <= 256 (exact: one bf16 piece, f32 sums of integers within 2^24)."""
        if not self.xtr_int_ok():
            raise RuntimeError("xtr_int needs a 0/1 design with P % 512 == 0")
        if D.dtype != torch.bfloat16 or D.shape[0] < (B + 31) // 32 * 32 or D.shape[1] != self.ld:
            raise ValueError("xtr_int: D must be bf16 [ceil(B/32)*32][ld]")
        w = _work(_lib.query("sglm_xtr_bits_int_work_bytes", self.P, B, self.ld), self.device,
                  "xtr")
        _lib.call("sglm_xtr_bits_int", _p(self.cbits_full()), self.ld, self.P, self.n, _p(D), B,
                  _p(g_out), _p(w), _stream())
        if mixed:
            self.mix_xtr(3, D, D.shape[1], 0, None, None, B, g_out)

    def eta(self, beta_dev, out=None, slots=None, direction=False):
        """eta[k] = X beta[k] for a (B, P) f32 device tensor; with ``slots`` (int32 device
        tensor) only those rows k (the rest of ``out`` is left as is).  ``direction``: beta
        holds Newton directions, which are rounded to bf16 in place (0/1 designs) and X times
        the rounded directions is returned -- the caller must step with the rounded values."""
        B = beta_dev.shape[0]
        if out is None:
            out = torch.empty((B, self.ld), dtype=torch.float32, device=self.device)
        if self.rbits is not None and ETA_BITS:
            nb = B if slots is None else int(slots.numel())
            work = _work(_lib.query("sglm_eta_bits_work_bytes", self.P, nb), self.device, "eta")
            _lib.call("sglm_gemv_eta_bits", _p(self.rbits), self.ld, self.P, _p(beta_dev), nb,
                      _p(slots), int(not direction), _p(out), _p(work), _stream())
            # the continuous columns of a mixed design (after the kernel rounded a direction in
            # place: the float64 sum uses the rounded values the step takes)
            self.mix_eta(beta_dev, out, slots, nb)
        else:
            if self.cont is not None:
                raise RuntimeError("a mixed design needs the bit-plane predictor kernel")
            _lib.call("sglm_gemv_eta", _p(self.xg), self.xtype, self.ld, self.P, self.n,
                      _p(beta_dev), B, _p(out), _stream())
        return out


def xtv_digits(d: Design, M, V64, pairs, out, mixed=True):
    """out[q] = X^T (M[m_q] * V64[v_q]) in float64 for pairs q = (v_q, m_q) of a 0/1 (or mixed)
    design: M = uint8 row masks [F][>= n], V64 = float64 rows [R][>= n] (device).  m*v is put on
    a fixed-point grid of 2^-(38 - e) (|m v| < 2^e) and split into XTV_DIGITS balanced base-256
    digits; each digit plane is an integer vector with |digit| <= 128, which the bit-plane
    gradient kernel (row slabs <= 65,536 rows) sums EXACTLY in f32 and float64, so out is
    float64-accurate (~1e-13 of |out|).  The X^T (m y) of the elastic-net path (enet.xty) and
    the exact Gram rows of a mixed design's continuous columns (Design.mix_gram_rows)."""
    n, ld, dev = d.n, d.ld, d.device
    nd = XTV_DIGITS
    top = 8 * nd - 2                                            # |m v| 2^sh < 2^top
    w8 = torch.tensor([256.0 ** q for q in range(nd)], dtype=torch.float64, device=dev)
    if d.xtr_int_ok():
        # the digit planes built by one HIP pass (sglm_digit_planes) and summed by the one-piece
        # integer gradient kernel (sglm_xtr_bits_int); the scale of a pair comes from the bound
        # max(m) max|v| of its mask and vector (|m v| < 2^e)
        mmax = M[:, :n].amax(1).to(torch.float64)               # [F]
        vmax = V64[:, :n].abs().amax(1)                         # [R]
        chunk = max(1, 384 // nd)                               # <= 384 digit columns a call
        ncol = (min(chunk, len(pairs)) * nd + 31) // 32 * 32
        D = torch.zeros((ncol, ld), dtype=torch.bfloat16, device=dev)   # rows >= n stay zero
        g = torch.empty((ncol, d.P), dtype=torch.float64, device=dev)
        for s in range(0, len(pairs), chunk):
            pr = pairs[s:s + chunk]
            c = len(pr)
            rm = torch.tensor([[r for r, _ in pr], [m for _, m in pr]], dtype=torch.int32,
                              device=dev)
            ri, mi = rm[0].long(), rm[1].long()
            bnd = mmax[mi] * vmax[ri]
            e = torch.where(bnd > 0, torch.floor(torch.log2(bnd.clamp_min(1e-300))) + 1,
                            torch.zeros_like(bnd))
            sh = top - e
            scale = torch.exp2(sh)
            _lib.call("sglm_digit_planes", _p(M), M.stride(0), _p(V64), V64.stride(0), n,
                      _p(rm[0]), _p(rm[1]), _p(scale), c, nd, _p(D), ld, _stream())
            d.xtr_int(D, nd * c, g, mixed=mixed)
            gq = g[: nd * c].view(nd, c, d.P)
            out[s:s + c] = (gq * w8[:, None, None]).sum(0) * torch.exp2(-sh)[:, None]
        return out
    chunk = max(1, 240 // nd)
    D = torch.zeros((chunk * nd, ld), dtype=torch.float32, device=dev)
    g = torch.empty((chunk * nd, d.P), dtype=torch.float64, device=dev)
    for s in range(0, len(pairs), chunk):
        pr = pairs[s:s + chunk]
        c = len(pr)
        ri = torch.tensor([r for r, _ in pr], dtype=torch.int64, device=dev)
        mi = torch.tensor([m for _, m in pr], dtype=torch.int64, device=dev)
        Rv = M[mi, :n].to(torch.float64) * V64[ri, :n]         # [c][n]
        amax = Rv.abs().amax(1)
        e = torch.where(amax > 0, torch.floor(torch.log2(amax.clamp_min(1e-300))) + 1,
                        torch.zeros_like(amax))
        sh = (top - e)                                          # per pair exponent
        Ri = torch.round(Rv * torch.exp2(sh)[:, None]).to(torch.int64)
        for q in range(nd):
            dq = torch.remainder(Ri + 128, 256) - 128           # balanced digit in [-128, 127]
            D[q * c:(q + 1) * c, :n] = dq.to(torch.float32)
            Ri = torch.div(Ri - dq, 256, rounding_mode="floor")
        d.xtr(D[: nd * c], nd * c, g[: nd * c], mixed=mixed)
        gq = g[: nd * c].view(nd, c, d.P)
        out[s:s + c] = (gq * w8[:, None, None]).sum(0) * torch.exp2(-sh)[:, None]
    return out


def _unpack_bits(bits, n: int):
    """uint8 [rows][n] of device bit rows (int32 [rows][nwords], bit r & 31 of word r >> 5)."""
    sh = torch.arange(32, dtype=torch.int32, device=bits.device)
    return ((bits.unsqueeze(-1) >> sh) & 1).to(torch.uint8).reshape(bits.shape[0], -1)[:, :n]


def _lag_block_split(cols, shifts):
    """L0 when columns 0 .. L0 - 1 are lags of the sources that are ever shifted and every later
    column is an unshifted column of another source (a lag block followed by extra columns);
    None otherwise (or when there are no extra columns)."""
    cols = np.asarray(cols)
    shifts = np.asarray(shifts)
    lagged = set(cols[shifts != 0].tolist())
    if not lagged:
        return None
    inl = np.fromiter((c in lagged for c in cols.tolist()), dtype=bool, count=cols.size)
    L0 = int(np.argmin(inl)) if not inl.all() else cols.size
    if L0 == 0 or L0 == cols.size or inl[L0:].any() or np.any(shifts[L0:] != 0):
        return None
    return L0


def _canonical_lags(cols, shifts, m, event_major):
    """(events, shift list) when the (column, shift) pairs are every event x every shift in
    the shift-major (col = b * m' + a) or event-major (col = a * K + b) order, else None."""
    p = cols.size
    if p == 0:
        return None
    if event_major:
        ev = cols[np.r_[0, np.flatnonzero(np.diff(cols) != 0) + 1]]
        K = p // max(1, ev.size)
        if ev.size * K != p:
            return None
        sl = shifts[:K]
        ok = (np.array_equal(cols, np.repeat(ev, K)) and np.array_equal(shifts, np.tile(sl, ev.size)))
    else:
        K = int(np.sum(cols == cols[0]))
        mm = p // max(1, K)
        if mm * K != p:
            return None
        ev, sl = cols[:mm], shifts[::mm]
        ok = (np.array_equal(cols, np.tile(ev, K)) and np.array_equal(shifts, np.repeat(sl, mm)))
    if not ok or len(set(ev.tolist())) != ev.size or len(set(sl.tolist())) != sl.size:
        return None
    return ev, [int(x) for x in sl]


class LagStructure:
    """A time-shifted 0/1 event design by its events (sglm_lag_xtr): X[t, col(b, a)] =
    E[t + row0 - shifts[b], a].  occ = every event's occurrence rows of E, event-major and
    ascending; tbeg / tend [m][ntiles] = the occurrence range of event a whose lag window meets
    design-row tile i (tiles of sglm_lag_tile_rows() rows).  Built on the device once per
    design."""

    @classmethod
    def build(cls, E, shifts, row0, n, event_major, ebits=None, nnz=None, n_raw=None):
        """E: the events (N_raw x m, device), or None with ``ebits`` (bit rows) and ``n_raw``."""
        self = cls()
        if E is None:
            dev = ebits.device
            N_raw, m = int(n_raw), int(ebits.shape[0])
            occ_src = _unpack_bits(ebits, N_raw)                       # (m, N_raw) uint8
        else:
            dev = E.device
            N_raw, m = E.shape
            occ_src = E.t()
        sh = np.asarray(shifts, dtype=np.int64)
        self.m, self.K = int(m), int(sh.size)
        self.layout = 1 if event_major else 0
        self.row0 = int(row0)
        self.shifts = torch.from_numpy(sh.astype(np.int32)).to(dev)
        # (event, row) of every occurrence, event-major; a known count sizes it without
        # waiting for the device
        nz = (torch.nonzero(occ_src != 0) if nnz is None
              else torch.nonzero_static(occ_src != 0, size=int(nnz)))
        ev, rows = nz[:, 0], nz[:, 1]
        self.occ = rows.to(torch.int32).contiguous()
        U = _lib.query("sglm_lag_tile_rows")
        ntiles = (int(n) + U - 1) // U
        big = np.int64(1) << 40
        keys = ev.to(torch.int64) * big + rows.to(torch.int64)
        t0 = torch.arange(ntiles, dtype=torch.int64, device=dev) * U
        a = torch.arange(m, dtype=torch.int64, device=dev)[:, None] * big
        lo = a + (t0 + row0 - int(sh.max()))[None, :]
        hi = a + (t0 + U + row0 - int(sh.min()))[None, :]
        self.tbeg = torch.searchsorted(keys, lo.reshape(-1)).to(torch.int32).contiguous()
        self.tend = torch.searchsorted(keys, hi.reshape(-1)).to(torch.int32).contiguous()
        self.ntiles = ntiles
        if self.m > 64 or self.K > 256:
            return None                                       # the kernel's bounds
        # for the constant-weight Gram (sglm_lag_gram): event segments of occ and the
        # occurrence bitmap [m][nwords] (bit v & 31 of word v >> 5)
        self.n, self.n_raw = int(n), int(N_raw)
        self.smin, self.smax = int(sh.min()), int(sh.max())
        cnt = torch.bincount(ev, minlength=m)
        self.ev_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                                 torch.cumsum(cnt, 0)]).to(torch.int32).contiguous()
        self.nwords = (int(N_raw) + 31) // 32
        if ebits is None:
            Eb = occ_src.contiguous().to(torch.bfloat16)
            ebits = torch.empty((m, self.nwords), dtype=torch.int32, device=dev)
            _lib.call("sglm_event_bits", _p(Eb), int(N_raw), int(m), int(N_raw), _p(ebits),
                      self.nwords, _stream())
        self.ebits = ebits
        return self


# ------------------------------------------------------------------------------ problem
# threads of the native host-side setup helpers (sglm_host_masks, sglm_host_copy)
# (SGLM_HOST_THREADS, else the process's OpenMP share -- 16 on a one-GPU box -- else 8)
HOST_THREADS = max(1, min(int(os.environ.get("SGLM_HOST_THREADS")
                              or os.environ.get("OMP_NUM_THREADS") or 8), os.cpu_count() or 8))
# row-chunk size of the pinned host->device design upload (Design.from_host)
UPLOAD_CHUNK_BYTES = int(os.environ.get("SGLM_UPLOAD_CHUNK_BYTES", str(256 << 20)))


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def host_masks(specs, n: int, ld: int, out: Optional[np.ndarray] = None):
    """uint8 row masks (nm x ld, zero past n) of mask specs (idx or None = every row,
    multiplicity) by the multithreaded native builder (sglm_host_masks; host only, no GPU).
    Returns (nnz, sums) per mask, and fills ``out`` (flat, >= nm * ld) or returns it as a
    third value when ``out`` is None."""
    nm = len(specs)
    ret = out is None
    if out is None:
        out = np.empty(max(nm * ld, 1), dtype=np.uint8)
    if out.dtype != np.uint8 or out.size < nm * ld or not out.flags.c_contiguous:
        raise ValueError("out must be a contiguous uint8 array of >= nm * ld entries")
    lists, kinds = [], np.empty(nm, dtype=np.int32)
    for f, (idx, mult) in enumerate(specs):
        if idx is None:
            kinds[f] = 0                                       # SGLM_MASK_ALL
            lists.append(None)
        else:
            kinds[f] = 1 if mult else 2                        # SGLM_MASK_FOLD / _ROWS
            lists.append(np.ascontiguousarray(np.asarray(idx).reshape(-1), dtype=np.int64))
    ptrs = (ctypes.c_void_p * max(nm, 1))(*[0 if a is None else a.ctypes.data for a in lists])
    lens = np.array([0 if a is None else a.size for a in lists], dtype=np.int64)
    nnz = np.zeros(nm, dtype=np.int64)
    sums = np.zeros(nm, dtype=np.float64)
    try:
        _lib.call("sglm_host_masks", nm, ctypes.cast(ptrs, ctypes.c_void_p), _np_ptr(lens),
                  _np_ptr(kinds), int(n), int(ld), _np_ptr(out), _np_ptr(nnz), _np_ptr(sums),
                  HOST_THREADS)
    except _lib.HipEngineError as e:
        raise ValueError(str(e).split(": ", 1)[-1]) from None
    return (nnz, sums, out[: nm * ld].reshape(nm, ld)) if ret else (nnz, sums)


class _LazyHost:
    """Host (numpy) view of a device array, copied on first access."""

    def __init__(self, t):
        self.t = t
        self._a = None
        self.shape = tuple(t.shape)

    def __getitem__(self, idx):
        if self._a is None:
            self._a = self.t.cpu().numpy()
        return self._a[idx]


class _Columns:
    """Read-only list view of the columns of an (n x R) array (host copies on access)."""

    def __init__(self, a):
        self.a = a

    def __len__(self):
        return self.a.shape[1]

    def __getitem__(self, r):
        return np.ascontiguousarray(self.a[:, r], dtype=np.float64)

    def __iter__(self):
        return (self[r] for r in range(len(self)))


class Problem:
    """A design plus the response columns and row masks that a batch of fits refers to."""

    def __init__(self, design: Design, ys, masks: Sequence[np.ndarray]):
        """``ys``: a list of response vectors, or one (n x R) float64 array of R responses
        (multi-response paths: uploaded once, transposed on the device; ``Yd64`` keeps the
        float64 device copy)."""
        self.design = design
        n, ld, dev = design.n, design.ld, design.device
        self._masks = [np.asarray(m, dtype=np.uint8).reshape(-1) for m in masks]
        for m in self._masks:
            if m.shape[0] != n:
                raise ValueError(f"mask length {m.shape[0]} != n_samples {n}")
        self._nnz = None
        self._y64r = None
        self._rolled = None
        self.Yd64 = None
        if isinstance(ys, torch.Tensor) and ys.ndim == 2:
            # device-resident responses (n x R float64 on the design's device): no upload
            if ys.shape[0] != n:
                raise ValueError(f"response length {ys.shape[0]} != n_samples {n}")
            if ys.device != torch.device(dev) and str(ys.device) != str(dev):
                ys = ys.to(dev)
            self.Yd64 = ys.to(torch.float64).contiguous()
            self.ys = _Columns(_LazyHost(self.Yd64))
            self.Y = torch.zeros((ys.shape[1], ld), dtype=torch.float32, device=dev)
            self.Y[:, :n] = self.Yd64.t().float()
        elif isinstance(ys, np.ndarray) and ys.ndim == 2:
            if ys.shape[0] != n:
                raise ValueError(f"response length {ys.shape[0]} != n_samples {n}")
            self.ys = _Columns(ys)
            self.Yd64 = torch.from_numpy(np.ascontiguousarray(ys, dtype=np.float64)).to(dev)
            self.Y = torch.zeros((ys.shape[1], ld), dtype=torch.float32, device=dev)
            self.Y[:, :n] = self.Yd64.t().float()
        else:
            self.ys = [np.asarray(y, dtype=np.float64).reshape(-1) for y in ys]
            for y in self.ys:
                if y.shape[0] != n:
                    raise ValueError(f"response length {y.shape[0]} != n_samples {n}")
            Y = np.zeros((len(self.ys), ld), dtype=np.float32)
            for r, y in enumerate(self.ys):
                Y[r, :n] = y
            self.Y = torch.from_numpy(Y).to(dev)
        M = np.zeros((len(self.masks), ld), dtype=np.uint8)
        for f, m in enumerate(self.masks):
            M[f, :n] = m
        self.M = torch.from_numpy(M).to(dev)
        self._ylo = None
        self._stats = {}
        self._groups = None
        self._compact = {}

    @classmethod
    def from_index_lists(cls, design: Design, y, rolls: Sequence[int], specs):
        """A CV grid's problem straight from its fold index lists (no host mask arrays): the
        masks are built by the multithreaded native builder (sglm_host_masks) into a pinned
        buffer and uploaded asynchronously; the responses ``np.roll(y, r)`` for r in ``rolls``
        are formed on the device from one float64 upload.  ``specs``: per mask (idx or None =
        every row, multiplicity) -- a fold list counts repeats, a row list marks rows."""
        self = cls.__new__(cls)
        self.design = design
        n, ld, dev = design.n, design.ld, design.device
        # a slab design (row-sharded solve): the index lists address all n_total rows; the
        # masks and responses are cut to the slab, the mask counts stay global
        s0, s1, ntot = design.slab if design.slab is not None else (0, n, n)
        y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(-1))
        if y.shape[0] != ntot:
            raise ValueError(f"response length {y.shape[0]} != n_samples {ntot}")
        nm = len(specs)
        buf = _pinned("problem_masks", max(nm * ld, 1), torch.uint8)
        ev = _scratch().pinned.get(("problem_masks_ev", None))
        if ev is not None:
            ev.synchronize()                                   # the previous upload has read it
        if design.slab is None:
            nnz, sums = host_masks(specs, n, ld, buf.numpy())
        else:
            ldt = pad_to(ntot + 1, ROW_PAD)
            full = np.empty(max(nm * ldt, 1), dtype=np.uint8)
            _, sums = host_masks(specs, ntot, ldt, full)
            full = full[: nm * ldt].reshape(nm, ldt)
            bm = buf.numpy()[: nm * ld].reshape(nm, ld)
            bm[:, :n] = full[:, s0:s1]
            bm[:, n:] = 0
            nnz = np.count_nonzero(bm[:, :n], axis=1).astype(np.int64)
            local = bm[:, :n].sum(axis=1, dtype=np.int64).astype(np.float64)
        self.M = torch.empty((nm, ld), dtype=torch.uint8, device=dev)
        self.M.view(-1).copy_(buf[: nm * ld], non_blocking=True)
        yb = _pinned("problem_y", max(ntot, 1), torch.float64)
        if ev is None:
            ev = torch.cuda.Event()
            _scratch().pinned[("problem_masks_ev", None)] = ev
        _lib.call("sglm_host_copy", yb.data_ptr(), y.ctypes.data, 8 * ntot, HOST_THREADS)
        yd = torch.empty(ntot, dtype=torch.float64, device=dev)
        yd.copy_(yb[:ntot], non_blocking=True)
        ev.record()
        rolls = [int(r) for r in rolls]
        self._y64r = (torch.stack([torch.roll(yd, r)[s0:s1] for r in rolls]) if rolls
                      else yd[None, :0])
        self.Y = torch.zeros((len(rolls), ld), dtype=torch.float32, device=dev)
        self.Y[:, :n] = self._y64r.float()
        self._masks = None
        self._nnz = nnz
        self._rolled = (y, rolls, s0, s1)
        self.Yd64 = None
        self._ylo = None
        self._stats = {("count", f): float(sums[f]) for f in range(nm)}
        # the slab's own multiplicity sums (the counts above stay global)
        self._local_count = None if design.slab is None else local
        self._groups = None
        self._compact = {}
        return self

    @property
    def masks(self):
        """Host uint8 masks (a device copy when the problem was built from index lists)."""
        if self._masks is None:
            self._masks = list(self.M[:, : self.design.n].cpu().numpy())
        return self._masks

    @property
    def ys(self):
        if self._rolled is not None:
            y, rolls, s0, s1 = self._rolled
            return [np.roll(y, r)[s0:s1] for r in rolls]
        return self._ys

    @ys.setter
    def ys(self, v):
        self._ys = v

    def y64_rows(self):
        """The responses as one device float64 (R, n) array."""
        if self._y64r is None:
            if self.Yd64 is not None:
                self._y64r = self.Yd64.t().contiguous()
            else:
                self._y64r = torch.from_numpy(np.stack(self.ys)).to(self.design.device)
        return self._y64r

    def mask_local_count(self, mask: int) -> float:
        """Sum of a mask's multiplicities over this process's rows (its slab's share in a
        row-sharded solve, else mask_count)."""
        lc = getattr(self, "_local_count", None)
        return float(lc[mask]) if lc is not None else self.mask_count(mask)

    def mask_nnz(self, mask: int) -> int:
        """Rows with a nonzero mask value."""
        if self._nnz is not None:
            return int(self._nnz[mask])
        return int(np.count_nonzero(self.masks[mask]))

    def y_lo(self):
        """f32 residual y - f32(y) of the responses ([R][ld], or None when every y is exact in
        f32, e.g. counts): X^T(m y) = X^T(m y_hi) + X^T(m y_lo) recovers the float64 sums."""
        if self._ylo is None:
            n = self.design.n
            y64 = self.y64_rows()
            lo = torch.zeros_like(self.Y)
            lo[:, :n] = (y64 - self.Y[:, :n].double()).float()
            self._ylo = lo if bool(lo.any()) else False
        return self._ylo if self._ylo is not False else None

    def _group_lists(self):
        """Row lists for the masked v2/v3 Gram (non-binary designs): the 8-row groups of every
        aligned 64-row block that holds a row of the mask (built on first use)."""
        if self._groups is None:
            n = self.design.n
            goff, gcnt, lists = [], [], []
            off = 0
            for m in self.masks:
                mp = np.zeros(pad_to(n, 64), dtype=bool)
                mp[:n] = m > 0
                blk = np.flatnonzero(mp.reshape(-1, 64).any(axis=1))
                g = (blk[:, None] * 8 + np.arange(8)[None, :]).reshape(-1).astype(np.int32)
                lists.append(g)
                goff.append(off)
                gcnt.append(g.size)
                off += g.size
            self._groups = (torch.from_numpy(np.concatenate(lists) if off else
                                             np.zeros(1, np.int32)).to(self.design.device),
                            np.array(goff, dtype=np.int64), np.array(gcnt, dtype=np.int32))
        return self._groups

    @property
    def groups(self):
        return self._group_lists()[0]

    @property
    def group_offset(self):
        return self._group_lists()[1]

    @property
    def group_count(self):
        return self._group_lists()[2]

    def compact(self, mask: int):
        """Row-compacted bit-plane design of one mask (Gram v6), built once and cached:
        (bits, rows in the mask, device row list or None when the mask is every row)."""
        c = self._compact.get(mask)
        if c is None:
            d = self.design
            nr = self.mask_nnz(mask)
            # the mask's row list, built on the device (no host pass, no synchronising upload)
            rows_d = None if nr == d.n else torch.nonzero_static(
                self.M[mask, :d.n], size=nr).view(-1).to(torch.int32)
            if rows_d is None and d.xbits is not None:
                c = self._compact[mask] = (d.cbits_full(), nr, None)
                return c
            bits = torch.empty(max(1, (nr + 63) // 64) * d.P * 2, dtype=torch.int32,
                               device=d.device)
            if d.rbits is not None:
                _lib.call("sglm_compact_rbits", _p(d.rbits), d.ld, d.P, _p(rows_d), nr,
                          _p(bits), _stream())
            elif d.xbits is not None:
                _lib.call("sglm_compact_bits", _p(d.xbits), d.ld, d.P, _p(rows_d), nr,
                          _p(bits), _stream())
            else:
                flag = torch.zeros(1, dtype=torch.int32, device=d.device)
                _lib.call("sglm_pack_bits_rows", _p(d.xb), d.ld, d.P, _p(rows_d), nr, _p(bits),
                          _p(flag), _stream())
            c = (bits, nr, rows_d)
            self._compact[mask] = c
        return c

    def mask_count(self, mask: int) -> float:
        """Sum of a mask's multiplicities (rows of the fit), cached."""
        key = ("count", int(mask))
        if key not in self._stats:
            self._stats[key] = float(self.masks[int(mask)].sum(dtype=np.int64))
        return self._stats[key]

    def seed_stats(self, resp: int, mask: int, cnt: float, sum_y: float):
        """Provide (count, sum y) of a (response, mask) pair computed elsewhere (the grid's
        batched float64 device statistics), so that mask_stats needs no host pass."""
        self._stats[(resp, mask)] = (cnt, sum_y, sum_y / cnt if cnt else 0.0)
        self._stats[("count", int(mask))] = cnt

    def mask_stats(self, resp: int, mask: int):
        """float64 (count, sum y, mean y) over a mask — host side, cached."""
        key = (resp, mask)
        if key not in self._stats:
            m = self.masks[mask].astype(np.float64)
            y = self.ys[resp]
            cnt = m.sum()
            s = float(m @ y)
            self._stats[key] = (cnt, s, s / cnt if cnt else 0.0)
        return self._stats[key]


@dataclass
class FitReq:
    family: int
    power: float
    lam: float                      # penalty in units of the SUM objective (lam/2 |w|^2)
    mask: int
    resp: int
    fit_intercept: bool = True
    max_iter: int = 100
    coef0: Optional[np.ndarray] = None
    intercept0: Optional[float] = None


@dataclass
class FitResult:
    coef: np.ndarray
    intercept: float
    n_iter: int
    converged: bool
    dropped: int = 0


@dataclass
class IrlsStats:
    """Optional instrumentation: per-launch events of the Gram kernel (bench.py)."""
    record: bool = False
    syrk_events: list = field(default_factory=list)    # (start, end, algorithmic flop)
    syrk_bytes: list = field(default_factory=list)     # algorithmic HBM bytes per Gram launch
    syrk_exec: list = field(default_factory=list)      # executed MFMA flop per Gram launch
    fit_iters: int = 0
    newton_iters: int = 0
    gram_fits: int = 0                                  # distinct Hessians formed
    gram_fit_iters: int = 0     # fit-iterations whose own Gram was computed (Gram-forming)
    reused: int = 0                                     # fit-iterations that kept a factor
    aliased: int = 0            # fit-iterations solved on a family representative's factor
    shared: int = 0             # fit-iterations on a lambda neighbour's Gram (own factor)
    lag_grams: int = 0          # Grams from the event cross-correlations (sglm_lag_gram)
    grad_dedup: int = 0         # fit gradients copied from an identical start (GRAD_DEDUP)
    rank_grams: int = 0         # exact mask Grams for the rank decisions of unpenalised fits
    chain_host_s: float = 0.0   # host time spent enqueueing the factorisation chains
    aa_fit_iters: int = 0       # fit-iterations whose direction took the secant correction
    # flop actually executed by the algorithm, summed over fit-iterations: each computed Gram at
    # the count of the kernel that formed it (dense: n p'(p'+1); event-structured: LagStructure
    # flop1; event correlations: their histogram adds), new factors p'^3/3, gradient / eta /
    # solves 4 n p' + 2 p'^2
    alg_flop: float = 0.0
    alg_flop_dense: float = 0.0  # the same with every computed Gram at SURVEY.md §8(d)'s dense F
    sync_wait_s: float = 0.0    # host time blocked in the per-iteration stream synchronisation
    roundtrips: int = 0         # host<->device round trips (stream synchronisations) of the solve
    trace_phases: bool = False                          # sync + time grid phases (tools)
    phases: dict = field(default_factory=dict)          # host wall seconds per phase
    # why fits stopped (converged fits: tol + line_search_converged)
    stops: dict = field(default_factory=lambda: dict.fromkeys(
        ("tol", "stagnation", "line_search_converged", "line_search_failed", "max_iter",
         "stale_factor_retry", "alias_dropped"), 0))

    host_phases: bool = False   # host (enqueue) seconds per phase, no device syncs (tools)
    iter_log: Optional[list] = None     # per Newton iteration: a dict of counts (tools)

    def mark(self, name, t0):
        """Add the wall time since t0 to phase `name` (after a device sync when trace_phases:
        device + host time; without it the host's own time); returns now."""
        import time
        if self.trace_phases:
            torch.cuda.synchronize()
        t = time.perf_counter()
        self.phases[name] = self.phases.get(name, 0.0) + (t - t0)
        return t


class _Buffers:
    """Re-usable device buffers keyed by (B, P, ld)."""

    def __init__(self):
        self.key = None

    def get(self, B, P, ld, dev):
        key = (B, P, ld)
        if key != self.key:
            f32 = torch.float32
            self.beta = torch.zeros((B, P), dtype=f32, device=dev)
            self.delta = torch.zeros((B, P), dtype=f32, device=dev)
            self.eta = torch.zeros((B, ld), dtype=f32, device=dev)
            self.deta = torch.zeros((B, ld), dtype=f32, device=dev)
            self.W = torch.zeros((B, ld), dtype=f32, device=dev)
            self.R = torch.zeros((B, ld), dtype=f32, device=dev)
            self.H = torch.empty((B, P, P), dtype=f32, device=dev)
            self.Minv = torch.empty((B, P, P), dtype=f32, device=dev) if SOLVE_INV else None
            # the factorisation chain's fit list (a stable address: the chain is a cached graph)
            self.fact_fits = torch.zeros((B,), dtype=torch.int32, device=dev)
            self.g = torch.zeros((B, P), dtype=torch.float64, device=dev)
            self.gtot = torch.zeros((B, P), dtype=torch.float64, device=dev)
            self.dshift = torch.zeros((B, P), dtype=f32, device=dev)
            self.frozen = torch.zeros((B, P), dtype=torch.uint8, device=dev)
            self.info = torch.zeros((B,), dtype=torch.int32, device=dev)
            self.cwork = torch.empty(_lib.query("sglm_chol_work_bytes", P, B), dtype=torch.uint8,
                                     device=dev)
            self._cwork = {0: self.cwork}
            self._P, self._B, self._dev = P, B, dev
            self.key = key
        return self

    def chol_work(self, j):
        """Work buffer of the j-th concurrent factorisation chain (the chain's scratch is
        indexed by list position, so concurrent chains need their own)."""
        w = self._cwork.get(j)
        if w is None:
            w = self._cwork[j] = torch.empty(_lib.query("sglm_chol_work_bytes", self._P,
                                                        self._B), dtype=torch.uint8,
                                             device=self._dev)
        return w


class _Scratch:
    """Per-thread engine scratch: device work buffers, pinned readback buffers, the IRLS batch
    buffers, and (for a thread that splits a batch into IRLS groups) its group threads'
    scratch and streams.  The reference calls fit / fit_set from several threads at once
    (backend/sglm_cv.py:162-170), so no two threads may share one."""

    def __init__(self):
        self.work = {}          # (device, tag) -> uint8 device buffer (grow-only)
        self.pinned = {}        # (tag, dtype) -> pinned host buffer (grow-only)
        self.buf = _Buffers()
        self.groups = {}        # group -> _Scratch of that IRLS group's thread
        self.streams = {}       # (device, group) -> torch stream


_TLS = threading.local()        # .scratch: this thread's _Scratch
_MAIN_SCRATCH = _Scratch()


def _scratch() -> _Scratch:
    """The calling thread's scratch: the main thread's lives for the process (so repeated
    grids reuse their buffers), other threads get their own (freed with the thread); IRLS group
    threads are handed their parent's persistent group scratch."""
    s = getattr(_TLS, "scratch", None)
    if s is None:
        s = _MAIN_SCRATCH if threading.current_thread() is threading.main_thread() else _Scratch()
        _TLS.scratch = s
    return s


_GRAM_LOCK = threading.Lock()   # orders the Gram launches of concurrent IRLS groups ...
_GRAM_DONE = {}                 # device -> event after the last Gram enqueued (any stream)


def _gram_turn():
    """Make the current stream's next Gram wait for every Gram already enqueued on the device
    (by any IRLS group): Grams of concurrent groups run one after another at full rate while
    the groups' latency-bound work overlaps them.  Call with _GRAM_LOCK held."""
    ev = _GRAM_DONE.get(torch.cuda.current_device())
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)


def _gram_done():
    ev = torch.cuda.Event()
    ev.record()
    _GRAM_DONE[torch.cuda.current_device()] = ev


def _side_stream(j: int = 0):
    """This thread's j-th side stream on the current device (the factorisation chains,
    overlapped with the gradient)."""
    streams = _scratch().streams
    prio = CHOL_STREAM == "prio"
    key = ((torch.cuda.current_device(), "chol") if j == 0 else (torch.cuda.current_device(),
                                                                  "chol", j)) + (prio,)
    sd = streams.get(key)
    if sd is None:
        # high priority: the chain's small latency-bound launches are dispatched ahead of the
        # gradient's workgroups as slots free up, instead of queueing behind a full-chip grid
        sd = streams[key] = torch.cuda.Stream(priority=-1 if prio else 0)
    return sd


def _pinned(tag, numel, dtype):
    """Grow-only pinned host buffer per (thread scratch, tag): page-locked allocation is slow,
    so the per-iteration readback buffers are allocated once and reused (flat; callers view)."""
    pinned = _scratch().pinned
    t = pinned.get((tag, dtype))
    if t is None or t.numel() < numel:
        t = torch.zeros(int(numel), dtype=dtype).pin_memory()
        pinned[(tag, dtype)] = t
    return t[:numel]


_NP2TORCH = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
             np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
             np.dtype(np.uint8): torch.uint8}


class _Uploads:
    """Asynchronous small host->device uploads for one IRLS thread.  A pageable ``.to(dev)``
    synchronises the stream (the host then waits for every queued kernel, and the GPU idles
    while the host prepares the next launches); arrays are instead staged in a pinned arena
    and copied with non_blocking=True into a device arena.  The arena has two halves that
    alternate at every stream synchronisation (``synced()``): a half is rewritten only after
    a synchronisation that followed every copy out of it, and an upload stays valid until
    the second synchronisation after it (kernels enqueued after the first may still read
    it)."""

    def __init__(self, dev, nbytes=1 << 20):
        self.half = nbytes // 2
        self.h = _pinned("up", nbytes, torch.uint8)
        self.d = _work(nbytes, dev, "up")
        self.dev = dev
        self.base = 0
        self.off = 0
        self.batch_at = None

    def __call__(self, a, dtype=None):
        a = np.ascontiguousarray(a if dtype is None else np.asarray(a).astype(dtype))
        nb = a.nbytes
        if self.off + nb > self.half:            # half full: a synchronous upload
            self.flush()
            return torch.from_numpy(a).to(self.dev)
        o = self.base + self.off
        self.h[o:o + nb].numpy()[:] = a.reshape(-1).view(np.uint8)
        dst = self.d[o:o + nb]
        if self.batch_at is None:
            dst.copy_(self.h[o:o + nb], non_blocking=True)
        self.off += (nb + 255) // 256 * 256
        return dst.view(_NP2TORCH[a.dtype]).view(a.shape)

    def batch(self):
        """Stage the next uploads without copying: ``flush()`` then moves them in ONE copy
        (the returned device views must not be read by a launch before the flush)."""
        self.flush()
        self.batch_at = self.off

    def flush(self):
        if self.batch_at is not None and self.off > self.batch_at:
            o0, o1 = self.base + self.batch_at, self.base + self.off
            self.d[o0:o1].copy_(self.h[o0:o1], non_blocking=True)
        self.batch_at = None

    def synced(self):
        """Call right after a synchronisation of the stream the uploads are ordered on."""
        self.flush()
        self.base = self.half - self.base
        self.off = 0


def _work(nbytes, dev, tag="main"):
    """Grow-only scratch buffer per (thread scratch, device, tag); stream-ordered reuse only
    (each thread that runs the engine has its own scratch)."""
    nbytes = max(int(nbytes), 16)
    work = _scratch().work
    t = work.get((dev, tag))
    if t is None or t.numel() < nbytes:
        t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        work[(dev, tag)] = t
    return t


def syrk_splits(n_tiles_total: int, nsteps: int, cus: int = 256) -> int:
    """Split the rows over workgroups when the tile count alone cannot fill the chip."""
    best, best_eff = 1, 0.0
    for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
        if s > max(1, nsteps // 16):
            break
        wgs = n_tiles_total * s
        rounds = math.ceil(wgs / cus)
        eff = wgs / (rounds * cus)
        if eff > best_eff + 0.02:
            best, best_eff = s, eff
    return best


# lower bound on the Gram v6 split-K factor (shorter-lived workgroups let the other IRLS
# group's small kernels interleave with a Gram; experiment knob)
SYRK6_MIN_SPLIT = int(__import__("os").environ.get("SGLM_SYRK6_MIN_SPLIT", "1"))
GRAM_LOG = None                 # a list: each Gram launch appends (nact, distinct masks, splits, rows)


def syrk6_splits(wgs1: int, nsteps: int, nact: int, P: int, slots: int = 1024) -> int:
    """Split-K factor for Gram v6: minimise (rounds of one-wave workgroups) x (workgroup
    time) + the split-K slab traffic (write + reduce-read of splits x nact x P^2 floats)."""
    t_step = 2048 / 2.4e9                     # 64 MFMA x 32 cycles per K-step
    best, best_t = 1, None
    for s in range(1, 65):              # every factor: whole rounds of the 1024 wave slots
        if s > max(1, nsteps // 8):
            break
        if s < SYRK6_MIN_SPLIT and s < max(1, nsteps // 8):
            continue
        t = math.ceil(wgs1 * s / slots) * math.ceil(nsteps / s) * t_step
        if s > 1:
            t += s * nact * P * P * 8.0 / 4e12
        if best_t is None or t < best_t:
            best, best_t = s, t
    return best


def irls(prob: Problem, reqs: List[FitReq], tol: Optional[float] = None,
         stats: Optional[IrlsStats] = None, bufs: Optional[_Buffers] = None, comm=None):
    """Run the batched damped-Newton (IRLS) solve; returns (results, final eta tensor).

    ``comm`` (sglm_hip.comm.RowComm / SimComm): the problem holds one slab of the rows of a
    row-sharded solve; sums over rows are all-reduced, maxima over rows max-reduced, and the
    new factorisations are dealt over the ranks (see comm.py)."""
    require_gpu()
    if not reqs:
        return [], None
    tol = STOP_TOL if tol is None else float(tol)
    d = prob.design
    fam, power = reqs[0].family, float(reqs[0].power)
    if any(r.family != fam or float(r.power) != power for r in reqs):
        raise ValueError("irls(): one loss family per batch")
    if (fam == FAM_SQUARED and GRAM_LS and d.xbits is not None
            and max(prob.mask_count(int(r.mask)) for r in reqs) < 2 ** 24):
        return _gram_ls(prob, reqs, stats, bufs, comm)
    B0, P, ld, n, p = len(reqs), d.P, d.ld, d.n, d.p
    dev = d.device
    bf = (bufs or _scratch().buf).get(B0, P, ld, dev)
    st = _stream()
    log_link = fam == FAM_TWEEDIE_LOG
    reqs0 = list(reqs)

    # the per-fit penalty rows, start coefficients and index arrays are built on the device from
    # per-fit scalars staged through the pinned upload arena (a pageable upload of each [B][P]
    # array would synchronise the stream several times before the first kernel)
    up = _Uploads(dev)
    lam = np.array([float(r.lam) for r in reqs])
    icpt = np.zeros(B0)
    warm = any(r.coef0 is not None for r in reqs)
    beta = np.zeros((B0, P), dtype=np.float64) if warm else None
    for k, r in enumerate(reqs):
        if r.coef0 is not None:
            beta[k, :p] = r.coef0
            icpt[k] = (r.intercept0 or 0.0) if r.fit_intercept else 0.0
        elif r.fit_intercept:
            cnt, s, ym = prob.mask_stats(r.resp, r.mask)
            if log_link:
                if ym <= 0:
                    raise ValueError("Some value(s) of y are out of the valid range of the loss")
                icpt[k] = math.log(ym)
            else:
                icpt[k] = ym
    fi = np.array([1.0 if r.fit_intercept else 0.0 for r in reqs])
    fresp_h = np.array([r.resp for r in reqs], dtype=np.int32)
    fmask_h = np.array([r.mask for r in reqs], dtype=np.int32)
    ts_h = np.concatenate([[0.0, 1.0, 0.5, 0.25, 0.125], TV2.astype(np.float32)])
    scal = up(np.concatenate([lam, icpt, fi, ts_h]), np.float64)
    ints = up(np.concatenate([fresp_h, fmask_h]), np.int32)
    lam_d, icpt_d, fi_d = scal[:B0], scal[B0:2 * B0], scal[2 * B0:3 * B0]
    # ridge shift per coordinate (lam on the predictors, 0 on a fitted intercept, -1 = frozen:
    # the intercept of fit_intercept=False and the padding columns)
    bf.dshift.fill_(-1.0)
    bf.dshift[:B0, :p] = lam_d[:, None]
    bf.dshift[:B0, p] = fi_d - 1.0
    # the coefficients live on the device (float64); the host sees per-fit scalars only
    if warm:
        beta[:, p] = icpt
        beta64_d = torch.from_numpy(beta).to(dev)
    else:
        beta64_d = torch.zeros((B0, P), dtype=torch.float64, device=dev)
        beta64_d[:, p] = icpt_d
    bf.beta[:B0].copy_(beta64_d)
    lamp_d = torch.zeros((B0, P), dtype=torch.float64, device=dev)      # lam * penalty mask
    lamp_d[:, :p] = lam_d[:, None]
    if not warm:
        # intercept-only start: X beta is the intercept on every row (exactly, as the MFMA
        # product of the ones column would give it)
        bf.eta[:, :n].copy_(bf.beta[:, p:p + 1].expand(B0, n))
        bf.eta[:, n:].zero_()
    else:
        d.eta(bf.beta, bf.eta)

    const_hess = fam == FAM_SQUARED
    reuse_tol = 0.0 if const_hess else HESS_REUSE_TOL / max(1.0, abs(2.0 - power))
    share_tol = 0.0 if const_hess else min(HESS_SHARE_TOL / max(1.0, abs(2.0 - power)),
                                           reuse_tol)
    # Device state is held per SLOT (one per fit, fixed for the whole solve); every per-fit
    # kernel takes the list of active slots, so stopped fits cost nothing and no state moves.
    B = B0
    fit_resp = torch.empty(B0, dtype=torch.int32, device=dev)
    fit_resp.copy_(ints[:B0])
    fit_mask = torch.empty(B0, dtype=torch.int32, device=dev)
    fit_mask.copy_(ints[B0:])
    drift = np.full(B0, np.inf)         # predictor drift since each fit's Hessian was formed
    # one host round trip per Newton iteration: the gradient, the step direction, the trial
    # losses and the step's predictor drift come back together (pinned buffers, async copies)
    dmax_d = torch.zeros(B0, dtype=torch.float32, device=dev)
    dmax_h = _pinned("dmax", B0, torch.float32)
    L_h = _pinned("L", B0 * 8, torch.float64)
    ts_all = torch.empty(ts_h.size, dtype=torch.float64, device=dev)
    ts_all.copy_(scal[3 * B0:])
    nts = int(ts_all.numel())
    sc_d = torch.empty(B0 * (6 + nts), dtype=torch.float64, device=dev)
    # fits still at their common start (same mask and response => bitwise equal Hessians)
    fresh_start = np.array([r.coef0 is None for r in reqs])
    gram_now = np.zeros(B0, dtype=bool)
    exact_h = np.zeros(B0, dtype=bool)     # Hessian = the fit's own Gram at its own predictor
    active = np.ones(B0, dtype=bool)
    n_iter = np.zeros(B0, dtype=np.int64)
    converged = np.zeros(B0, dtype=bool)
    prev_rel = np.full(B0, np.inf)
    max_iter = np.array([max(1, int(r.max_iter)) for r in reqs])
    out_beta = np.zeros((B0, P), dtype=np.float64)
    out_iter = np.zeros(B0, dtype=np.int64)
    out_conv = np.zeros(B0, dtype=bool)
    out_info = np.zeros(B0, dtype=np.int64)
    factored = False
    xtr_work = _work(max(_lib.query("sglm_xtr_work_bytes", P, B0, n),
                         _lib.query("sglm_rowsum_work_bytes", B0, 8, n)), dev)
    tv1 = ts_all[:5].float()
    tv2 = ts_all[5:].float()
    Ltr = torch.zeros(B0 * 8, dtype=torch.float64, device=dev)    # dense [B][T] per call
    nsteps = (n + 31) // 32
    ntile1 = (P // 256) * (P // 256 + 1) // 2
    rows = np.array([prob.mask_stats(r.resp, r.mask)[0] for r in reqs], dtype=np.float64)
    # rows of the Grams this process computes (its slab's rows of each mask in a row-sharded
    # solve; ``rows`` stays the fit's global count: penalty scale, alias ratios, flop count)
    gram_rows = rows if comm is None else np.array([float(prob.mask_nnz(r.mask)) for r in reqs])
    # row-sharded solve: the rank holding each slot's current factor, and whether the new
    # factorisations are dealt over the ranks (explicit-inverse solves only)
    dist_f = comm is not None and comm.distribute and SOLVE_INV
    # fits whose mask is every row with multiplicity 1 (the refits): a constant weight at the
    # start, so the first Gram can come from the event cross-correlations (sglm_lag_gram)
    ntot = d.n if d.slab is None else d.slab[2]
    # every row of this process with multiplicity exactly 1 (nnz == n and the local sum == n;
    # a slab's rows can repeat while the global sum still equals the global row count) ...
    umask = sorted(set(int(r.mask) for r in reqs))
    mall = {m: prob.mask_nnz(m) == d.n and prob.mask_local_count(m) == d.n
            and prob.mask_count(m) == ntot for m in umask}
    if comm is not None and umask:
        # ... on EVERY rank (min-reduced: all ranks take the same first-Gram decision)
        flag = torch.tensor([1 if mall[m] else 0 for m in umask], dtype=torch.int32,
                            device=dev)
        comm.min_(flag)
        mall = dict(zip(umask, (flag.cpu().numpy() > 0).tolist()))
    all_rows = np.array([mall[int(r.mask)] for r in reqs])
    # the weight m * h(y, eta) is one constant on such a mask only when h does not depend on y:
    # the Poisson log link (h = exp(eta)); Gamma / Tweedie's h carries y on every row
    use_lag_gram = (LAG_GRAM and fam == FAM_TWEEDIE_LOG and power == 1.0 and d.lag is not None
                    and getattr(d.lag, "ebits", None) is not None
                    and d.lag.smax - d.lag.smin <= 2048)
    fowner = np.zeros(B0, dtype=np.int64)
    rot = 0
    # secant (Anderson-1) correction of the directions of fits that step on the same stale
    # factor as in their previous iteration (see ANDERSON): the previous raw and used
    # directions, the step taken, and the factor each fit solved on (slot, formation epoch)
    use_aa = ANDERSON and fam != FAM_SQUARED and SOLVE_INV
    if use_aa:
        aa_raw = torch.zeros((B0, P), dtype=torch.float32, device=dev)
        aa_used = torch.zeros((B0, P), dtype=torch.float32, device=dev)
        # per slot, this iteration's raw direction size (max |f_j|, j < p; |f_p|) where the
        # correction ran: convergence is also judged on the raw Newton step
        aa_rm = torch.zeros((B0, 2), dtype=torch.float32, device=dev)
        aa_rm_h = _pinned("aa_rm", 2 * B0, torch.float32)
    aa_t = np.zeros(B0)
    aa_key = np.full(B0, -1, dtype=np.int64)
    fepoch = np.zeros(B0, dtype=np.int64)

    def sum_hess(idx):
        """The slab Grams of a row-sharded solve summed over the ranks (one all-reduce each;
        a mixed design's float64 Gram rows of the continuous columns too)."""
        if comm is not None:
            store = getattr(bf, "mixS", None) or {}
            for k in np.asarray(idx).reshape(-1):
                comm.sum_(bf.H[int(k)])
                if int(k) in store:
                    comm.sum_(store[int(k)])
    bf.prob, bf.fit_mask, bf.fit_mask_d = prob, fmask_h, fit_mask
    bf.mixS = {}
    # cross-mask families (slot of the representative per slot, -1: none / is one)
    xmask_tol = 0.0 if const_hess else HESS_XMASK_TOL / max(1.0, abs(2.0 - power))
    repl = np.full(B0, -1, dtype=np.int64)
    if xmask_tol > 0.0:
        fams = {}
        for k, r in enumerate(reqs):
            key = _family_key(r, rows[k])
            if key is not None:
                fams.setdefault(key, []).append(k)
        for members in fams.values():
            if len(members) > 1:
                rk = max(members, key=lambda k: (rows[k], -k))
                for k in members:
                    if k != rk:
                        repl[k] = rk
    alias = np.full(B0, -1, dtype=np.int64)     # slot whose factor the fit used this iteration
    no_alias = np.zeros(B0, dtype=bool)
    no_share = np.zeros(B0, dtype=bool)     # failed a step on a lambda neighbour's Hessian

    bf.up = up
    pd_h = _pinned("pairdist", 4 * B0, torch.float32)

    # float64 factors (sglm_chol64_factor) with exact rank decisions: every squared-loss fit
    # solves on the factor of its (mask, penalty, intercept) -- the reference's closed forms
    # run in float64 (lstsq / cholesky, sklearn _base.py:701, _ridge.py:201-213) -- and an
    # unpenalised log-link fit takes its dependent columns from the float64 factor of its mask's
    # exact Gram (null(X~^T W X~) = null(X~^T M X~) for W > 0).  Unpenalised fits end at the
    # minimum-norm point of their solution set (lstsq; lbfgs from 0 stays in the row space).
    lam0 = lam == 0.0
    f64, fkey = None, np.full(B0, -1, dtype=np.int64)
    if const_hess:
        mrep = {}
        for k, r in enumerate(reqs):
            mrep.setdefault(int(r.mask), k)
        keys, k_h, k_d = {}, [], []
        # the unpenalised fits' factors first: the minimum-norm pass needs only those
        for k in np.argsort(~lam0, kind="stable"):
            r = reqs[k]
            key = (int(r.mask), float(r.lam), bool(r.fit_intercept))
            if key not in keys:
                keys[key] = len(k_h)
                k_h.append(mrep[int(r.mask)])
                k_d.append(k)
            fkey[k] = keys[key]
        # a persistent copy: an upload-arena view is only valid until the second sync after it
        fkey_d = torch.empty(B0, dtype=torch.int32, device=dev)
        fkey_d.copy_(up(fkey, np.int32))
    elif lam0.any():
        keys, k_h = {}, []
        for k in np.flatnonzero(lam0):
            key = (int(reqs[k].mask), bool(reqs[k].fit_intercept))
            if key not in keys:
                keys[key] = len(k_h)
                k_h.append(int(k))
            fkey[k] = keys[key]
        k_h = np.asarray(k_h, dtype=np.int32)
        # the exact mask Gram of each (W = the mask's multiplicities; the first link update
        # overwrites W)
        kh_d = up(k_h, np.int64)
        bf.W[kh_d] = prob.M[up(fmask_h[k_h], np.int64)].float()
        _syrk(d, bf, k_h, nsteps, ntile1, None, st, exact=True, rows=gram_rows)
        sum_hess(k_h)
        f64 = _Factor64(d, bf, k_h, k_h, lamp_d, st)
        sel = np.flatnonzero(lam0)
        sel_d = up(sel, np.int64)
        stt = f64.state[up(fkey[sel], np.int64)]
        frz = (stt == 1) | (stt == 3)
        ds = bf.dshift[sel_d]
        bf.dshift[sel_d] = torch.where(frz, torch.full_like(ds, -1.0), ds)
        if stats is not None:
            stats.rank_grams += int(k_h.size)

    def hkey(k):
        """Fits with equal keys have bitwise equal Hessians: one (mask, response) at the
        common start -- which depends on the intercept setting (log(mean y) or 0) -- or the
        fit itself once it has moved."""
        return ((reqs[k].mask, reqs[k].resp, -1, bool(reqs[k].fit_intercept)) if fresh_start[k]
                else (reqs[k].mask, reqs[k].resp, int(k)))

    def hess_plan(act):
        """Hessian decisions of the next iteration that need no device data, and one launch of
        the max-row distances they depend on (copied back asynchronously): fits with a valid
        factor keep it (drift <= reuse_tol); fits of a cross-mask family without one are
        candidates for the representative's factor (distance to it); the rest form a new
        Hessian -- once per distinct (mask, response, beta) -- and the distinct ones of one
        (mask, response) may share along the lambda path (distances of neighbours)."""
        own_ok = drift[act] <= reuse_tol
        cand = act[(repl[act] >= 0) & ~no_alias[act] & ~own_ok]
        rest = act[~np.isin(act, cand)]
        keep = rest[drift[rest] <= reuse_tol]
        form = rest[drift[rest] > reuse_tol]
        reps, dup = {}, []
        for k in form:
            rk = reps.setdefault(hkey(k), k)
            if rk != k:
                dup.append((k, rk))
        uniq = np.array(sorted(reps.values()), dtype=np.int32)
        chains = []
        if share_tol > 0.0 and uniq.size > 1:
            groups = {}
            for k in uniq:
                if not no_share[k]:
                    groups.setdefault((reqs[k].mask, reqs[k].resp), []).append(int(k))
            chains = [sorted(g, key=lambda k: lam[k]) for g in groups.values() if len(g) > 1]
        pairs = [(int(k), int(repl[k])) for k in cand]
        pairs += [(c[i], c[i + 1]) for c in chains for i in range(len(c) - 1)]
        ev = None
        if pairs and len(pairs) > pd_h.numel():
            raise RuntimeError("pair distance buffer too small")
        if pairs and not warm and all(fresh_start[a] and fresh_start[b]
                                      and prob.mask_count(reqs[a].mask) > 0 for a, b in pairs):
            # both fits still at their intercept-only start: eta is one constant per fit, so
            # the max-row distance is |f32(b_a) - f32(b_b)| (what the kernel would compute)
            ic32 = icpt.astype(np.float32)
            pa = np.array(pairs, dtype=np.int64)
            pd_h[:len(pairs)].copy_(torch.from_numpy(np.abs(ic32[pa[:, 0]] - ic32[pa[:, 1]])))
        elif pairs:
            npair = len(pairs)
            pd_d = _pair_dist_async(bf, prob, np.array(pairs, dtype=np.int32), n, ld, st)
            if comm is not None:
                comm.max_(pd_d)
            pd_h[:npair].copy_(pd_d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        return dict(cand=cand, keep=keep, form=form, reps=reps, dup=dup, uniq=uniq,
                    chains=chains, npairs=len(pairs), ev=ev)

    def hess_finish(pl):
        """Apply the distances of a plan: lambda-neighbour sharing, then aliasing of the
        candidates whose distance to the representative plus the representative's own drift
        after this iteration's decision stays <= xmask_tol (the others form their own).
        Every Hessian copy is resolved to a Hessian this iteration actually computes (a copy
        of a fit that itself shares along the lambda chain follows the chain), and the copy's
        drift is the summed distance along that path.  Returns (keep, form, uniq, copies,
        aliased, failed candidates, exact): ``exact`` flags the fits whose Hessian is their
        own Gram at their own predictor (computed, or an exact duplicate of one)."""
        if pl["ev"] is not None:
            pl["ev"].synchronize()
        dist = pd_h[:pl["npairs"]].numpy().astype(np.float64)
        cand, keep, form, reps, dup, uniq = (pl[k] for k in ("cand", "keep", "form", "reps",
                                                             "dup", "uniq"))
        dist_c, dist_s = dist[:cand.size], dist[cand.size:]
        drift[form] = 0.0
        src = {int(k): (int(rk), 0.0) for k, rk in dup}     # fit -> (source fit, distance)
        if pl["chains"]:
            uniq, shared = _share_chains(uniq, pl["chains"], dist_s, share_tol)
            for k, rk, dist_k in shared:
                src[int(k)] = (int(rk), float(dist_k))
        ok = dist_c + drift[repl[cand]] <= xmask_tol
        ali, fail = cand[ok], cand[~ok]
        for k in fail:
            rk = reps.setdefault(hkey(k), k)
            if rk != k:
                src[int(k)] = (int(rk), 0.0)
            else:
                uniq = np.append(uniq, np.int32(k))
        drift[fail] = 0.0
        copies = _resolve_copies(src, uniq)
        for k, _, dk in copies:
            drift[k] = dk
        copies = [(k, r) for k, r, _ in copies]
        newh = np.concatenate([form, fail])
        exact = np.zeros(B0, dtype=bool)
        exact[newh] = drift[newh] == 0.0
        return keep, newh, uniq, copies, ali, fail, exact
    # the gradient: from the event occurrences for a time-shifted event design (sglm_lag_xtr,
    # R in f32 by slot), else the bit-plane MFMA with R packed into its operand
    use_lag = d.lag is not None and LAG_XTR and d.cont is None
    use_rp = d.xbits is not None and XTR_BITS and not use_lag
    fused = use_rp or use_lag          # link fused with the previous step's predictor update
    if use_rp:
        rp_buf = _work(3 * pad_to(B0, 32) * ld * 2, dev, "rp")
        gx_work = _work(_lib.query("sglm_xtr_bits_packed_work_bytes", P, B0, ld), dev, "xtr")
    if use_lag:
        lag_work = _work(_lib.query("sglm_lag_xtr_work_bytes", P, d.lag.K, B0, n), dev, "xtr")
    R_out, Rp_out = (_p(bf.R), None) if use_lag else (None, _p(rp_buf) if use_rp else None)
    # device-side decisions (packed-R designs, one process): the iteration's verdicts come back
    # with its losses while the step and the next link already run; the next gradient reads the
    # packed R rows of the fits that continue at the positions the device gave them
    dev_dec = DEV_DECIDE and use_rp and comm is None
    if dev_dec:
        dec64 = torch.empty((3, B0), dtype=torch.float64, device=dev)     # step, relv, prop
        dec32 = torch.empty(B0, dtype=torch.float32, device=dev)          # step (f32)
        deci = torch.empty(4 * B0 + 1, dtype=torch.int32, device=dev)     # flags tix rpos nxt cnt
        dec64_h = _pinned("dec64", 3 * B0, torch.float64)
        deci_h = _pinned("deci", 4 * B0 + 1, torch.int32)
        ev_dec = torch.cuda.Event()
    grad_d, grad_n, grad_bp = None, 0, 0     # the gradient's slots, count and R plane stride
    dev_linked = False                       # this iteration's link ran at the previous one's end

    import time
    tick = stats.mark if (stats is not None and (stats.trace_phases or stats.host_phases)) \
        else (lambda name, t: t)
    t0 = tick("irls_setup", time.perf_counter())
    plan = None
    pending_inv = None      # event after the last deferred inversion (side stream)
    linked = None           # slot list whose link (and predictor update) is already enqueued
    for it in range(int(max_iter.max()) + 1):
        # every per-fit kernel runs over the active slots only (slot lists): no compaction,
        # so factors, predictors and the representatives' factors stay where they are
        act = np.flatnonzero(active)
        na = int(act.size)
        if na == 0:
            break
        if dev_linked:
            act_d = up(act, np.int32)        # the gradient keeps the device's list (grad_d)
        else:
            act_d = linked if linked is not None else up(act, np.int32)
            grad_d, grad_n, grad_bp = act_d, na, pad_to(na, 32)
        g_copy = None                        # (fits, their lead fits): gradient rows copied
        link_d, link_n = act_d, na
        if GRAD_DEDUP and use_rp and fused and not dev_linked and linked is None:
            # fits still at their common start with one (mask, response, intercept) key
            # (hkey) have one predictor, hence bitwise one W, R and X^T R: the link and the
            # gradient run once per key and the other fits' gradient rows are copies (at C4:
            # 6 of 120 fits in the first iteration, where the factorisation chain runs beside
            # the gradient); nothing else reads a copied fit's W or R before its next link
            lead_of, first = {}, {}
            for k in act:
                if fresh_start[k]:
                    rk = first.setdefault(hkey(k), int(k))
                    if rk != k:
                        lead_of[int(k)] = rk
            if lead_of:
                lead = np.array([k for k in act if int(k) not in lead_of], dtype=np.int32)
                link_d, link_n = up(lead, np.int32), int(lead.size)
                grad_d, grad_n, grad_bp = link_d, link_n, pad_to(link_n, 32)
                cp = up(np.array([[k, r] for k, r in lead_of.items()], np.int64).T.reshape(-1),
                        np.int64)
                g_copy = (cp[:len(lead_of)], cp[len(lead_of):])
                if stats is not None:
                    stats.grad_dedup += len(lead_of)
        if fused and not dev_linked:
            if linked is None:
                _lib.call("sglm_link_update", fam, power, n, ld, link_n, _p(link_d), _p(bf.eta),
                          _p(prob.Y), _p(prob.M), _p(fit_resp), _p(fit_mask), _p(bf.W), R_out,
                          Rp_out, None, None, st)
        else:
            _lib.call("sglm_link_update", fam, power, n, ld, B, None, _p(bf.eta), _p(prob.Y),
                      _p(prob.M), _p(fit_resp), _p(fit_mask), _p(bf.W), _p(bf.R), None, None,
                      None, st)

        grad_done = [False]

        def _gradient(cochain_ok=True):
            """X^T R on the current stream, then + lam w (the Hessian step needs only W, so
            its Grams go first and the new factorisations overlap this).  Once per iteration."""
            if grad_done[0]:
                return
            grad_done[0] = True
            if use_lag:
                lg = d.lag
                _lib.call("sglm_lag_xtr", _p(lg.occ), _p(lg.tbeg), _p(lg.tend), _p(lg.shifts),
                          lg.m, lg.K, lg.layout, lg.row0, n, P, _p(bf.R), ld, _p(act_d), na,
                          _p(bf.g), _p(lag_work), st)
            elif use_rp:
                # a factorisation chain runs beside this gradient: the kernel variant that
                # leaves it room on the SIMDs (sglm_xtr_prefer)
                cochain = (cochain_ok and XTR_COCHAIN and nref > 0 and SOLVE_INV
                           and CHOL_STREAM != "serial")
                if cochain:
                    _lib.call("sglm_xtr_prefer", 1)
                try:
                    _lib.call("sglm_xtr_bits_packed_bp", _p(d.cbits_full()), ld, P, n,
                              _p(rp_buf), grad_n, grad_bp, _p(grad_d), _p(bf.g), _p(gx_work), st)
                finally:
                    if cochain:
                        _lib.call("sglm_xtr_prefer", -1)
                # a mixed design's continuous coordinates, float64 from the same packed R
                d.mix_xtr(2, rp_buf, ld, grad_bp, None, grad_d, grad_n, bf.g)
                if g_copy is not None:
                    bf.g[g_copy[0]] = bf.g[g_copy[1]]
            else:
                d.xtr(bf.R, B, bf.g)
            if comm is not None:
                comm.sum_(bf.g[:B])
            torch.addcmul(bf.g[:B], lamp_d, beta64_d[:B], out=bf.gtot[:B])   # + lam * w

        # ---- Hessian
        if pending_inv is not None:
            # the previous iteration's deferred inversion reads bf.H: this iteration's Grams
            # (main stream) write it only after (it ran beside the line search and link)
            torch.cuda.current_stream().wait_event(pending_inv)
            pending_inv = None
        gram_comp = np.zeros(B, dtype=bool)     # fits whose Gram is computed this iteration
        pipe_groups = None
        if const_hess:
            gram_now[:] = not factored
            if not factored:
                reps = {}
                for k in act:
                    reps.setdefault(reqs[k].mask, k)
                rep_idx = np.array(sorted(reps.values()), dtype=np.int32)
                _syrk(d, bf, rep_idx, nsteps, ntile1, stats, st, exact=True, rows=gram_rows)
                sum_hess(rep_idx)
                gram_comp[rep_idx] = True
                # one float64 factor per (mask, penalty, intercept), from its mask's Gram
                f64 = _Factor64(d, bf, np.asarray([reps[reqs[k].mask] for k in k_d]),
                                np.asarray(k_d), lamp_d, st)
        else:
            # decisions planned at the end of the previous iteration (their device distances are
            # long computed): keep / form / share / alias (see _hess_plan)
            if plan is None:
                plan = hess_plan(act)
            if GRAD_FIRST and plan["form"].size == 0 and plan["npairs"] and SOLVE_INV:
                # no Hessian is certain to be formed: the gradient goes ahead of the wait for
                # the pair distances (a failed alias candidate's Gram then follows it)
                _gradient(cochain_ok=False)
            keep, form, uniq, dup, ali, fail, exact_h = hess_finish(plan)
            plan = None
            alias[:] = -1
            alias[ali] = repl[ali]
            pipe_groups = _gram_groups(form, uniq, dup) if (
                GRAM_PIPE > 0 and SOLVE_INV and CHOL_STREAM != "serial" and comm is None) else None
            if pipe_groups is None:
                # fits at their start on an all-rows mask have one weight on every row: their
                # Gram is w X^T X, from the event cross-correlations for a lagged event design
                lagg = np.array([k for k in uniq if fresh_start[k] and all_rows[k]],
                                dtype=np.int32) if use_lag_gram else np.zeros(0, np.int32)
                if lagg.size:
                    _lag_gram(d, bf, lagg, st)
                    if stats is not None:
                        stats.lag_grams += int(lagg.size)
                        stats.alg_flop += _lag_corr_flop(d.lag)
                _syrk(d, bf, np.sort(np.setdiff1d(uniq, lagg)).astype(np.int32), nsteps,
                      ntile1, stats, st, rows=gram_rows)
                sum_hess(uniq)
                for k, rk in dup:
                    bf.H[k].copy_(bf.H[rk])
            else:
                # Grams one source at a time, each group's factorisation chain started on the
                # side stream as soon as its Gram is done (below): the chains overlap the next
                # Grams instead of all waiting for the last one
                form = np.concatenate([g for _, g in pipe_groups]).astype(form.dtype)
            gram_comp[uniq] = True
            gram_now[:] = False
            gram_now[form] = True
            if stats is not None:
                stats.gram_fits += int(uniq.size)
                stats.reused += int(keep.size)
                stats.aliased += int(ali.size)
                stats.shared += int(np.sum(~exact_h[form]))
        t0 = tick("it_gram", t0)
        bf.delta[:B].zero_()
        if const_hess:
            # the float64 step on the fit's own (mask, penalty) factor; with the exact gradient
            # one refinement pass absorbs the f32 / bf16 roundings of the step
            order, nref = act, 0
            _gradient()
            t0 = tick("it_gradient", t0)
            _lib.call("sglm_chol64_solve", _p(f64.U), P, _p(f64.state), _p(act_d),
                      _p(fkey_d[act_d.long()]), na, _p(bf.gtot), _p(bf.delta), st)
        elif SOLVE_INV:
            order, nref = np.concatenate([form, keep]), form.size
            # one list: factored and kept fits on their own inverses, then the aliased fits
            # grouped by representative (tiles of <= 32 fits sharing one inverse)
            al = ali[np.argsort(repl[ali], kind="stable")] if (not const_hess and ali.size) \
                else np.zeros(0, dtype=np.int64)
            src = repl[al]
            if dist_f:
                # row-sharded: this iteration's new factorisations dealt over the ranks; a
                # rank factors and solves only on the factors it holds (its directions are
                # summed with the other ranks' below)
                fowner[order[:nref]] = comm.owners(int(nref), rot)
                rot += int(nref)
                mine_f = fowner == comm.rank
                fo, ko = order[:nref], order[nref:]
                fo, ko = fo[mine_f[fo]], ko[mine_f[ko]]
                order, nref = np.concatenate([fo, ko]), int(fo.size)
                sel = mine_f[src]
                al, src = al[sel], src[sel]
            lst = np.concatenate([order, al]).astype(np.int32)
            fsrc = np.concatenate([order, src]).astype(np.int32)
            rsc = np.concatenate([np.ones(order.size), rows[src] / rows[al]]).astype(np.float32)
            tiles = [(q, 1) for q in range(order.size)]
            q = order.size
            while q < lst.size:
                e = q
                while e < lst.size and e - q < 32 and fsrc[e] == fsrc[q]:
                    e += 1
                tiles.append((q, e - q))
                q = e
            ints = up(np.concatenate([lst, fsrc, np.asarray(tiles, np.int32).reshape(-1)]),
                      np.int32)
            rsc_d = up(rsc, np.float32)
            nl = int(lst.size)
            fact_done = None
            defer = False                  # this iteration's inverses formed after its solve
            if pending_inv is not None:
                # the last deferred inversion reads bf.fact_fits / writes Minv: the main stream
                # orders after it before rewriting the list or reading those inverses (long
                # done by now: it ran beside the previous iteration's main-stream work)
                torch.cuda.current_stream().wait_event(pending_inv)
                pending_inv = None
            if nref and CHOL_STREAM == "serial":
                bf.fact_fits[:nref].copy_(ints[:nref])
                _lib.call("sglm_chol_solve_inv", _p(bf.H), _p(bf.Minv), P, _p(bf.fact_fits), None,
                          None, int(nref), int(nref), None, 0, None, _p(bf.dshift), _p(bf.delta),
                          _p(bf.info), _p(bf.frozen), B, _p(bf.cwork), st)
            elif nref:
                # factor + invert the new Hessians on a side stream while the gradient runs.
                # Everything the main stream does first (the Grams one source at a time with
                # pipelining, then the gradient) is enqueued BEFORE the chains: a chain's graph
                # launch holds the host for ~1-2 ms (one submission per node), and the main
                # stream must not wait behind it
                side = _side_stream()
                bf.fact_fits[:nref].copy_(ints[:nref])
                chains = []
                if pipe_groups is not None:
                    off = 0
                    dsrc = dict(dup)
                    if GRAM_PIPE == 1:                 # one source per batch
                        batches = [[g] for g in pipe_groups]
                    else:                              # two batches, the larger first
                        h = (len(pipe_groups) + 1) // 2
                        batches = [pipe_groups[:h], pipe_groups[h:]]
                    for bt in batches:
                        srcs = np.array(sorted(int(r) for r, _ in bt), dtype=np.int32)
                        _syrk(d, bf, srcs, nsteps, ntile1, stats, st, rows=gram_rows)
                        nb_ = 0
                        for r, grp in bt:
                            for k in grp:
                                if int(k) != int(r):
                                    bf.H[int(k)].copy_(bf.H[int(dsrc[int(k)])])
                            nb_ += int(len(grp))
                        ready = torch.cuda.Event()
                        ready.record()
                        chains.append((ready, off, nb_))
                        off += nb_
                else:
                    ready = torch.cuda.Event()
                    ready.record()
                    # the chain is latency-bound (~0.9 ms fixed + ~0.23 ms per representative
                    # at P = 2048): a large batch runs as CHOL_SPLIT concurrent chains, each on
                    # its own side stream with its own work buffer
                    nsplit = CHOL_SPLIT if nref >= CHOL_SPLIT_MIN else 1
                    cuts = np.linspace(0, int(nref), nsplit + 1).round().astype(int)
                    chains += [(ready, int(cuts[j]), int(cuts[j + 1] - cuts[j]))
                               for j in range(nsplit) if cuts[j + 1] > cuts[j]]
                    defer = (DEFER_INV_MIN > 0 and nref >= DEFER_INV_MIN and len(chains) == 1
                             and comm is None)
                _gradient()
                t0 = tick("it_gradient", t0)
                dones = []
                for j, (ready, off, ng) in enumerate(chains):
                    sd = side if (pipe_groups is not None or j == 0) else _side_stream(j)
                    sd.wait_event(ready)
                    t_ch = time.perf_counter()
                    if defer:
                        _lib.call("sglm_chol_factor", _p(bf.H), _p(bf.Minv), P,
                                  _p(bf.fact_fits[off:]), ng, _p(bf.dshift), _p(bf.info),
                                  _p(bf.frozen), B, _p(bf.chol_work(0)), sd.cuda_stream)
                    else:
                        _lib.call("sglm_chol_solve_inv", _p(bf.H), _p(bf.Minv), P,
                                  _p(bf.fact_fits[off:]), None, None, ng, ng, None, 0, None,
                                  _p(bf.dshift), _p(bf.delta), _p(bf.info), _p(bf.frozen), B,
                                  _p(bf.chol_work(j if pipe_groups is None else 0)),
                                  sd.cuda_stream)
                    if stats is not None:
                        stats.chain_host_s += time.perf_counter() - t_ch
                    if sd is not side:
                        ev_ = torch.cuda.Event()
                        ev_.record(sd)
                        dones.append(ev_)
                for ev_ in dones:
                    side.wait_event(ev_)
                fact_done = torch.cuda.Event()
                fact_done.record(side)
                if defer:
                    # the inverses of these factors, behind the chain on the side stream
                    _lib.call("sglm_chol_invert", _p(bf.H), _p(bf.Minv), P, _p(bf.fact_fits),
                              int(nref), B, _p(bf.chol_work(0)), side.cuda_stream)
                    pending_inv = torch.cuda.Event()
                    pending_inv.record(side)
            if fact_done is None:
                _gradient()
                t0 = tick("it_gradient", t0)
            if fact_done is not None:
                torch.cuda.current_stream().wait_event(fact_done)
            if nl and defer:
                # fits on this iteration's factors: substitution on the factors (the same
                # delta = -r F^-1 F^-T g as the inverse's two GEMMs, other rounding); the rest
                # (kept factors, aliases of older representatives) on their complete inverses
                newf = np.isin(fsrc, order[:nref])
                if (~newf).any():
                    lo, fo, ro = lst[~newf], fsrc[~newf], rsc[~newf]
                    tl, q = [], 0               # runs of <= 32 fits sharing one factor
                    while q < lo.size:
                        e = q + 1
                        while e < lo.size and e - q < 32 and fo[e] == fo[q]:
                            e += 1
                        tl.append((q, e - q))
                        q = e
                    io = up(np.concatenate([lo, fo, np.asarray(tl, np.int32).reshape(-1)]),
                            np.int32)
                    no = int(lo.size)
                    _lib.call("sglm_chol_solve_inv", _p(bf.H), _p(bf.Minv), P, _p(io),
                              _p(io[no:]), _p(up(ro, np.float32)), no, 0, _p(io[2 * no:]),
                              len(tl), _p(bf.gtot), _p(bf.dshift), _p(bf.delta), _p(bf.info),
                              _p(bf.frozen), B, _p(bf.cwork), st)
                ln, fn, rn = lst[newf], fsrc[newf], rsc[newf]
                idn = up(np.stack([ln, fn]), np.int32)
                _lib.call("sglm_chol_solve_alias", _p(bf.H), P, _p(idn[0]), _p(idn[1]),
                          int(ln.size), _p(bf.gtot), _p(up(rn, np.float32)), _p(bf.delta),
                          _p(bf.frozen), B, _p(bf.cwork), st)
            elif nl:
                _lib.call("sglm_chol_solve_inv", _p(bf.H), _p(bf.Minv), P, _p(ints),
                          _p(ints[nl:]), _p(rsc_d), nl, 0, _p(ints[2 * nl:]), len(tiles),
                          _p(bf.gtot), _p(bf.dshift), _p(bf.delta), _p(bf.info), _p(bf.frozen),
                          B, _p(bf.cwork), st)
            if comm is not None and (dist_f or not comm.distribute):
                owned = np.zeros(B0, dtype=np.uint8)
                owned[lst] = 1
                comm.directions_(bf.delta[:B], up(owned, np.uint8))
        else:
            order, nref = np.concatenate([form, keep]), form.size
            _gradient()
            t0 = tick("it_gradient", t0)
            fits_d = up(order, np.int32)
            _lib.call("sglm_chol_solve_mixed", _p(bf.H), P, _p(fits_d), int(order.size),
                      int(nref), _p(bf.gtot), _p(bf.dshift), _p(bf.delta), _p(bf.info),
                      _p(bf.frozen), B, _p(bf.cwork), st)
        if not SOLVE_INV and not const_hess and ali.size:
            # the representatives' factors are complete: solve the aliased fits on them
            src = repl[ali]
            al_d = up(np.stack([ali, src]), np.int32)
            rscale_d = up(rows[src] / rows[ali], np.float32)
            _lib.call("sglm_chol_solve_alias", _p(bf.H), P, _p(al_d[0]), _p(al_d[1]),
                      int(ali.size), _p(bf.gtot), _p(rscale_d), _p(bf.delta), _p(bf.frozen), B,
                      _p(bf.cwork), st)
        factored = True
        aa_idx = None
        if use_aa:
            fepoch[form] += 1
            src_now = np.where(alias[act] >= 0, alias[act], act)
            key_now = src_now * 1_000_000 + fepoch[src_now]
            aa_idx = up(act, np.int64)
            selm = (aa_key[act] == key_now) & ~gram_now[act] & (aa_t[act] > 0)
            sel = np.flatnonzero(selm)
            if AA_KERNEL:
                # one launch (sglm_aa_step): the correction, the raw directions kept, rm
                _lib.call("sglm_aa_step", P, p, na, _p(act_d), _p(up(selm.astype(np.uint8))),
                          _p(up(aa_t[act], np.float32)), _p(bf.delta), _p(aa_raw), _p(aa_used),
                          _p(bf.gtot), _p(aa_rm), st)
                if stats is not None:
                    stats.aa_fit_iters += int(sel.size)
                sel = sel[:0]
            else:
                raw = bf.delta[aa_idx]                 # this iteration's raw directions
                aa_rm.zero_()
            if sel.size:
                # d = f - gamma (dbeta + df), gamma = df.f / df.df (f: raw direction, df its
                # change on the same factor, dbeta the previous step taken); kept only when
                # it is a descent direction and gamma lies in [-2, 0.5]
                sel_d = up(sel, np.int64)
                f = raw[sel_d]
                df = f - aa_raw[aa_idx[sel_d]]
                db = aa_used[aa_idx[sel_d]] * up(aa_t[act[sel]], np.float32)[:, None]
                den = (df * df).sum(1)
                gam = (df * f).sum(1) / den.clamp_min(1e-30)
                dnew = f - gam[:, None] * (db + df)
                gdn = (bf.gtot[aa_idx[sel_d]].float() * dnew).sum(1)
                good = (den > 1e-12 * (f * f).sum(1)) & (gam >= -2.0) & (gam <= 0.5) & (gdn < 0)
                bf.delta[aa_idx[sel_d]] = torch.where(good[:, None], dnew, f)
                aa_rm[aa_idx[sel_d], 0] = f[:, :p].abs().amax(1)
                aa_rm[aa_idx[sel_d], 1] = f[:, p].abs()
                if stats is not None:
                    stats.aa_fit_iters += int(sel.size)
            if not AA_KERNEL:
                aa_raw[aa_idx] = raw
            aa_key[act] = key_now
        # the directions are rounded to bf16 in place (X d on one MFMA piece); the step below
        # uses the rounded values, so eta stays X beta and the fixed point (exact gradient) is
        # unchanged -- the rounding only perturbs the Newton direction by 2^-9 relative
        d.eta(bf.delta, bf.deta, slots=act_d, direction=True)
        # per-fit scalars of the line search and the stopping rule, reduced on the device
        # over the coefficients (no B x P array crosses to the host): g.d, the penalty terms
        # lam|w|^2, 2 lam w.d, lam|d|^2, max|d| and max|w + t d| for every trial step t
        sc = sc_d[: na * (6 + nts)]
        _lib.call("sglm_step_scalars", P, P if STOP_LEGACY else p, na, _p(act_d), _p(bf.gtot), _p(beta64_d), _p(bf.delta),
                  _p(lamp_d), _p(ts_all), nts, _p(sc), st)
        t0 = tick("it_solve_eta", t0)
        # ---- line search (rows of L, dmax and sc: active fits in slot order)
        _lib.call("sglm_loss_trials_max", fam, power, n, ld, na, _p(act_d), _p(bf.eta),
                  _p(bf.deta), _p(prob.Y), _p(prob.M), _p(fit_resp), _p(fit_mask), _p(tv1), 5,
                  _p(Ltr), _p(dmax_d), _p(xtr_work), st)
        if comm is not None:
            comm.sum_(Ltr[: na * 5])
            comm.max_(dmax_d[:na])
        L_h[: na * 5].copy_(Ltr[: na * 5], non_blocking=True)
        dmax_h[:na].copy_(dmax_d[:na], non_blocking=True)
        sc_h = _pinned("sc", sc.numel(), torch.float64)
        sc_h.copy_(sc, non_blocking=True)
        if use_aa:
            aa_rm_h.copy_(aa_rm.view(-1), non_blocking=True)
            aa_used[aa_idx] = bf.delta[aa_idx]       # the rounded directions the step uses
        if dev_dec:
            up.batch()
            prev_d = up(prev_rel[act], np.float64)
            fresh_d = up(((gram_now[act] & exact_h[act]) | const_hess).astype(np.uint8))
            nit_d = up(n_iter[act], np.int32)
            mit_d = up(max_iter[act], np.int32)
            up.flush()
            _lib.call("sglm_step_decide", na, _p(act_d), _p(Ltr), _p(sc), nts, _p(ts_all),
                      ARMIJO_SIGMA, float(tol), STOP_SCALE_FLOOR, int(STOP_LEGACY),
                      _p(aa_rm) if use_aa else None, _p(prev_d), _p(fresh_d), _p(nit_d),
                      _p(mit_d), _p(dec64[0]), _p(dec32), _p(dec64[1]), _p(dec64[2]), _p(deci),
                      _p(deci[B0:]), _p(deci[2 * B0:]), _p(deci[3 * B0:]), _p(deci[4 * B0:]), st)
            dec64_h.copy_(dec64.view(-1), non_blocking=True)
            deci_h.copy_(deci, non_blocking=True)
            ev_dec.record()
            # the step (coefficients) and the next link with the fused predictor update, for
            # every active fit (t = 0 where stage 2 decides): the GPU runs them while the host
            # reads the verdicts and plans the next iteration
            _lib.call("sglm_step_update", P, na, _p(act_d), _p(dec64[0]), _p(bf.delta),
                      _p(beta64_d), st)
            _lib.call("sglm_link_update_rp", fam, power, n, ld, na, _p(act_d), _p(bf.eta),
                      _p(prob.Y), _p(prob.M), _p(fit_resp), _p(fit_mask), _p(bf.W), None,
                      _p(rp_buf), pad_to(na, 32), _p(deci[2 * B0:]), _p(dec32), _p(bf.deta), st)
        t_sync = time.perf_counter()
        if dev_dec:
            ev_dec.synchronize()                 # the iteration's round trip (not the link)
        else:
            torch.cuda.current_stream().synchronize()          # the iteration's round trip
        if stats is not None:
            stats.sync_wait_s += time.perf_counter() - t_sync
            stats.roundtrips += 1
        up.synced()
        L = L_h[: na * 5].numpy().reshape(na, 5).copy()
        dmaxeta = dmax_h[:na].numpy().astype(np.float64)
        scn = sc_h.numpy().reshape(na, -1).copy()
        gdir, A_, B_, C_, maxd = scn[:, 0], scn[:, 1], scn[:, 2], scn[:, 3], scn[:, 4]
        maxb = scn[:, 5:5 + nts]                # max|w_j + t d_j| (j < p) for t in TS_ALL
        maxdi = scn[:, 5 + nts]                 # |d| of the intercept
        ts = np.array([0.0, 1.0, 0.5, 0.25, 0.125])

        def objectives(Lm, tv):
            return Lm + 0.5 * (A_[:, None] + 2 * tv[None, :] * B_[:, None]
                               + tv[None, :] ** 2 * C_[:, None])
        if dev_dec:
            # the device's stage-1 verdicts (sglm_step_decide)
            dh = dec64_h.numpy().reshape(3, B0)
            di = deci_h.numpy()
            step_a = dh[0, :na].copy()
            tix = di[B0:B0 + na].astype(np.int64)
            dflags = di[:na].copy()
            hit = (dflags & 1) != 0
        else:
            step_a = np.zeros(na)
            tix = np.zeros(na, dtype=np.int64)  # index of the chosen step in TS_ALL
            obj = objectives(L, ts)
            ok = ((obj[:, 1:] - obj[:, :1] <= ARMIJO_SIGMA * ts[None, 1:] * gdir[:, None]) |
                  (np.abs(obj[:, 1:] - obj[:, :1]) <= 1e-13 * np.abs(obj[:, :1])))
            first = np.argmax(ok, axis=1)
            hit = ok[np.arange(na), first]
            step_a[hit] = ts[1:][first[hit]]
            tix[hit] = 1 + first[hit]
        more = np.flatnonzero(~hit)                         # positions in act
        if more.size:
            sub_d = up(act[more], np.int32)
            _lib.call("sglm_loss_trials", fam, power, n, ld, int(more.size), _p(sub_d),
                      _p(bf.eta), _p(bf.deta), _p(prob.Y), _p(prob.M), _p(fit_resp),
                      _p(fit_mask), _p(tv2), 7, _p(Ltr), _p(xtr_work), st)
            if comm is not None:
                comm.sum_(Ltr[: more.size * 7])
            t_sync = time.perf_counter()
            L2 = Ltr[: more.size * 7].view(more.size, 7).cpu().numpy()
            if stats is not None:
                stats.sync_wait_s += time.perf_counter() - t_sync
                stats.roundtrips += 1
            ts2 = TV2.astype(np.float32).astype(np.float64)
            obj0 = objectives(L[:, :1], np.zeros(1))[more]
            o2 = L2 + 0.5 * (A_[more, None] + 2 * ts2[None, :] * B_[more, None]
                             + ts2[None, :] ** 2 * C_[more, None])
            ok2 = o2 - obj0 <= ARMIJO_SIGMA * ts2[None, :] * gdir[more, None]
            f2 = np.argmax(ok2, axis=1)
            h2 = ok2[np.arange(more.size), f2]
            step_a[more[h2]] = ts2[f2[h2]]
            tix[more[h2]] = 5 + f2[h2]
        t0 = tick("it_linesearch", t0)
        # ---- stopping decisions first (they need only this iteration's readback), so the
        # coefficient / predictor update and the next link go to the GPU before the host's
        # remaining bookkeeping (drift, sharing / aliasing flags, statistics, the next plan)
        # the step is measured against the coefficients' own scale (max|w_j| over j < p after
        # the step, the intercept excluded), floored at STOP_SCALE_FLOOR: the parity tests
        # measure errors relative to max|coef|, so a fit with small coefficients (strong
        # penalty) must converge in those units too
        if STOP_LEGACY:
            scale = 1.0 + maxb[np.arange(na), tix]
            prop = maxd / scale                        # the proposed Newton step
        else:
            # coefficients in units of their own scale, the intercept in absolute units (it
            # is O(1) and its parity bar is absolute): the measures the parity tests apply
            scale = np.maximum(maxb[np.arange(na), tix], STOP_SCALE_FLOOR)
            prop = np.maximum(maxd / scale, maxdi)
        relv = step_a * prop
        if use_aa:
            # a secant-corrected step can be small while the raw Newton step is not
            # (cancellation in f - gamma (dbeta + df)): such a fit is not converged
            rm = aa_rm_h.numpy().reshape(B0, 2)[act].astype(np.float64)
            rawp = np.maximum(rm[:, 0] / scale, rm[:, 1])
            relv = np.maximum(relv, rawp)
        stepa = step_a
        fresh = (gram_now[act] & exact_h[act]) | const_hess
        ls_fail = stepa == 0.0
        stop_tol = ~ls_fail & (relv <= tol)
        # stagnation (the f32 noise floor): a step no better than half the previous one, judged
        # only on steps taken with a fresh Hessian -- a kept factor contracts by up to
        # e^(c D) - 1, which may legitimately exceed 1/2 (Gaussian: the exact Hessian, always).
        # It stops the fit but is NOT convergence: the fit is reported unconverged.
        stop_stag = (~ls_fail & ~stop_tol & fresh & (relv < 1e-4)
                     & (relv >= 0.5 * prev_rel[act]))
        # a failed search on a fresh Hessian: converged only if the proposed step itself is
        # within tol (the iterate already sits at the minimiser up to rounding)
        stop_fail = ls_fail & fresh
        if dev_dec and hit.any():
            # the device's verdicts for the fits its stage 1 decided (the packed R rows of the
            # next gradient follow them); the host's own formulas only for the stage-2 fits
            relv[hit] = dh[1, :na][hit]
            prop[hit] = dh[2, :na][hit]
            stop_tol[hit] = (dflags[hit] & 16) != 0
            stop_stag[hit] = (dflags[hit] & 32) != 0
        stop = stop_tol | stop_stag | stop_fail
        conv_now = stop_tol | (stop_fail & (prop <= tol))
        n_iter[act] += 1
        out_of_iters = ~stop & (n_iter[act] >= max_iter[act])
        cont = ~stop & ~out_of_iters
        nxt = act[cont]
        if dev_dec and not np.array_equal(cont[hit], (dflags[hit] & 512) != 0):
            raise RuntimeError("sglm_step_decide disagrees with the host's stopping rule")
        # predictor update eta += t d_eta: fused into the next iteration's link for the fits
        # that continue (0/1 designs), a plain axpy for the others
        linked = None
        up.batch()
        step_d = up(step_a, np.float64)
        if dev_dec:
            # the device enqueued the step and the link; the stage-2 fits (t = 0 there) take
            # their step now, and those that continue refresh their link at the same rows
            if more.size:
                mv = more[step_a[more] != 0.0]
                if mv.size:
                    mv_d = up(act[mv], np.int32)
                    ms_d = up(step_a[mv], np.float64)
                    mt_d = up(step_a[mv], np.float32)
                    mc = mv[cont[mv]]
                    if mc.size:
                        mc_d = up(act[mc], np.int32)
                        mr_d = up(di[2 * B0:2 * B0 + na][mc], np.int32)
                    up.flush()
                    _lib.call("sglm_step_update", P, int(mv.size), _p(mv_d), _p(ms_d),
                              _p(bf.delta), _p(beta64_d), st)
                    _lib.call("sglm_eta_axpy", n, ld, int(mv.size), _p(mv_d), _p(mt_d),
                              _p(bf.deta), _p(bf.eta), st)
                    if mc.size:
                        _lib.call("sglm_link_update_rp", fam, power, n, ld, int(mc.size),
                                  _p(mc_d), _p(bf.eta), _p(prob.Y), _p(prob.M), _p(fit_resp),
                                  _p(fit_mask), _p(bf.W), None, _p(rp_buf), pad_to(na, 32),
                                  _p(mr_d), None, None, st)
            up.flush()
            grad_d, grad_n, grad_bp = deci[3 * B0:], int(di[4 * B0]), pad_to(na, 32)
            dev_linked = True
        elif fused and nxt.size:
            done = np.flatnonzero(~cont & (step_a != 0.0))
            if done.size:
                done_d, tdone_d = up(act[done], np.int32), up(step_a[done], np.float32)
            linked = up(nxt, np.int32)
            tcont_d = up(step_a[cont], np.float32)
            up.flush()
            _lib.call("sglm_step_update", P, na, _p(act_d), _p(step_d), _p(bf.delta),
                      _p(beta64_d), st)
            if done.size:
                _lib.call("sglm_eta_axpy", n, ld, int(done.size), _p(done_d), _p(tdone_d),
                          _p(bf.deta), _p(bf.eta), st)
            _lib.call("sglm_link_update", fam, power, n, ld, int(nxt.size), _p(linked),
                      _p(bf.eta), _p(prob.Y), _p(prob.M), _p(fit_resp), _p(fit_mask), _p(bf.W),
                      R_out, Rp_out, _p(tcont_d), _p(bf.deta), st)
        else:
            t32_d = up(step_a, np.float32)
            up.flush()
            _lib.call("sglm_step_update", P, na, _p(act_d), _p(step_d), _p(bf.delta),
                      _p(beta64_d), st)
            _lib.call("sglm_eta_axpy", n, ld, na, _p(act_d), _p(t32_d), _p(bf.deta),
                      _p(bf.eta), st)
        # ---- bookkeeping of this iteration (overlaps the update on the GPU)
        if not const_hess:
            drift[act] += step_a * dmaxeta            # max_i |t d_eta_i| over the fit's rows
        fresh_start[act[step_a != 0.0]] = False
        aa_t[act] = step_a
        if stats is not None:
            stats.newton_iters += 1
            stats.fit_iters += na
            # SURVEY.md §8(d) F per fit-iteration, charged for work actually done: the Gram
            # term only where a Gram was computed (not for a Hessian shared from another fit),
            # the factorisation where a new factor was formed (a kept or aliased factor costs
            # the two triangular solves only)
            pa = float(p + 1)
            nr = rows[act]
            rest = float(np.sum(np.where(gram_now[act], pa ** 3 / 3, 0.0)
                                + 4.0 * nr * pa + 2 * pa * pa))
            stats.alg_flop += rest              # the Grams were charged where they were formed
            stats.alg_flop_dense += rest + float(np.sum(np.where(gram_comp[act],
                                                                 nr * pa * (pa + 1), 0.0)))
            stats.gram_fit_iters += int(np.sum(gram_comp[act]))
        # a failed line search on a kept (stale) factor, or on a Hessian shared from a lambda
        # neighbour, is not a verdict: the next iteration forms a fresh Hessian of the fit's
        # own instead of stopping it
        if not const_hess:
            drift[act[ls_fail & ~fresh]] = np.inf
            no_share[act[ls_fail & gram_now[act] & ~exact_h[act]]] = True
            # a fit whose step on the representative's factor failed, or contracted slowly,
            # forms its own Hessians from here on
            was_alias = alias[act] >= 0
            slow = was_alias & (relv > XMASK_SLOW * prev_rel[act]) & (relv > tol)
            drop = was_alias & (ls_fail | slow)
            no_alias[act[drop]] = True
            if stats is not None:
                stats.stops["alias_dropped"] += int(np.sum(drop))
        active[act[stop]] = False
        converged[act[stop]] = conv_now[stop]
        active[act[out_of_iters]] = False
        if stats is not None and stats.iter_log is not None:
            stats.iter_log.append(dict(
                it=it, active=int(na), keep=int(0 if const_hess else keep.size),
                alias=int(0 if const_hess else ali.size), form=int(nref if not dist_f else -1),
                grams=int(gram_comp.sum()), stop_tol=int(stop_tol.sum()),
                ls_fail=int(ls_fail.sum()), step1=int(np.sum(step_a == 1.0)),
                rel_max=float(relv.max()), rel_med=float(np.median(relv)),
                lam_active=[float(lam[k]) for k in act[~stop]][:40],
                rate=[float(x) for x in (relv / np.maximum(prev_rel[act], 1e-300))[~stop]][:40]))
        prev_rel[act] = relv
        if stats is not None:
            stats.stops["tol"] += int(np.sum(stop_tol))
            stats.stops["stagnation"] += int(np.sum(stop_stag))
            stats.stops["line_search_converged"] += int(np.sum(stop_fail & (prop <= tol)))
            stats.stops["line_search_failed"] += int(np.sum(stop_fail & (prop > tol)))
            stats.stops["max_iter"] += int(np.sum(out_of_iters))
            stats.stops["stale_factor_retry"] += int(np.sum(ls_fail & ~fresh))
        if not const_hess and nxt.size:
            # the next iteration's Hessian decisions and their distances, enqueued behind
            # this iteration's predictor update (read back without a stall next iteration)
            plan = hess_plan(nxt)
        t0 = tick("it_update", t0)

    if pending_inv is not None:              # a deferred inversion still reads bf.H / fact_fits
        torch.cuda.current_stream().wait_event(pending_inv)
    # unpenalised fits: the minimum-norm point of the solution set (lstsq's answer on a
    # rank-deficient design; the fitted values on the fit's rows are unchanged)
    pf = np.zeros(0, dtype=np.int64)
    if f64 is not None:
        pf = np.flatnonzero(lam0 & (fkey >= 0))
        f64.minnorm(d, bf, pf, fkey[pf], beta64_d, st)
    # final linear predictor from the final coefficients, enqueued before the readbacks so
    # the host's one wait covers it.  The loop keeps eta = X beta up to one f32 rounding per
    # step, so only fits whose beta moved without eta (the minimum-norm projection) or that
    # took many steps are recomputed (the full pass costs ~1.2 ms on a 120-fit grid)
    bf.beta[:B0].copy_(beta64_d)
    if ETA_FINAL_ALL or d.rbits is None or not ETA_BITS:
        d.eta(bf.beta, bf.eta)
    else:
        ref = np.union1d(pf, np.flatnonzero(n_iter > ETA_FINAL_ITERS))
        if ref.size:
            d.eta(bf.beta, bf.eta, slots=torch.from_numpy(ref.astype(np.int32)).to(dev))
    out_iter[:] = n_iter
    out_conv[:] = converged
    if dist_f:
        # a factor's dropped-pivot count lives on the rank that formed it
        inf = bf.info[:B].clone()
        inf[torch.from_numpy(fowner != comm.rank).to(dev)] = 0
        comm.sum_owned_(inf)
    else:
        inf = bf.info[:B]
    parts = [beta64_d.reshape(-1), inf.to(torch.float64)]
    if f64 is not None:
        parts.append(f64.counts[:, 1].to(torch.float64))
    outs = torch.cat(parts).cpu().numpy()
    out_beta[:] = outs[: B0 * P].reshape(B0, P)
    out_info[:] = outs[B0 * P:B0 * P + B0].astype(np.int64)
    if f64 is not None:
        # coordinates the float64 factor found dependent or zero
        cnt = outs[B0 * P + B0:].astype(np.int64)
        has = fkey >= 0
        out_info[has] = np.maximum(0 if const_hess else out_info[has], cnt[fkey[has]])
    bf.prob = bf.keep = bf.up = bf.fit_mask_d = None   # drop the compacted designs with the problem
    bf.mixS = None
    res = []
    for k, r in enumerate(reqs0):
        res.append(FitResult(coef=out_beta[k, :p].copy(),
                             intercept=float(out_beta[k, p]) if r.fit_intercept else 0.0,
                             n_iter=int(out_iter[k]), converged=bool(out_conv[k]),
                             dropped=int(out_info[k])))
    return res, bf.eta


# squared-loss fits of a 0/1 (or mixed) design in Gram space: the exact mask Gram (integer
# counts in f32, a mixed design's continuous rows in float64), the exact X^T (m y) (digit
# planes), a float64 factor per (mask, penalty, intercept), the solve and GRAM_LS_REFINE float64
# refinements -- no pass over the rows per iteration, and no f32 residual in the fixed point
GRAM_LS = __import__("os").environ.get("SGLM_GRAM_LS", "1") == "1"
GRAM_LS_REFINE = int(__import__("os").environ.get("SGLM_GRAM_LS_REFINE", "2"))
# device bytes the float64 factors of one _gram_ls chunk may take
GRAM_LS_FACTOR_BYTES = float(__import__("os").environ.get("SGLM_GRAM_LS_FACTOR_BYTES", "16e9"))


def _gram_ls(prob: Problem, reqs: List[FitReq], stats: Optional[IrlsStats], bufs, comm):
    """Squared-loss (OLS / Ridge) fits of a 0/1 or mixed design: x = (G + lam I')^-1 X^T (m y)
    in float64 -- the normal equations sklearn's Ridge(solver='cholesky') solves
    (_ridge.py:201-213) and, with the minimum-norm projection of unpenalised fits on their exact
    rank decisions, lstsq's LinearRegression answer (_base.py:701; backend/sglm.py:96-105).
    G = the mask's exact Gram (sglm_syrk_cbits at the mask multiplicities: integer counts, exact
    in f32 below 2^24; a mixed design's continuous rows in float64), X^T (m y) exact to float64
    rounding (xtv_digits); the solve on the float64 factor (sglm_chol64_factor_mixed) plus
    GRAM_LS_REFINE float64 refinements r = c - (G + lam I') x (sglm_chol64_resid).  Returns
    (results, final eta [B][ld]) like irls()."""
    d = prob.design
    B0, P, ld, n, p = len(reqs), d.P, d.ld, d.n, d.p
    dev = d.device
    bf = (bufs or _scratch().buf).get(B0, P, ld, dev)
    st = _stream()
    up = _Uploads(dev)
    fmask_h = np.array([r.mask for r in reqs], dtype=np.int32)
    lam = np.array([float(r.lam) for r in reqs])
    fi = np.array([1.0 if r.fit_intercept else 0.0 for r in reqs])
    bf.prob, bf.fit_mask, bf.up, bf.fit_mask_d = prob, fmask_h, up, None
    bf.mixS = {}
    scal = up(np.concatenate([lam, fi]), np.float64)
    lam_d, fi_d = scal[:B0], scal[B0:]
    # coordinate shifts: lam on the predictors, 0 on a fitted intercept, -1 excluded (an
    # unfitted intercept, the padding)
    bf.dshift.fill_(-1.0)
    bf.dshift[:B0, :p] = lam_d[:, None]
    bf.dshift[:B0, p] = fi_d - 1.0
    lamp_d = torch.zeros((B0, P), dtype=torch.float64, device=dev)
    lamp_d[:, :p] = lam_d[:, None]
    # one exact Gram per distinct mask (weights = the mask's multiplicities)
    mrep = {}
    for k, r in enumerate(reqs):
        mrep.setdefault(int(r.mask), k)
    rep = np.array(sorted(mrep.values()), dtype=np.int32)
    bf.W[up(rep, np.int64)] = prob.M[up(fmask_h[rep], np.int64)].float()
    gram_rows = np.array([float(prob.mask_nnz(int(r.mask))) if comm is not None
                          else prob.mask_count(int(r.mask)) for r in reqs])
    nsteps = (n + 31) // 32
    ntile1 = (P // 256) * (P // 256 + 1) // 2
    _syrk(d, bf, rep, nsteps, ntile1, stats, st, exact=True, rows=gram_rows)
    if comm is not None:
        for k in rep:
            comm.sum_(bf.H[int(k)])
            if int(k) in bf.mixS:
                comm.sum_(bf.mixS[int(k)])
    # X^T (m y) of every distinct (response, mask), exact to float64 rounding
    pairs = sorted(set((int(r.resp), int(r.mask)) for r in reqs))
    pidx = {pr: i for i, pr in enumerate(pairs)}
    c = torch.empty((len(pairs), P), dtype=torch.float64, device=dev)
    xtv_digits(d, prob.M, prob.y64_rows(), pairs, c)
    if comm is not None:
        comm.sum_(c)
    cidx = np.array([pidx[(int(r.resp), int(r.mask))] for r in reqs], dtype=np.int32)
    # one float64 factor per (mask, penalty, intercept); the unpenalised fits' factors first
    lam0 = lam == 0.0
    keys, k_h, k_d = {}, [], []
    fkey = np.full(B0, -1, dtype=np.int64)
    for k in np.argsort(~lam0, kind="stable"):
        r = reqs[k]
        key = (int(r.mask), float(r.lam), bool(r.fit_intercept))
        if key not in keys:
            keys[key] = len(k_h)
            k_h.append(mrep[int(r.mask)])
            k_d.append(int(k))
        fkey[k] = keys[key]
    x = torch.zeros((B0, P), dtype=torch.float64, device=dev)
    res_d = torch.empty_like(x)
    dropped = torch.zeros(len(k_h), dtype=torch.float64, device=dev)
    # the factors in chunks of keys within GRAM_LS_FACTOR_BYTES (a factor and, for the
    # unpenalised keys, the minimum-norm work: 16 B per P^2 entry each)
    per = max(1, int(GRAM_LS_FACTOR_BYTES // (16 * P * P)))
    k_h, k_d = np.asarray(k_h), np.asarray(k_d)
    for a in range(0, len(k_h), per):
        b = min(len(k_h), a + per)
        sel = np.flatnonzero((fkey >= a) & (fkey < b))
        nq = int(sel.size)
        f64 = _Factor64(d, bf, k_h[a:b], k_d[a:b], lamp_d, st)
        ints = up(np.concatenate([sel, fkey[sel] - a, cidx[sel], k_h[a:b]]).astype(np.int32))
        fits_d, fsrc_d, csrc_d = ints[:nq], ints[nq:2 * nq], ints[2 * nq:3 * nq]
        hsrc_d = ints[3 * nq:]
        _lib.call("sglm_chol64_solve_add", _p(f64.U), P, _p(f64.state), _p(fits_d),
                  _p(fsrc_d), _p(csrc_d), nq, _p(c), _p(x), st)
        S, k_c, cmap = f64._S, (d.k if f64._S is not None else 0), (
            d._mix["cmap"] if f64._S is not None else None)
        for _ in range(GRAM_LS_REFINE):
            _lib.call("sglm_chol64_resid", _p(bf.H), P, _p(hsrc_d), _p(S), k_c, _p(cmap),
                      _p(fits_d), _p(fsrc_d), _p(csrc_d), nq, _p(c), _p(lamp_d),
                      _p(bf.dshift), _p(x), _p(res_d), st)
            _lib.call("sglm_chol64_solve_add", _p(f64.U), P, _p(f64.state), _p(fits_d),
                      _p(fsrc_d), None, nq, _p(res_d), _p(x), st)
        # unpenalised fits: the minimum-norm point of the solution set (lstsq)
        pf = sel[lam0[sel]]
        f64.minnorm(d, bf, pf, fkey[pf] - a, x, st)
        dropped[a:b] = f64.counts[:, 1].to(torch.float64)
        del f64
    bf.beta[:B0].copy_(x)
    d.eta(bf.beta, bf.eta)
    outs = torch.cat([x.reshape(-1), dropped]).cpu().numpy()
    if stats is not None:
        stats.newton_iters += 1
        stats.fit_iters += B0
        stats.gram_fits += int(rep.size)
        stats.gram_fit_iters += int(rep.size)
        stats.rank_grams += int(rep.size)
        stats.roundtrips += 1
        stats.stops["tol"] += B0
        pa = float(p + 1)
        nr = np.array([prob.mask_count(int(reqs[k].mask)) for k in rep])
        stats.alg_flop += float(np.sum(nr * pa * (pa + 1)) + len(k_h) * pa ** 3 / 3
                                + B0 * (1 + GRAM_LS_REFINE) * 4 * pa * pa)
    xb = outs[: B0 * P].reshape(B0, P)
    cnt = outs[B0 * P:].astype(np.int64)
    bf.prob = bf.up = bf.mixS = None
    res = []
    for k, r in enumerate(reqs):
        res.append(FitResult(coef=xb[k, :p].copy(),
                             intercept=float(xb[k, p]) if r.fit_intercept else 0.0,
                             n_iter=1 + GRAM_LS_REFINE, converged=True,
                             dropped=int(cnt[fkey[k]])))
    return res, bf.eta


IRLS_GROUPS = int(__import__("os").environ.get("SGLM_IRLS_GROUPS", "1"))
IRLS_GROUP_MIN = int(__import__("os").environ.get("SGLM_IRLS_GROUP_MIN", "24"))            # fits per group below which the batch is not split


def _family_key(r: FitReq, rows: float):
    """Cross-mask family of a fit (see HESS_XMASK_TOL): response, penalty per row, intercept."""
    if r.lam > 0 and rows > 0:
        return (r.resp, float("%.12g" % (r.lam / rows)), bool(r.fit_intercept))
    return None


GROUP_SPLIT = __import__("os").environ.get("SGLM_GROUP_SPLIT", "contig")


def _partition(reqs: List[FitReq], ngroups: int, rows=None) -> List[List[int]]:
    """Fit indices per group.  With cross-mask families (log link, HESS_XMASK_TOL > 0) the
    unit is a family -- a penalty's split fits and refit, which share the refit's factor --
    and the families, in penalty order, are cut into contiguous groups (lambda-neighbours share
    Grams) or dealt in snake order (SGLM_GROUP_SPLIT=snake).  Otherwise whole row masks go to
    the lighter group (fits of one mask share their first Hessian and the lambda-path Hessian
    sharing); with fewer masks than groups the largest mask's fits are dealt alternately in
    penalty order."""
    if (rows is not None and HESS_XMASK_TOL > 0 and reqs[0].family == FAM_TWEEDIE_LOG):
        fams = {}
        for i, r in enumerate(reqs):
            fams.setdefault(_family_key(r, rows[i]) or ("solo", i), []).append(i)
        units = sorted(fams.values(), key=lambda u: (reqs[u[0]].lam / max(rows[u[0]], 1.0), u[0]))
        if len(units) >= ngroups:
            out = [[] for _ in range(ngroups)]
            if GROUP_SPLIT == "snake":
                for q, u in enumerate(units):
                    g = q % (2 * ngroups)
                    out[g if g < ngroups else 2 * ngroups - 1 - g] += u
            else:
                cut = np.linspace(0, len(units), ngroups + 1).round().astype(int)
                for g in range(ngroups):
                    for u in units[cut[g]:cut[g + 1]]:
                        out[g] += u
            return [sorted(o) for o in out if o]
    by_mask = {}
    for i, r in enumerate(reqs):
        by_mask.setdefault(r.mask, []).append(i)
    units = [sorted(v, key=lambda i: reqs[i].lam) for v in by_mask.values()]
    while len(units) < ngroups:
        units.sort(key=len)
        big = units.pop()
        if len(big) < 2:
            units.append(big)
            break
        units += [big[0::2], big[1::2]]
    cost = [0.0] * ngroups
    out = [[] for _ in range(ngroups)]
    for u in sorted(units, key=len, reverse=True):
        g = int(np.argmin(cost))
        out[g] += u
        cost[g] += len(u)
    return [sorted(o) for o in out if o]


def irls_scored(prob: Problem, reqs: List[FitReq], sets: np.ndarray,
                stats: Optional[IrlsStats] = None, ngroups: Optional[int] = None, comm=None):
    """IRLS + score sums for a batch, as ``ngroups`` independent fit groups, each driven by
    its own host thread on its own HIP stream.  A group's latency-bound phases (the blocked
    Cholesky chain, the host decisions between iterations) then run while another group's
    Gram keeps the MFMA busy.  Returns (results, score sums [B, 2, 2]) in request order."""
    require_gpu()
    ng = IRLS_GROUPS if ngroups is None else int(ngroups)
    fam, power = reqs[0].family, float(reqs[0].power)
    fresp = [r.resp for r in reqs]
    # groups pay off when each still fills the chip with Gram work (C4 on one GPU: 120 fits);
    # a rank's share at 8 GPUs (~15 fits) runs as one group
    rows = [prob.mask_stats(r.resp, r.mask)[0] for r in reqs]
    parts = (_partition(reqs, ng, rows) if ng > 1 and len(reqs) >= IRLS_GROUP_MIN * ng
             and comm is None else [list(range(len(reqs)))])
    if len(parts) == 1:
        res, eta = irls(prob, reqs, stats=stats, comm=comm)
        return res, score_sums(prob, fam, power, eta, fresp, sets, comm=comm)
    d = prob.design
    # shared lazily-built state, built once here before the threads start
    for r in reqs:
        prob.mask_stats(r.resp, r.mask)
    if d.xbits is not None and SYRK_CBITS:
        for m in sorted({r.mask for r in reqs}):
            prob.compact(m)
    if d.xbits is not None and XTR_BITS:
        d.cbits_full()
    main = torch.cuda.current_stream()
    out = [None] * len(parts)
    errs = []
    parent = _scratch()
    streams = []
    for g in range(len(parts)):
        key = (d.device, g)
        if key not in parent.streams:
            parent.streams[key] = torch.cuda.Stream(device=d.device)
        streams.append(parent.streams[key])

    def run(g, idx):
        try:
            _TLS.scratch = parent.groups.setdefault(g, _Scratch())
            s = streams[g]
            s.wait_stream(main)
            with torch.cuda.stream(s):
                sg = None
                if stats is not None:
                    sg = IrlsStats(record=stats.record, trace_phases=stats.trace_phases,
                                   host_phases=stats.host_phases)
                res, eta = irls(prob, [reqs[i] for i in idx], stats=sg)
                sums = score_sums(prob, fam, power, eta, [fresp[i] for i in idx], sets[idx])
            s.synchronize()
            out[g] = (res, sums, sg)
        except BaseException as e:  # re-raised in the caller's thread
            errs.append(e)

    ths = [threading.Thread(target=run, args=(g, idx)) for g, idx in enumerate(parts)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    res = [None] * len(reqs)
    sums = np.zeros((len(reqs), 2, 2))
    for (rg, sg_sums, sg), idx in zip(out, parts):
        for q, i in enumerate(idx):
            res[i] = rg[q]
            sums[i] = sg_sums[q]
        if stats is not None and sg is not None:
            stats.syrk_events += sg.syrk_events
            stats.syrk_bytes += sg.syrk_bytes
            stats.fit_iters += sg.fit_iters
            stats.gram_fits += sg.gram_fits
            stats.gram_fit_iters += sg.gram_fit_iters
            stats.reused += sg.reused
            stats.aliased += sg.aliased
            stats.shared += sg.shared
            stats.sync_wait_s += sg.sync_wait_s
            stats.roundtrips += sg.roundtrips
            stats.alg_flop += sg.alg_flop
            for k, v in sg.stops.items():
                stats.stops[k] += v
            for k, v in sg.phases.items():
                stats.phases[k] = stats.phases.get(k, 0.0) + v
    if stats is not None:       # the groups iterate concurrently: the batch's count is the max
        stats.newton_iters += max(sg.newton_iters for _, _, sg in out if sg is not None)
    for s_ in streams:
        main.wait_stream(s_)
    return res, sums


def _pair_dist_async(bf, prob, pairs, n, ld, st):
    """Device float32 [len(pairs)]: max over the rows of fit a's mask of |eta_a - eta_b| for
    each (a, b) in pairs (enqueued, not waited for)."""
    dev = bf.eta.device
    upl = getattr(bf, "up", None)
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1)
    pd_ = upl(pairs) if upl is not None else torch.from_numpy(pairs).to(dev)
    fm = getattr(bf, "fit_mask_d", None)
    if fm is None:
        fm = torch.from_numpy(np.asarray(bf.fit_mask, dtype=np.int32)).to(dev)
    out = torch.empty(pairs.size // 2, dtype=torch.float32, device=dev)
    _lib.call("sglm_eta_pair_absmax", n, ld, pairs.size // 2, _p(pd_), _p(prob.M), _p(fm),
              _p(bf.eta), _p(out), st)
    return out


def _resolve_copies(src, formed):
    """Hessian copies of one iteration, each resolved to a Hessian that is actually computed.
    ``src``: fit -> (source fit, distance) -- exact duplicates (distance 0), lambda-chain shares
    and failed alias candidates; a source may itself be a copy (e.g. an exact duplicate of a
    fit that was then shared along its lambda chain).  ``formed``: the fits whose Gram is
    computed.  Returns [(fit, formed source, summed distance)], so every copy reads a
    Hessian written this iteration, whatever order the copies run in."""
    formed = set(int(u) for u in formed)
    out = []
    for k in src:
        r, dk, hops = int(k), 0.0, 0
        while r not in formed:
            if r not in src or hops > len(src):
                raise RuntimeError(f"Hessian copy of fit {k} does not reach a formed Hessian")
            r, dd = src[r]
            dk += dd
            hops += 1
        out.append((int(k), r, dk))
    return out


def _share_chains(uniq, chains, dist, tol):
    """Approximate Hessian dedup along the lambda path.  ``chains``: fits of one (mask,
    response) ordered by penalty (neighbours have the closest solutions); ``dist``: the
    max-row predictor distances of consecutive chain members.  A greedy chain lets each fit
    share the Gram of the chain's representative while the summed distance (a bound on the
    true one, triangle inequality) stays <= tol.  Returns (representatives, [(fit, rep,
    distance bound)])."""
    shared, drop, q = [], set(), 0
    for c in chains:
        rep, acc = c[0], 0.0
        for i in range(1, len(c)):
            acc += dist[q]
            q += 1
            if acc <= tol:
                shared.append((c[i], rep, acc))
                drop.add(c[i])
            else:
                rep, acc = c[i], 0.0
    keep = np.array([k for k in uniq if int(k) not in drop], dtype=np.int32)
    return keep, shared


def _lag_gram(d: Design, bf, fits: np.ndarray, st):
    """H[k] = w_k X^T X for fits at a constant weight over every row (sglm_lag_gram: event
    cross-correlations instead of the MFMA Gram)."""
    lg = d.lag
    work = _work(_lib.query("sglm_lag_gram_work_bytes", lg.m, lg.smin, lg.smax), d.device,
                 "laggram")
    upl = getattr(bf, "up", None)
    fits = np.ascontiguousarray(fits, dtype=np.int32)
    fits_d = upl(fits, np.int32) if upl is not None else torch.from_numpy(fits).to(d.device)
    _lib.call("sglm_lag_gram_pc", _p(lg.occ), _p(lg.ev_off), _p(lg.ebits), lg.nwords,
              _p(lg.shifts), lg.m, lg.K, lg.layout, lg.smin, lg.smax, lg.row0, lg.n, lg.n_raw,
              d.P, d.p, _p(bf.W), d.ld, _p(fits_d), int(fits.size), _p(bf.H), _p(work), st)
    if d.cont is not None:
        _mix_hess(d, bf, fits, False)


def _lag_corr_flop(lg) -> float:
    """Work of one sglm_lag_gram call counted as flop: per occurrence of an event, one bitmap
    test and histogram add per (other event, lag difference d in (-K, K)) -- 2 ops each."""
    if lg is None:
        return 0.0
    nnz = float(lg.occ.numel())
    return 2.0 * nnz * (lg.m + 1) * (2 * lg.K - 1)


def _max_gram_count(bf, slots) -> float:
    """Largest multiplicity sum over the masks of the given slots (an upper bound on every entry
    of their exact 0/1 mask Grams); inf when the problem is unknown."""
    prob = getattr(bf, "prob", None)
    fm = getattr(bf, "fit_mask", None)
    if prob is None or fm is None:
        return float("inf")
    fm = np.asarray(fm)
    return max((prob.mask_count(int(fm[int(h)])) for h in np.asarray(slots).reshape(-1)),
               default=0.0)


class _Factor64:
    """Float64 factors of Grams (sglm_chol64_factor): U [nf][P][P], coordinate states, the
    dependent coordinates and their counts, all on the device."""

    def __init__(self, d: Design, bf, hsrc, dsrc, lamp_d, st):
        P, dev = d.P, d.device
        nf = len(hsrc)
        self.nf = nf
        self.U = torch.empty((nf, P, P), dtype=torch.float64, device=dev)
        self.state = torch.empty((nf, P), dtype=torch.uint8, device=dev)
        self.nulls = torch.empty((nf, P), dtype=torch.int32, device=dev)
        self.counts = torch.zeros((nf, 2), dtype=torch.int32, device=dev)
        upl = getattr(bf, "up", None)
        idx = np.concatenate([np.asarray(hsrc), np.asarray(dsrc)]).astype(np.int32)
        idx_d = upl(idx, np.int32) if upl is not None else torch.from_numpy(idx).to(dev)
        work = _work(_lib.query("sglm_chol64_work_bytes", P, nf), dev, "chol64")
        # the f32 Gram of a 0/1 design holds exact integer counts while every entry (at most the
        # mask's multiplicity sum) stays below 2^24; past that f32 rounding enters the Schur
        # complements and the float32-level threshold applies
        tol = RANK_TOL_EXACT if (d.xbits is not None and _max_gram_count(bf, hsrc) < 2 ** 24) \
            else RANK_TOL_F32
        S = None
        if d.cont is not None:
            store = getattr(bf, "mixS", None) or {}
            missing = [int(h) for h in hsrc if int(h) not in store]
            if missing:
                raise RuntimeError(f"mixed design: no float64 Gram rows for slots {missing}")
            S = torch.stack([store[int(h)] for h in hsrc]).contiguous()
        _lib.call("sglm_chol64_factor_mixed", _p(bf.H), P, _p(idx_d[:nf]), _p(bf.dshift),
                  _p(lamp_d), _p(idx_d[nf:]), nf, tol, _p(S), d.k if S is not None else 0,
                  _p(d._mix["cmap"]) if S is not None else None, _p(self.U), _p(self.state),
                  _p(self.nulls), _p(self.counts), _p(work), st)
        self._S = S                     # alive until the factorisation has run

    def minnorm(self, d: Design, bf, fits, fsrc, beta64_d, st):
        """beta[fits[q]] <- the minimum-norm point of its solution set on factor fsrc[q] (the
        factors 0 .. max(fsrc) take part)."""
        if len(fits) == 0:
            return
        nf = int(np.max(fsrc)) + 1
        upl = getattr(bf, "up", None)
        idx = np.concatenate([np.asarray(fits), np.asarray(fsrc)]).astype(np.int32)
        idx_d = upl(idx, np.int32) if upl is not None else torch.from_numpy(idx).to(d.device)
        nq = len(fits)
        work = _work(_lib.query("sglm_chol64_minnorm_work_bytes", d.P, nf), d.device,
                     "minnorm")
        _lib.call("sglm_chol64_minnorm", _p(self.U), d.P, d.p, _p(self.state), _p(self.nulls),
                  _p(self.counts), nf, _p(idx_d[:nq]), _p(idx_d[nq:]), nq, _p(beta64_d),
                  _p(work), st)


def _syrk(d: Design, bf, fits: np.ndarray, nsteps: int, ntile1: int, stats, st, exact=False,
          rows=None):
    """H[k] = X^T diag(W[k]) X for k in fits.  bf16 MFMA, or the exact-f32 MFMA variant when
    the design is not bf16-exact and the caller needs an accurate Gram (CD, Gaussian)."""
    nact = int(fits.size)
    if nact == 0:
        return
    use_f32 = exact and d.xf is not None
    prob = getattr(bf, "prob", None)
    use_cb = not use_f32 and d.xbits is not None and SYRK_CBITS and prob is not None
    ev = None
    if stats is not None and stats.record:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    lg = _lagw(d) if (use_cb or (exact and d.xf is None and d.xbits is not None)) else None
    if lg is not None and not _lagw_pays(d, lg, nact):
        lg = None
    if lg is not None:
        ab, flop, xflop = _lag_gram_w(d, lg, bf, fits, st, ev)
        if stats is not None:
            stats.alg_flop += flop
        if ev is not None:
            stats.syrk_bytes.append(ab)
            stats.syrk_exec.append(xflop)
            stats.syrk_events.append((ev[0], ev[1], nact, flop))   # the structured products
        if d.cont is not None:
            _mix_hess(d, bf, fits, exact)
        return
    if use_cb:
        ab = _syrk_cbits(d, bf, prob, fits, st, ev)
        if ev is not None:
            stats.syrk_bytes.append(ab)
    else:
        if ev is not None:
            ev[0].record()
        if use_f32:
            nt = d.P // 128
            ntile1 = nt * (nt + 1) // 2
            nsteps = (d.n + 15) // 16
        splits = syrk_splits(ntile1 * nact, nsteps)
        wb = _lib.query("sglm_syrk_work_bytes", d.P, nact, splits)
        work = _work(wb, d.device) if wb else None
        fits_d = torch.tensor(fits, dtype=torch.int32, device=d.device)
        if use_f32:
            _lib.call("sglm_syrk_f32", _p(d.xf), d.ld, d.P, d.n, _p(bf.W), _p(fits_d), nact,
                      splits, _p(bf.H), _p(work), st)
        elif prob is not None and not use_f32:          # non-binary design, masked fits
            goff = torch.from_numpy(prob.group_offset[bf.fit_mask]).to(d.device)
            gcnt = torch.from_numpy(prob.group_count[bf.fit_mask]).to(d.device)
            _lib.call("sglm_syrk_masked", _p(d.xb), d.ld, d.P, d.n, _p(bf.W), _p(fits_d), nact,
                      splits, _p(bf.H), _p(work), _p(prob.groups), _p(goff), _p(gcnt), st)
        else:
            _lib.call("sglm_syrk", _p(d.xb), d.ld, d.P, d.n, _p(bf.W), _p(fits_d), nact,
                      splits, _p(bf.H), _p(work), st)
        if ev is not None:
            ev[1].record()
    if stats is not None:
        pa = d.p + 1
        nrows = float(np.sum(rows[fits])) if rows is not None else float(d.n) * nact
        stats.alg_flop += nrows * pa * (pa + 1)
    if ev is not None:
        stats.syrk_events.append((ev[0], ev[1], nact, nrows * pa * (pa + 1)))  # algorithmic flop
    if d.cont is not None:
        _mix_hess(d, bf, fits, exact)


def _mix_hess(d: Design, bf, fits, exact: bool):
    """The continuous rows / columns of the Hessians H[fits] of a mixed design (float64 Gram
    rows S, scattered into the f32 Hessians; S kept per slot in bf.mixS for the float64 factors
    of the exact Grams).  exact: the fits' weights are their masks' multiplicities."""
    fits = np.asarray(fits, dtype=np.int64).reshape(-1)
    if fits.size == 0:
        return
    upl = getattr(bf, "up", None)
    if exact and getattr(bf, "prob", None) is not None:
        S = d.mix_gram_rows(M=bf.prob.M, mrows=np.asarray(bf.fit_mask)[fits], upl=upl)
    else:
        S = d.mix_gram_rows(W=bf.W, wslots=fits, upl=upl)
    d.mix_to_h(S, fits, bf.H, upl=upl)
    store = getattr(bf, "mixS", None)
    if store is None:
        store = bf.mixS = {}
    for q, k in enumerate(fits):
        store[int(k)] = S[q]


def _lagw(d: Design):
    """The design's event structure for sglm_lag_gram_w (row words and the shift table built
    on first use), or None: no structure, > 63 events, or events too dense for the structured
    product to pay.  A mixed design's continuous rows / columns come from _mix_hess after it."""
    lg = getattr(d, "lag", None)
    if not LAG_GRAM_W or lg is None or lg.m > 63 or (d.cont is not None
                                                      and not LAG_GRAM_W_MIXED):
        return None
    if getattr(lg, "R", None) is None:
        if getattr(lg, "R_off", False):
            return None
        cnt = np.diff(lg.ev_off.cpu().numpy().astype(np.int64))
        rho = float(cnt.sum()) / max(1.0, float(lg.m) * float(lg.n_raw))
        sh = lg.shifts.cpu().numpy().astype(np.int64)
        if (rho > LAG_GRAM_W_MAX_RHO or d.p != lg.m * lg.K + d.k
                or not np.array_equal(np.sort(sh), np.arange(lg.smin, lg.smin + sh.size))):
            lg.R_off = True
            return None
        R = torch.empty(max(1, lg.n_raw), dtype=torch.int64, device=d.device)
        _lib.call("sglm_lag_rowwords", _p(lg.ebits), lg.m, lg.nwords, lg.n_raw, _p(R),
                  _stream())
        bidx = np.full(lg.smax - lg.smin + 1, -1, dtype=np.int32)
        bidx[sh - lg.smin] = np.arange(sh.size, dtype=np.int32)
        lg.bidx = torch.from_numpy(bidx).to(d.device)
        # algorithmic flop per fit, in the kernel's own decomposition (each H entry's terms
        # once): per occurrence of a1, the rows d = s_b1 - s_b2 >= 0 -- at d = 0 the events
        # a2 >= a1 and the ones column, K columns each; at d > 0 every event a2 and the K - d
        # shifts s_b1 whose s_b1 - d is a column.  The launch also forms the G entries whose
        # second shift is no column and pads rows and columns to 32 (_lagw_exec_flop >= this)
        # the occurrences the launch iterates: those whose window of design rows
        # [v - row0 + smin, v - row0 + smax] meets [0, n) -- every occurrence for a whole design,
        # a row slab's own share for one rank of a row-sharded solve (the others only ever meet
        # zero weights)
        lo, hi = lg.row0 - lg.smax, lg.row0 + lg.n - 1 - lg.smin
        lg.w_occ, lg.w_ev_off = lg.occ, lg.ev_off
        if lo > 0 or hi < lg.n_raw - 1:
            keep = (lg.occ >= lo) & (lg.occ <= hi)
            evi = torch.repeat_interleave(
                torch.arange(lg.m, device=lg.occ.device),
                torch.from_numpy(cnt).to(lg.occ.device))
            lg.w_occ = lg.occ[keep].contiguous()
            wc = torch.bincount(evi[keep], minlength=lg.m)
            lg.w_ev_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=lg.occ.device),
                                     torch.cumsum(wc, 0)]).to(torch.int32).contiguous()
            cnt = wc.cpu().numpy().astype(np.int64)
        lg.flop1 = _lagw_alg_flop1(lg.m, lg.K, cnt)
        lg.cnt = cnt
        lg.R = R
    return lg


def _lagw_alg_flop1(m: int, K: int, cnt) -> float:
    """Algorithmic flop of the event-structured Gram per fit, in the kernel's decomposition:
    per occurrence of event a1 the H entries it forms -- at d = s_b1 - s_b2 = 0 the events
    a2 >= a1 and the ones column over all K shifts, at d > 0 every event a2 over the K - d
    shifts s_b1 whose s_b1 - d is a column -- one multiply-add each."""
    return float(2.0 * sum(int(c) * (K * (m - a + 1) + m * K * (K - 1) // 2)
                           for a, c in enumerate(cnt)))


def _lag_gram_w(d: Design, lg, bf, fits: np.ndarray, st, ev=None):
    """H[k] = X^T diag(bf16 W[k]) X for k in fits from the design's events (sglm_lag_gram_w);
    returns (algorithmic bytes, structured flop) of the launch."""
    nact = int(fits.size)
    upl = getattr(bf, "up", None)
    fits_d = upl(fits, np.int32) if upl is not None else \
        torch.from_numpy(np.asarray(fits, dtype=np.int32)).to(d.device)
    # the launch's scratch (8 shifted bf16 copies of the fits' weights over every raw row,
    # ~16 B per raw row per fit, and a P x P image per fit for the split pieces' second halves)
    # stays within LAGW_WORK_BUDGET: fits in chunks of at most that
    per1 = _lib.query("sglm_lag_gram_w_work_bytes", lg.n_raw, lg.K, 1, d.P)
    chunk = max(1, min(nact, int(LAGW_WORK_BUDGET // max(1, per1))))
    work = _work(_lib.query("sglm_lag_gram_w_work_bytes", lg.n_raw, lg.K, chunk, d.P), d.device,
                 "lagw")
    with _GRAM_LOCK:
        _gram_turn()
        if ev is not None:
            ev[0].record()
        for c0 in range(0, nact, chunk):
            nc = min(chunk, nact - c0)
            _lib.call("sglm_lag_gram_w", _p(lg.R), _p(lg.w_occ), _p(lg.w_ev_off), lg.m, lg.n_raw,
                      _p(lg.shifts), _p(lg.bidx), lg.K, lg.smin, lg.smax, lg.layout, lg.row0,
                      lg.n, _p(bf.W), d.ld, _p(fits_d[c0:c0 + nc]), nc, _p(bf.H), d.P, d.p,
                      _p(work), st)
        if ev is not None:
            ev[1].record()
        _gram_done()
    bf.keep = (fits_d,)
    pa = d.p + 1
    return (8 * lg.n_raw + nact * (4 * lg.n + 4 * pa * (pa + 1) // 2), nact * lg.flop1,
            _lagw_exec_flop(lg, nact))


# bytes of sglm_lag_gram_w scratch one launch may use (its fits are split into launches beyond
# that; the buffer is cached per device, so this bounds what a session keeps allocated)
LAGW_WORK_BUDGET = float(os.environ.get("SGLM_LAGW_WORK_BUDGET", str(2 << 30)))


def _lagw_pays(d: Design, lg, nact: int) -> bool:
    """Whether the event-structured Gram beats the dense bit-plane one for this launch: MFMA
    work at the rates each reaches on the C4 grid (0.28 / 0.8 of the dense bf16 peak) plus the
    structured path's weight copies (8 x 2 B per raw row per fit) and launch overheads."""
    nb = d.P // 128
    dense = 2.0 * d.n * (nb * (nb + 1) // 2) * 128 * 128 * nact / (0.8 * 2.5e15)
    lag = (_lagw_exec_flop(lg, nact) / (0.28 * 2.5e15) + 16.0 * lg.n_raw * nact / 3e12
           + 40e-6)
    return lag < dense


def _lagw_exec_flop(lg, nact: int) -> float:
    """MFMA flop the sglm_lag_gram_w launch executes (csrc/lagw.hip's tiling: per event, its
    occurrences in stages of 128; pieces of 8 waves x 2 M tiles -- the (d, 32-event half) rows
    -- by a window of NN (shift, fit) columns starting at the piece's first d row; each wave runs
    the contiguous range of its 32-column tiles that meet a d of its rows with a second shift
    that is a column): the structured products plus the G entries that are no H entry and the
    padding."""
    memo = lg.__dict__.setdefault("exec_flop", {})
    if nact in memo:
        return memo[nact]
    K, MT, WM = lg.K, 2, 8
    NH = 2 if lg.m + 1 > 32 else 1
    NT = 2 if nact * K <= 64 else 4
    NN, MB, Tm = NT * 32, WM * MT, K * NH
    Gm, Gy = -(-Tm // MB), -(-(nact * K) // NN)
    tiles = 0
    for g in range(Gm):
        t0 = g * MB
        di0 = t0 // NH
        for y in range(Gy):
            n0 = y * NN + di0 * nact
            if t0 >= Tm or n0 // nact >= K or min(K - 1, (n0 + NN - 1) // nact) < di0:
                continue
            for wm in range(WM):
                rows = [t for t in range(t0 + wm * MT, t0 + wm * MT + MT) if t < Tm]
                if not rows:
                    continue
                dmin = min(t // NH for t in rows)
                live = [j for j in range(NT) if (n0 + 32 * j) // nact < K
                        and min(K - 1, (n0 + 32 * j + 31) // nact) >= dmin]
                if live:
                    tiles += MT * (max(live) - min(live) + 1)
    occ = float(sum(-(-int(c) // 128) * 128 for c in lg.cnt))
    memo[nact] = 2.0 * occ * tiles * 32 * 32
    return memo[nact]

def _syrk_cbits(d: Design, bf, prob: Problem, fits: np.ndarray, st, ev=None):
    """Gram v6 over per-mask compacted bit-planes.  Slots are ordered by mask so that the
    workgroups resident at any time read the same compacted design (Infinity Cache)."""
    masks = np.asarray(bf.fit_mask)[fits]
    order = np.argsort(masks, kind="stable")
    fits, masks = fits[order], masks[order]
    nact = int(fits.size)
    cbs = [prob.compact(int(m)) for m in masks]
    maxrows = max(c[1] for c in cbs)
    stride = max(64, pad_to(maxrows, 64))
    need = nact * stride
    wc = getattr(bf, "wc", None)
    if wc is None or wc.numel() < need:
        wc = bf.wc = torch.empty(need, dtype=torch.bfloat16, device=d.device)
    desc = np.array([[c[0].data_ptr(), c[1], wc.data_ptr() + 2 * i * stride,
                      0 if c[2] is None else c[2].data_ptr()] for i, c in enumerate(cbs)],
                    dtype=np.int64)
    upl = getattr(bf, "up", None)
    if upl is not None:
        desc_d, fits_d = upl(desc), upl(fits, np.int32)
    else:
        desc_d = torch.from_numpy(desc).to(d.device)
        fits_d = torch.from_numpy(fits.astype(np.int32)).to(d.device)
    nb = d.P // 128
    splits = syrk6_splits(nb * (nb + 1) // 2 * nact, max(1, (maxrows + 63) // 64), nact, d.P)
    if GRAM_LOG is not None:
        GRAM_LOG.append((nact, len(set(masks.tolist())), splits, maxrows))
    wb = _lib.query("sglm_syrk_work_bytes", d.P, nact, splits)
    work = _work(wb, d.device) if wb else None
    _lib.call("sglm_gather_w", _p(bf.W), d.ld, _p(fits_d), nact, _p(desc_d), maxrows, st)
    with _GRAM_LOCK:
        _gram_turn()
        if ev is not None:              # the roofline times the Gram kernel alone
            ev[0].record()
        _lib.call("sglm_syrk_cbits", _p(desc_d), d.P, _p(fits_d), nact, splits, _p(bf.H),
                  _p(work), st)
        if ev is not None:
            ev[1].record()
        _gram_done()
    bf.keep = (desc_d, fits_d)          # alive until the next launch is enqueued
    # algorithmic bytes of the launch: each distinct compacted design once (rows/64 K-steps x P
    # predictors x 8 B), each slot's bf16 weights, each slot's upper 128-block triangle (f32)
    planes = {int(c[0].data_ptr()): int(c[1]) for c in cbs}
    return (sum((r + 63) // 64 * d.P * 8 for r in planes.values())
            + sum(2 * int(c[1]) for c in cbs) + nact * nb * (nb + 1) // 2 * 128 * 128 * 4)


def score_sums(prob: Problem, family: int, power: float, eta, fit_resp: Sequence[int],
               sets: np.ndarray, comm=None) -> np.ndarray:
    """[B, 2, 2] float64: per fit and set (train, test): sum m (y - mu)^2, sum m loss
    (summed over the ranks' slabs of a row-sharded solve when ``comm`` is given)."""
    d = prob.design
    B = len(fit_resp)
    dev = d.device
    fr = torch.tensor(list(fit_resp), dtype=torch.int32, device=dev)
    sd = torch.tensor(np.asarray(sets, dtype=np.int32).reshape(-1), dtype=torch.int32, device=dev)
    out = torch.zeros((B, 4), dtype=torch.float64, device=dev)
    work = _work(_lib.query("sglm_rowsum_work_bytes", B, 4, d.n), dev)
    _lib.call("sglm_score_sums", family, float(power), d.n, d.ld, B, _p(eta), _p(prob.Y),
              _p(prob.M), _p(fr), _p(sd), _p(out), _p(work), _stream())
    if comm is not None:
        comm.sum_(out)
    return out.cpu().numpy().reshape(B, 2, 2)
