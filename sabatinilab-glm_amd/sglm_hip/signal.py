"""Host entry to the signal/trial-table kernels (sglm_scatter_rows, sglm_signal_trials;
csrc/prep.hip) behind ``sglm.features.gen_signal_df.generate_signal_df``
(sglm/sglm/features/gen_signal_df.py:327-470).

``aligned_columns(n, rows, vals)``: trial-table values aligned onto the n signal rows by
index label (NaN where a row is not listed) -- the reference's
``signal_df[col] = df_t_tmp.set_index(col)[...]``, one column per row of ``vals``.
``trial_runs(center_in, side_out, k_before, k_after)``: nTrial, nEndTrial, diffTrialNums and
the row map of the per-trial duplication loop (:430-458).  The ``*_device`` forms take and
return device tensors (the bench times those).  No CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.HipEngineUnavailable("no ROCm GPU visible: the signal kernels have no CPU "
                                        "fallback")
    _lib.load()
    return torch


def aligned_columns_device(n: int, rows_d, vals_d, out_d) -> None:
    """out_d (nc, >= n) float64 on the device: NaN, then out[c][rows[t]] = vals[c][t]."""
    torch = _torch()
    nr = 0 if rows_d is None else int(rows_d.numel())
    nc = int(out_d.shape[0])
    if nr and (rows_d.dtype != torch.int64 or vals_d.dtype != torch.float64
               or tuple(vals_d.shape) != (nc, nr) or not vals_d.is_contiguous()
               or not rows_d.is_contiguous()):
        raise ValueError("rows_d int64 (nr,), vals_d float64 contiguous (nc, nr)")
    if out_d.dtype != torch.float64 or out_d.stride(1) != 1 or out_d.shape[1] < n:
        raise ValueError("out_d float64 (nc, >= n) with unit column stride")
    _lib.call("sglm_scatter_rows", int(n), rows_d.data_ptr() if nr else None, nr,
              vals_d.data_ptr() if nr else None, nc, out_d.data_ptr(), out_d.stride(0),
              torch.cuda.current_stream().cuda_stream)


def aligned_columns(n: int, rows: np.ndarray, vals: np.ndarray) -> np.ndarray:
    """(ncols, n) float64: NaN, then out[c][rows[t]] = vals[c][t] (rows distinct)."""
    torch = _torch()
    rows = np.ascontiguousarray(rows, dtype=np.int64).reshape(-1)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    if vals.ndim == 1:
        vals = vals[None]
    if vals.ndim != 2 or vals.shape[1] != rows.size:
        raise ValueError("vals must be (ncols, len(rows))")
    nc = vals.shape[0]
    out = torch.empty((nc, max(int(n), 1)), dtype=torch.float64, device="cuda")
    if n == 0 or nc == 0:
        return out.cpu().numpy()[:, :n]
    rd = torch.from_numpy(rows).cuda() if rows.size else None
    vd = torch.from_numpy(vals).cuda() if rows.size else None
    aligned_columns_device(int(n), rd, vd, out)
    return out.cpu().numpy()


class TrialWorkspace:
    """Device buffers of ``trial_runs_device`` for sessions of up to ``n`` rows."""

    def __init__(self, n: int):
        torch = _torch()
        n = max(int(n), 1)
        self.n = n
        self.cols = torch.empty((3, n), dtype=torch.float64, device="cuda")
        self.src = torch.empty(2 * n, dtype=torch.int64, device="cuda")
        self.dup = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
        self.ncopies = torch.zeros(1, dtype=torch.float64, device="cuda")
        self.work = torch.empty(int(_lib.query("sglm_signal_trials_work_bytes", n)),
                                dtype=torch.uint8, device="cuda")


def trial_runs_device(ci_d, so_d, k_before: int, k_after: int, ws: TrialWorkspace) -> None:
    """Fills ws.cols (nTrial, nEndTrial, diffTrialNums), ws.src / ws.dup (output row map, the
    first ``n_out(n, k_before, ws.ncopies)`` entries) and ws.ncopies, asynchronously."""
    torch = _torch()
    n = int(ci_d.numel())
    if so_d.numel() != n:
        raise ValueError("center_in and side_out must have the same length")
    if n > ws.n:
        raise ValueError(f"workspace holds {ws.n} rows, session has {n}")
    for t in (ci_d, so_d):
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("center_in / side_out must be contiguous float64")
    if n == 0:
        return
    _lib.call("sglm_signal_trials", ci_d.data_ptr(), so_d.data_ptr(), n, int(k_before),
              int(k_after), ws.cols[0].data_ptr(), ws.cols[1].data_ptr(),
              ws.cols[2].data_ptr(), ws.src.data_ptr(), ws.dup.data_ptr(),
              ws.ncopies.data_ptr(), ws.work.data_ptr(),
              torch.cuda.current_stream().cuda_stream)


def n_out(n: int, k_before: int, ncopies: int) -> int:
    """Output rows: the rows whose nTrial is not NaN (all but |k_before|) plus the copies."""
    return n - min(abs(int(k_before)), n) + int(ncopies)


def trial_runs(center_in: np.ndarray, side_out: np.ndarray, k_before: int, k_after: int):
    """Returns (ntrial, nend, diff) float64 (n,) and (src int64, dup bool) of the output rows."""
    torch = _torch()
    ci = torch.from_numpy(np.ascontiguousarray(center_in, dtype=np.float64)).cuda()
    so = torch.from_numpy(np.ascontiguousarray(side_out, dtype=np.float64)).cuda()
    n = int(ci.numel())
    if so.numel() != n:
        raise ValueError("center_in and side_out must have the same length")
    if n == 0:
        e = np.zeros(0)
        return e, e, e, np.zeros(0, np.int64), np.zeros(0, bool)
    ws = TrialWorkspace(n)
    trial_runs_device(ci, so, k_before, k_after, ws)
    m = n_out(n, k_before, int(ws.ncopies.item()))
    c = ws.cols[:, :n].cpu().numpy()
    return (c[0], c[1], c[2], ws.src[:m].cpu().numpy(),
            ws.dup[:m].cpu().numpy().astype(bool))
