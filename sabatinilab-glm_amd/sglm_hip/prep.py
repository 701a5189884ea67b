"""Host entry to the session-preprocessing kernels (sglm_prep_session, csrc/prep.hip).

``session_columns(X, k)`` takes the (9 x n) float64 block of renamed session columns
(``IN_COLS`` order = enum sglm_prep_in) and returns the (40 x n) float64 block of derived
columns (``OUT_COLS`` order = enum sglm_prep_out) of lynne_pp.preprocess_lynne
(lynne_pp.py:217-249).  ``session_columns_device`` is the same on device tensors (no host
copies; bench.py times it).  No CPU fallback: without the library or a GPU it raises.
"""
from __future__ import annotations

import numpy as np

from . import _lib

IN_COLS = ("cpn", "lpx", "rpx", "lpn", "rpn", "r", "nr", "rl", "ll")
OUT_COLS = (
    "event_col", "trial_start_flag", "nTrial", "event_col_end", "trial_end_flag", "nEndTrial",
    "r_trial", "nr_trial",
    "rpxr", "rpxnr", "lpxr", "lpxnr", "rpnr", "rpnnr", "lpnr", "lpnnr",
    "spn", "spx", "spnr", "spnnr", "spxr", "spxnr", "sl",
    "nn", "xx",
    "ft_nn", "ft_xx", "ft_lpn", "ft_rpn", "ft_spn", "ft_lpx", "ft_rpx", "ft_spx", "ft_cpn",
    "ft_r_rpn", "ft_r_lpn", "ft_r_spn", "ft_nr_rpn", "ft_nr_lpn", "ft_nr_spn",
)


class Workspace:
    """Reusable device scratch for sessions of up to ``n`` rows."""

    def __init__(self, n: int):
        import torch
        self.n = int(n)
        nbytes = int(_lib.query("sglm_prep_work_bytes", self.n))
        self.buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")


def session_columns_device(X, k: int, out=None, work: Workspace = None):
    """X: (9, n) float64 CUDA tensor (row c = input column c); returns (40, n) float64."""
    import torch
    if X.dim() != 2 or X.shape[0] != len(IN_COLS) or X.dtype != torch.float64 or not X.is_cuda:
        raise ValueError(f"expected a (9, n) float64 CUDA tensor, got {tuple(X.shape)} "
                         f"{X.dtype} on {X.device}")
    if X.stride(1) != 1:
        X = X.contiguous()
    n = X.shape[1]
    if out is None:
        out = torch.empty((len(OUT_COLS), n), dtype=torch.float64, device=X.device)
    if out.shape != (len(OUT_COLS), n) or out.stride(1) != 1:
        raise ValueError("out must be a row-contiguous (40, n) float64 tensor")
    if n == 0:
        return out
    if work is None or work.n < n:
        work = Workspace(n)
    _lib.call("sglm_prep_session", X.data_ptr(), X.stride(0), n, int(k), out.data_ptr(),
              out.stride(0), work.buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    return out


def session_columns(X: np.ndarray, k: int) -> np.ndarray:
    """Host arrays in and out: (9, n) float64 -> (40, n) float64."""
    import torch
    from .engine import require_gpu
    require_gpu()
    X = np.ascontiguousarray(X, dtype=np.float64)
    if X.ndim != 2 or X.shape[0] != len(IN_COLS):
        raise ValueError(f"expected a (9, n) array, got {X.shape}")
    out = session_columns_device(torch.from_numpy(X).cuda(), k)
    return out.cpu().numpy()
