"""Host entry to the HIP lag-expansion kernel (sglm_timeshift_expand).

``shift_columns(A, cols, shifts, fill)`` returns the (n x len(cols)) array whose column j
is column ``cols[j]`` of A moved down by ``shifts[j]`` rows (up when negative) with
``fill`` in the vacated rows — the arithmetic of backend/sglm_pp.py:298-357 for every
requested (column, shift) pair in ONE kernel launch (the reference starts one Python
thread and one np.concatenate per shift, sglm_pp.py:83-98).
"""
from __future__ import annotations

import numpy as np

from . import _lib

_UINT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}
_SINT = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}     # torch-friendly views


def fill_bits(fill, dtype) -> int:
    v = np.array(fill).astype(dtype)
    return int(v.reshape(1).view(_UINT[v.itemsize])[0])


def shift_columns(A: np.ndarray, cols, shifts, fill=np.nan, out_dtype=None) -> np.ndarray:
    import torch
    from .engine import require_gpu
    require_gpu()
    A = np.asarray(A)
    if A.ndim != 2:
        raise ValueError("expected a 2-D array")
    out_dtype = np.dtype(out_dtype or A.dtype)
    if out_dtype.itemsize not in _UINT or out_dtype.kind not in "fiub":
        raise TypeError(f"unsupported dtype {out_dtype}")
    n, m = A.shape
    cols = np.asarray(cols, dtype=np.int32).reshape(-1)
    shifts = np.asarray(shifts, dtype=np.int32).reshape(-1)
    k = cols.size
    if k == 0 or n == 0:
        return np.empty((n, k), dtype=out_dtype)
    if cols.min() < 0 or cols.max() >= m:
        raise IndexError("column index out of range")
    src = torch.from_numpy(np.ascontiguousarray(A.astype(out_dtype, copy=False)).view(
        _SINT[out_dtype.itemsize])).cuda()
    out = torch.empty((n, k), dtype=src.dtype, device="cuda")
    c = torch.from_numpy(cols).cuda()
    s = torch.from_numpy(shifts).cuda()
    _lib.call("sglm_timeshift_expand", src.data_ptr(), n, m, 1, c.data_ptr(), s.data_ptr(), k,
              out.data_ptr(), n, k, 1, 0, out_dtype.itemsize, fill_bits(fill, out_dtype),
              torch.cuda.current_stream().cuda_stream)
    return out.cpu().numpy().view(out_dtype)
