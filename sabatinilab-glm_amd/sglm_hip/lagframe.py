"""Lagged DataFrames whose lag columns stay on the device (the production flow, resident).

The reference's production driver (er_refactored_from_scratch_cleanup.py:421-452) runs

    dfrel, X_cols_sftd = timeshift_vals(dfrel, X_cols, neg, pos)     # sglm_ez.timeshift_cols
    dfrel = dfrel[(dfrel[cols + X_cols_sftd + [y]].isna().sum(axis=1) == 0) & ...]
    dfrel_setup, dfrel_holdout = holdout_splits(dfrel, ...)          # .loc[bool mask]
    kfold_cv_idx = sglm_ez.cv_idx_by_trial_id(dfrel_setup, ['nTrial'], ...)
    X_setup, y_setup = dfrel_setup[X_cols_sftd], dfrel_setup[y_col]
    sglm_ez.simple_cv_fit(X_setup, y_setup, kfold_cv_idx, ...)        # X.values -> sklearn

where ``timeshift_multiple`` (backend/sglm_pp.py:58-103) materialises N x (m K) float64 values
(16 GB at 1M x 2000) only for the NaN filter to read them and the fit to copy them again.

``LagFrame`` is that frame without the materialisation: the source columns live on the device
(float64, column-major), every lag column is the spec (source column, shift), and row
selections are position lists.  The operations of the flow above are answered from the specs:
column / row selections are bookkeeping, ``isna().sum(axis=1)`` counts the out-of-range and
NaN source cells of each row on the device, id columns are host Series, and ``simple_cv_fit`` /
``GLM.fit`` / ``predict`` build their design straight from the device sources
(``engine.Design.from_lagged``: the event-correlation Gram and gradient when the rows are
contiguous and the columns are the canonical lag layout).  Anything else -- ``.values``,
printing, arithmetic, any other pandas method -- materialises exactly the values the reference
would have held (``to_pandas()``), so the frame behaves as the reference's DataFrame.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import pandas as pd

from . import _lib

NAN = float("nan")


class _Snapshot:
    """The columns, index and row count of a DataFrame as they were when a lagged frame was
    made from it (the reference's timeshift_multiple returns a copy, sglm_pp.py:436-486).  Each
    column's Series is taken at construction -- a view, no copy -- so a later column assignment
    (``X['A'] = ...``), column insertion / deletion or row-dropping change of the caller's frame
    (``X.dropna(inplace=True)``) leaves these arrays, and their length, as they were; only
    element writes into the same array (``X.loc[r, 'A'] = v``) would show through."""

    def __init__(self, X: pd.DataFrame):
        self.index = X.index
        self.columns = X.columns
        self._cols = {c: X[c] for c in X.columns}
        self._n = len(X)

    def __getitem__(self, name):
        return self._cols[name]

    def __len__(self):
        return self._n


class LagSource:
    """The frame a lagged frame was made from (a _Snapshot of its columns) and the device
    float64 copies of the columns the lag columns read (uploaded once, on first use)."""

    def __init__(self, base: pd.DataFrame):
        self.base = _Snapshot(base)
        self.N = len(base)
        self._dev = {}           # column name -> row of self._E
        self._E = None
        self._bits = {}          # 0/1 column name -> its device bit row (int32 [ceil(N / 32)])
        self._hasnan = {}        # column name -> holds a NaN cell
        self._ones = {}          # 0/1 column name -> its count of 1 cells (host pack)
        self._numeric = {}       # column name -> numeric dtype
        self.cast = {}           # base column name -> dtype of its shift-0 copy in the frame
        self.all_rows = None     # arange(N), built once

    def upload(self, names):
        """Upload the named base columns once: a 0/1 column as its device bit row (crossing
        PCIe as 1 bit per row, sglm_host_pack_bits_cols; kept packed -- the lag design's bit
        planes and event occurrences are built from it), any other column as a float64 row of
        the device source block (NaN kept)."""
        import ctypes
        import torch
        from .engine import HOST_THREADS, _pinned, _scratch, require_gpu
        require_gpu()
        need = [c for c in dict.fromkeys(names) if c not in self._dev and c not in self._bits]
        if not need:
            return
        N, m = self.N, len(need)
        arrs = [self._f64(c) for c in need]
        # address order: the columns of one row-major block then arrive as the packer's block
        # (each row's run of values read once) whatever order the names came in
        order = sorted(range(m), key=lambda i: (arrs[i].strides[0], arrs[i].ctypes.data))
        need = [need[i] for i in order]
        arrs = [arrs[i] for i in order]
        nw = (N + 31) // 32
        bits = _pinned("lagbits", max(1, m * nw), torch.int32)
        evk = ("lagbits_ev", None)
        if _scratch().pinned.get(evk) is not None:
            _scratch().pinned[evk].synchronize()      # the last upload has read the stage
        binary = np.zeros(m, dtype=np.uint8)
        ones = np.zeros(m, dtype=np.int64)
        ptrs = (ctypes.c_void_p * m)(*[a.ctypes.data for a in arrs])
        strides = np.array([a.strides[0] // 8 for a in arrs], dtype=np.int64)
        _lib.call("sglm_host_pack_bits_cols", ctypes.cast(ptrs, ctypes.c_void_p),
                  strides.ctypes.data, m, N, bits.data_ptr(), binary.ctypes.data,
                  ones.ctypes.data, HOST_THREADS)
        bsel = np.flatnonzero(binary)
        if bsel.size:
            # the 0/1 columns' bit rows, one asynchronous copy out of the pinned stage
            bd = bits[: m * nw].view(m, nw)
            bd = (bd if bsel.size == m else bd[torch.from_numpy(bsel)]).to("cuda",
                                                                           non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            _scratch().pinned[evk] = ev
            for q, i in enumerate(bsel):
                self._bits[need[i]] = bd[q]
                self._ones[need[i]] = int(ones[i])
                self._hasnan[need[i]] = False
        raw = np.flatnonzero(binary == 0)
        if not raw.size:
            return
        need_raw = [need[i] for i in raw]
        arr_raw = [arrs[i] for i in raw]
        new = torch.empty((len(need_raw), N), dtype=torch.float64, device="cuda")
        # column groups of <= 64 MB through two pinned stages: the threaded host gather of
        # group g + 1 overlaps the DMA of group g
        per = max(1, (64 << 20) // max(1, 8 * N))
        stages = [_pinned(f"lagsrc{i}", max(1, per * N), torch.float64) for i in range(2)]
        evs = [None, None]
        for g, c0 in enumerate(range(0, len(need_raw), per)):
            grp = arr_raw[c0:c0 + per]
            b = g % 2
            if evs[b] is not None:
                evs[b].synchronize()
            ptrs = (ctypes.c_void_p * len(grp))(*[a.ctypes.data for a in grp])
            strides = np.array([a.strides[0] // 8 for a in grp], dtype=np.int64)
            _lib.call("sglm_host_gather_cols", ctypes.cast(ptrs, ctypes.c_void_p),
                      strides.ctypes.data, len(grp), N, 8, stages[b].data_ptr(), HOST_THREADS)
            new[c0:c0 + len(grp)] = stages[b][: len(grp) * N].view(len(grp), N).to(
                "cuda", non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            evs[b] = ev
        for ev in evs:
            if ev is not None:
                ev.synchronize()
        self._append_rows(need_raw, new)
        has = torch.isnan(new).any(1).cpu().numpy()
        for i, c in enumerate(need_raw):
            self._hasnan[c] = bool(has[i])

    def _append_rows(self, names, new):
        import torch
        base = 0 if self._E is None else self._E.shape[0]
        self._E = new if self._E is None else torch.cat([self._E, new])
        for i, c in enumerate(names):
            self._dev[c] = base + i

    def bits(self, names):
        """Device int32 [len(names)][ceil(N / 32)] bit rows of the named columns when every one
        of them is 0/1 (bit r & 31 of word r >> 5 = row r), else None."""
        import torch
        self.upload(names)
        if not all(c in self._bits for c in names):
            return None
        return torch.stack([self._bits[c] for c in names])

    def device(self, names):
        """Device float64 [rows][N] holding the named base columns (uploaded once, NaN kept;
        0/1 columns unpacked from their bit rows on first use here), and the device int64 row
        index of each name."""
        import torch
        self.upload(names)
        lazy = [c for c in dict.fromkeys(names) if c not in self._dev]
        if lazy:
            B = torch.stack([self._bits[c] for c in lazy])
            sh = torch.arange(32, dtype=torch.int32, device="cuda")
            unp = ((B.unsqueeze(-1) >> sh) & 1).reshape(len(lazy), -1)[:, :self.N]
            self._append_rows(lazy, unp.to(torch.float64))
        rows = [self._dev[c] for c in names]
        if rows and rows == list(range(rows[0], rows[0] + len(rows))):
            # consecutive rows (names in upload order): no host->device copy to wait on
            idx = torch.arange(rows[0], rows[0] + len(rows), dtype=torch.int64, device="cuda")
        else:
            idx = torch.tensor(rows, dtype=torch.int64, device="cuda")
        return self._E, idx

    def _f64(self, name) -> np.ndarray:
        """Host float64 values of a base column: a (possibly strided) view when it already is
        float64 -- the columns of a row-major block are gathered by sglm_host_gather_cols."""
        col = self.base[name]
        if isinstance(col.dtype, np.dtype):
            v = col.to_numpy()
            if not (v.dtype == np.float64 and v.ndim == 1 and v.strides[0] % 8 == 0
                    and v.strides[0] > 0):
                v = np.ascontiguousarray(v.astype(np.float64))
        else:
            v = np.ascontiguousarray(col.to_numpy(dtype=np.float64, na_value=NAN))
        # the native packers read N elements from this pointer
        if v.ndim != 1 or v.shape[0] != self.N:
            raise ValueError(f"lagged frame source column {name!r} has {v.shape} values, "
                             f"expected {self.N}")
        return v

    def numeric(self, name) -> bool:
        if name not in self._numeric:
            dt = self.base[name].dtype
            self._numeric[name] = (isinstance(dt, np.dtype) and dt.kind in "biuf") or \
                pd.api.types.is_numeric_dtype(dt)
        return self._numeric[name]

    def ones(self, name):
        """Count of 1 cells of an uploaded 0/1 column (None for any other column)."""
        return self._ones.get(name)

    def has_nan(self, name) -> bool:
        """Whether an uploaded column holds a NaN cell."""
        return self._hasnan[name]


def _lazy(fn):
    """A LagFrame method answered from the specs while the frame is lazy, and by pandas'
    DataFrame implementation once it has been materialised."""
    name = fn.__name__

    def wrap(self, *a, **k):
        if self._mat is not None:
            return getattr(super(LagFrame, self), name)(*a, **k)
        return fn(self, *a, **k)
    wrap.__name__, wrap.__doc__, wrap.__qualname__ = name, fn.__doc__, fn.__qualname__
    return wrap


class LagFrame(pd.DataFrame):
    """A pandas DataFrame whose values stay on the device until something needs them:
    columns ``cols`` (names), each either a base column of ``src.base`` (``spec[c] = (name, 0,
    False)``), a lag column (``spec[c] = (source name, shift, True)``: value at frame row r =
    base[name] at row r - shift, NaN outside), or a column assigned to this frame (``overlay``);
    rows = positions into the base (None = all).

    It IS a ``pd.DataFrame`` (``isinstance`` holds, as for the frame the reference's
    timeshift_multiple returns, backend/sglm_pp.py:485): the operations of the production flows
    (column / row selections, boolean ``.loc``, ``dropna``, ``isna().sum(axis=1)``, assignments,
    ``drop``, ``copy``, the fits) are answered lazily from the specs; anything else -- pandas
    methods, ``pd.concat``, ``to_parquet``, arithmetic -- reads the frame's block manager, which
    is then built once from the materialised values (``to_pandas()``), and from there on the
    object behaves exactly as that DataFrame (every lazy method defers to pandas)."""

    def __init__(self, src: LagSource, cols, spec, rows: Optional[np.ndarray] = None,
                 index: Optional[pd.Index] = None, overlay: Optional[dict] = None,
                 inc: bool = False):
        # the attributes pandas' NDFrame.__init__ sets -- without a manager: it is built from
        # the materialised values on first use (_mgr below)
        object.__setattr__(self, "_is_copy", None)
        object.__setattr__(self, "_item_cache", {})
        object.__setattr__(self, "_attrs", {})
        object.__setattr__(self, "_flags", pd.Flags(self, allows_duplicate_labels=True))
        object.__setattr__(self, "_mat", None)
        self._src = src
        self._cols = list(cols)
        self._spec = spec
        self._rows = rows
        self._inc = rows is None or inc     # rows known to be strictly increasing
        self._index = index
        self._overlay = overlay if overlay is not None else {}
        self._design = None

    # ------------------------------------------------------------------ pandas plumbing
    @property
    def _mgr(self):
        """pandas' block manager: built from the materialised values the first time pandas
        code touches it (the frame is a plain DataFrame from then on)."""
        if self._mat is None:
            object.__setattr__(self, "_mat", self.to_pandas()._mgr)
        return self._mat

    @_mgr.setter
    def _mgr(self, value):
        object.__setattr__(self, "_mat", value)

    @property
    def _constructor(self):
        return pd.DataFrame

    def __setattr__(self, name, value):
        if name.startswith("_"):
            object.__setattr__(self, name, value)
        else:
            self._mgr                                     # materialise, then as pandas does
            super().__setattr__(name, value)

    def __reduce__(self):
        return (pd.DataFrame, (self.to_pandas() if self._mat is None else
                               pd.DataFrame(self._mat),))

    @property
    def is_lazy(self) -> bool:
        """True while the values live on the device only (no block manager built yet)."""
        return self._mat is None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_shifts(cls, X: pd.DataFrame, shift_inx, shift_amt_list, unshifted_keep_all=True):
        """The frame ``sglm_pp.timeshift_multiple(X, shift_inx, shift_amt_list)`` returns
        (backend/sglm_pp.py:58-103, 436-486): per shift s in order, s == 0 -> every column
        (``unshifted_keep_all``) or the shifted ones, else the shifted columns renamed
        ``f"{col}_{s}"``.  None when the names would not be unique (materialise instead)."""
        inx = list(range(X.shape[1])) if len(shift_inx) == 0 else list(shift_inx)
        names = [X.columns[i] for i in inx]
        cols, spec = [], {}
        for s in shift_amt_list:
            if s == 0:
                keep = list(X.columns) if unshifted_keep_all else names
                for c in keep:
                    cols.append(c)
                    spec[c] = (c, 0, False)
            else:
                for c in names:
                    nm = f"{c}_{s}"
                    cols.append(nm)
                    spec[nm] = (c, int(s), True)
        if len(set(cols)) != len(cols) or not X.columns.is_unique:
            return None
        src = LagSource(X)
        if 0 in list(shift_amt_list):
            # the shift-0 block writes np.asarray(X)[:, inx] back into the selected columns
            # (sglm_pp.shifted_cols_to_pandas): they take the frame's common value dtype
            common = np.asarray(X.iloc[:0]).dtype
            for c in names:
                if X[c].dtype != common:
                    src.cast[c] = common
        return cls(src, cols, spec)

    # ------------------------------------------------------------------ shape / labels
    @property
    def columns(self):
        if self._mat is not None:
            return pd.DataFrame.columns.__get__(self, type(self))
        return pd.Index(self._cols)

    @columns.setter
    def columns(self, value):
        self._mgr
        pd.DataFrame.columns.__set__(self, value)

    @property
    def index(self):
        if self._mat is not None:
            return pd.DataFrame.index.__get__(self, type(self))
        if self._index is None:
            b = self._src.base.index
            sp = self._span()
            self._index = b if self._rows is None else (b[sp[0]:sp[1]] if sp else b[self._rows])
        return self._index

    @index.setter
    def index(self, value):
        self._mgr
        pd.DataFrame.index.__set__(self, value)

    @property
    def shape(self):
        if self._mat is not None:
            return super().shape
        return (self._nrows(), len(self._cols))

    def _nrows(self):
        return self._src.N if self._rows is None else int(self._rows.size)

    def __len__(self):
        if self._mat is not None:
            return super().__len__()
        return self._nrows()

    @property
    def ndim(self):
        return 2

    @property
    def size(self):
        k, m = self.shape
        return k * m

    @property
    def empty(self):
        return self.size == 0

    @property
    def dtypes(self):
        if self._mat is not None:
            return super().dtypes
        b = self._src.base
        return pd.Series([self._overlay[c].dtype if c in self._overlay else
                          (np.dtype(np.float64) if self._spec[c][2] else
                           self._src.cast.get(c, b[self._spec[c][0]].dtype))
                          for c in self._cols], index=self.columns, dtype=object)

    @_lazy
    def keys(self):
        return self.columns

    @_lazy
    def __iter__(self):
        return iter(self._cols)

    @_lazy
    def __contains__(self, c):
        return c in self._spec or c in self._overlay

    def _span(self):
        """(a, b) when this frame's rows are the base rows a .. b - 1 in order, else None --
        O(1): the rows of boolean-mask / dropna selections are known to be increasing, and an
        increasing list spanning b - a rows is the range (the NaN-row filter's result)."""
        if self._rows is None:
            return (0, self._src.N)
        r = self._rows
        if not self._inc or r.size == 0:
            return None
        a, b = int(r[0]), int(r[-1]) + 1
        return (a, b) if b - a == r.size else None

    def positions(self):
        """Row positions into the base frame (int64)."""
        if self._rows is not None:
            return self._rows
        if self._src.all_rows is None:
            self._src.all_rows = np.arange(self._src.N, dtype=np.int64)
        return self._src.all_rows

    # ------------------------------------------------------------------ derived frames
    def _derive(self, cols=None, rows=None, index=None, keep_rows=True, inc=False):
        ov = self._overlay
        if rows is not None:
            ov = {k: v[rows] for k, v in ov.items()}
            base_rows = rows if self._rows is None else self._rows[rows]
            inc = inc and self._inc
        else:
            base_rows = self._rows
            inc = self._inc
        cols = self._cols if cols is None else list(cols)
        ov = {k: v for k, v in ov.items() if k in cols}
        return LagFrame(self._src, cols, self._spec, base_rows,
                        index if index is not None else (self._index if rows is None else None),
                        dict(ov), inc=inc)

    def _take(self, pos, inc=False):
        return self._derive(rows=np.asarray(pos, dtype=np.int64), inc=inc)

    def _bool_rows(self, mask):
        if isinstance(mask, pd.Series):
            if not mask.index.equals(self.index):
                mask = mask.reindex(self.index)
            mask = mask.to_numpy(dtype=bool, na_value=False)
        mask = np.asarray(mask, dtype=bool).reshape(-1)
        if mask.size != self._nrows():
            raise ValueError(f"Item wrong length {mask.size} instead of {self._nrows()}.")
        return self._take(np.flatnonzero(mask), inc=True)

    def _check_cols(self, cols):
        missing = [c for c in cols if c not in self._spec and c not in self._overlay]
        if missing:
            raise KeyError(f"{missing} not in index")

    @_lazy
    def __getitem__(self, key):
        if isinstance(key, str) or (np.isscalar(key) and not isinstance(key, (bool, np.bool_))):
            return self._col_series(key)
        if isinstance(key, slice):
            return self._take(np.arange(self._nrows())[key])
        if isinstance(key, LagFrame):
            raise TypeError("boolean frames as keys are not supported on a lagged frame")
        arr = key if isinstance(key, (pd.Series, pd.Index, np.ndarray)) else np.asarray(key)
        if getattr(arr, "dtype", None) is not None and pd.api.types.is_bool_dtype(arr.dtype):
            return self._bool_rows(key)
        cols = list(key)
        self._check_cols(cols)
        if all(c not in self._overlay and not self._spec[c][2] for c in cols):
            return self._base_frame(cols)               # id / response columns: a real frame
        return self._derive(cols=cols)

    @_lazy
    def __setitem__(self, name, value):
        if isinstance(name, (list, pd.Index, np.ndarray)):
            # frame[[a, b]] = other[[a, b]] (sglm_cb_concat_make_design_mat.py:275): column by
            # column, a DataFrame's columns by position, aligned on the index
            names = list(name)
            if isinstance(value, pd.DataFrame):
                if value.shape[1] != len(names):
                    raise ValueError("Columns must be same length as key")
                for nm, c in zip(names, range(value.shape[1])):
                    self[nm] = value.iloc[:, c]
            elif np.ndim(value) == 2:
                value = np.asarray(value)
                if value.shape[1] != len(names):
                    raise ValueError("Columns must be same length as key")
                for j, nm in enumerate(names):
                    self[nm] = value[:, j]
            else:
                for nm in names:
                    self[nm] = value
            return
        n = self._nrows()
        if isinstance(value, pd.Series):
            value = value.reindex(self.index).to_numpy()
        elif np.isscalar(value):
            value = np.full(n, value)
        value = np.asarray(value)
        if value.shape[0] != n:
            raise ValueError(f"Length of values ({value.shape[0]}) does not match length of "
                             f"index ({n})")
        self._overlay[name] = value
        if name not in self._cols:
            self._cols.append(name)
        self._design = None

    @property
    def loc(self):
        return super().loc if self._mat is not None else _Loc(self)

    @property
    def iloc(self):
        return super().iloc if self._mat is not None else _ILoc(self)

    @_lazy
    def copy(self, deep=True):
        return LagFrame(self._src, self._cols, self._spec, self._rows, self._index,
                        {k: v.copy() for k, v in self._overlay.items()}, inc=self._inc)

    @_lazy
    def reset_index(self, drop=False, **kw):
        if drop and not kw:
            return LagFrame(self._src, self._cols, self._spec, self._rows,
                            pd.RangeIndex(self._nrows()), dict(self._overlay), inc=self._inc)
        return getattr(self.to_pandas(), "reset_index")(drop=drop, **kw)

    @_lazy
    def drop(self, labels=None, axis=0, columns=None, **kw):
        if columns is None and axis in (1, "columns"):
            columns, labels = labels, None
        if columns is not None and labels is None and not kw:
            drop = [columns] if isinstance(columns, str) else list(columns)
            self._check_cols(drop)
            return self._derive(cols=[c for c in self._cols if c not in set(drop)])
        return self.to_pandas().drop(labels=labels, axis=axis, columns=columns, **kw)

    # ------------------------------------------------------------------ missing values
    @_lazy
    def isna(self):
        return _LagNA(self)

    isnull = isna

    @_lazy
    def notna(self):
        return _LagNA(self, negate=True)

    notnull = notna

    @_lazy
    def dropna(self, axis=0, how="any", subset=None, inplace=False, **kw):
        if axis not in (0, "index") or inplace or kw:
            return self.to_pandas().dropna(axis=axis, how=how, subset=subset, inplace=inplace,
                                           **kw)
        cols = self._cols if subset is None else list(subset)
        cnt = self.nan_counts(cols)
        keep = cnt == 0 if how == "any" else cnt < len(cols)
        return self._take(np.flatnonzero(keep), inc=True)

    def nan_counts(self, cols=None) -> np.ndarray:
        """Per row of this frame, the number of NaN cells among ``cols`` (default: all): lag
        columns from the device (a lag cell is NaN when its source row is outside the base or
        the source cell is NaN) together with the unshifted copies of their sources; every
        other base column (ids, responses) and assigned columns on the host, without an
        upload."""
        cols = self._cols if cols is None else list(cols)
        self._check_cols(cols)
        n = self._nrows()
        cnt = np.zeros(n, dtype=np.int64)
        lag = {}
        ov, spec = self._overlay, self._spec
        # one pass over the (thousands of) column specs: lag columns grouped by shift, the
        # unshifted copies of numeric lag sources with them, everything else on the host
        specs = [spec[c] for c in cols if c not in ov]
        srcs = {t[0] for t in specs if t[2]}
        num = {nm: self._src.numeric(nm) for nm in srcs}
        host = []
        for t in specs:
            if t[2] or num.get(t[0], False):
                lag.setdefault(t[1], []).append(t[0])
            else:
                host.append(t[0])
        if ov:
            for c in cols:
                if c in ov:
                    cnt += pd.isna(ov[c]).astype(np.int64)
        sp = self._span()
        for nm in host:
            v = self._src.base[nm]
            if isinstance(v.dtype, np.dtype) and v.dtype.kind in "iub":
                continue                                    # integer / bool: no NaN
            na = np.isnan(v.to_numpy()) if (isinstance(v.dtype, np.dtype) and
                                            v.dtype.kind == "f") else v.isna().to_numpy()
            cnt += na[sp[0]:sp[1]] if sp is not None else na[self.positions()]
        if lag:
            self._lag_nan_counts(lag, cnt)
        return cnt

    def _any_nan(self) -> bool:
        """Whether any cell of this frame is NaN.  A row range whose lag columns read only
        base rows inside the base, from numeric sources without NaN, has none (O(1) after the
        upload); anything else counts per row."""
        sp = self._span()
        specs = [self._spec.get(c) for c in self._cols]
        if sp is None or self._overlay or any(sc is None or not self._src.numeric(sc[0])
                                              for sc in specs):
            return bool(self.nan_counts().any())
        if not specs:
            return False
        sh = [sc[1] for sc in specs]
        a, b = sp
        if a - max(max(sh), 0) < 0 or b - 1 - min(min(sh), 0) > self._src.N - 1:
            return bool(self.nan_counts().any())
        names = sorted({sc[0] for sc in specs}, key=str)
        self._src.upload(names)
        if any(self._src.has_nan(nm) for nm in names):
            return bool(self.nan_counts().any())
        return False

    def _lag_nan_counts(self, lag, out: np.ndarray) -> None:
        """Adds the NaN lag cells per row to ``out``; ``lag``: shift -> source names (one per
        lag column).  A cell is NaN when its source row u - s is outside the base (counted on
        the host from the edge rows only) or its source cell is NaN (device, for sources that
        hold any)."""
        import torch
        N = self._src.N
        pos = self.positions()
        n = pos.size
        sh = np.array(sorted(lag), dtype=np.int64)
        w = np.array([len(lag[s]) for s in sh], dtype=np.int64)
        smin, smax = int(sh[0]), int(sh[-1])
        sp = self._span()
        lo, hi = max(smax, 0), N + min(smin, 0)
        if sp is not None and lo <= hi:
            # rows a .. b - 1: the edge rows are the two ends of the range
            a, b = sp
            edge = np.r_[np.arange(a, min(b, lo)), np.arange(max(a, hi), b)] - a
        else:
            edge = np.flatnonzero((pos < lo) | (pos >= hi))
        if edge.size:
            u = pos[edge]
            cw = np.r_[0, np.cumsum(w)]
            # shifts s > u (source row u - s < 0) plus shifts s <= u - N (u - s >= N)
            gt = cw[-1] - cw[np.searchsorted(sh, u, side="right")]
            le = cw[np.searchsorted(sh, u - N, side="right")]
            out[edge] += gt + le
        names = sorted({nm for v in lag.values() for nm in v}, key=str)
        self._src.upload(names)
        if not any(self._src.has_nan(nm) for nm in names):
            return
        E, idx = self._src.device(names)
        row_of = {nm: int(r) for nm, r in zip(names, idx.tolist())}
        pos_d = torch.arange(sp[0], sp[1], dtype=torch.int64, device="cuda") if sp is not None \
            else torch.from_numpy(pos).to("cuda")
        acc = torch.zeros(n, dtype=torch.int64, device="cuda")
        for s, nms in lag.items():
            nn = [x for x in nms if self._src.has_nan(x)]
            if not nn:
                continue
            rws = torch.tensor([row_of[x] for x in nn], dtype=torch.int64, device="cuda")
            per_row = torch.isnan(E[rws]).sum(0)                 # NaN sources per base row
            u = pos_d - int(s)
            inside = (u >= 0) & (u < N)
            acc += torch.where(inside, per_row[u.clamp(0, N - 1)], torch.zeros_like(u))
        out += acc.cpu().numpy()

    # ------------------------------------------------------------------ values
    def _col_series(self, name) -> pd.Series:
        if name in self._overlay:
            return pd.Series(self._overlay[name], index=self.index, name=name)
        if name not in self._spec:
            raise KeyError(name)
        src, s, lag = self._spec[name]
        if not lag:
            return pd.Series(self._base_values(src), index=self.index, name=name)
        return pd.Series(self._lag_values([name])[:, 0], index=self.index, name=name)

    def _base_values(self, name) -> np.ndarray:
        v = self._src.base[name].to_numpy()
        sp = self._span()
        if self._rows is not None and sp is not None:
            v = v[sp[0]:sp[1]].copy()
        elif self._rows is not None:
            v = v[self._rows]
        elif v.base is not None or not v.flags.owndata:
            v = v.copy()
        cast = self._src.cast.get(name)
        return v if cast is None else v.astype(cast)

    def _base_frame(self, cols):
        return pd.DataFrame({c: self._base_values(self._spec[c][0]) for c in cols},
                            index=self.index, columns=cols)

    def _lag_values(self, names, rows=None) -> np.ndarray:
        """float64 host [n][len(names)] of lag columns, expanded on the device."""
        import torch
        from .timeshift import fill_bits
        srcs = [self._spec[c][0] for c in names]
        E, idx = self._src.device(sorted(set(srcs), key=str))
        rowmap = {nm: int(r) for nm, r in zip(sorted(set(srcs), key=str), idx.tolist())}
        cols_d = torch.tensor([rowmap[x] for x in srcs], dtype=torch.int32, device="cuda")
        sh_d = torch.tensor([self._spec[c][1] for c in names], dtype=torch.int32, device="cuda")
        pos = self.positions() if rows is None else self.positions()[rows]
        pos_d = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.int64)).to("cuda")
        k, n, N = len(names), int(pos.size), self._src.N
        out = torch.empty((n, k), dtype=torch.float64, device="cuda")
        _lib.call("sglm_timeshift_gather", E.data_ptr(), N, 1, N, cols_d.data_ptr(),
                  sh_d.data_ptr(), k, out.data_ptr(), n, k, 1, pos_d.data_ptr(), 8,
                  fill_bits(NAN, np.float64), torch.cuda.current_stream().cuda_stream)
        return out.cpu().numpy()

    def to_pandas(self) -> pd.DataFrame:
        """The DataFrame the reference would hold (every value materialised on the host)."""
        b = self._src.base
        pos = self.positions()
        lag = [c for c in self._cols if c not in self._overlay and self._spec[c][2]]
        lv = self._lag_values(lag) if lag else None
        li = {c: i for i, c in enumerate(lag)}
        data = {}
        for c in self._cols:
            if c in self._overlay:
                data[c] = self._overlay[c]
            elif c in li:
                data[c] = lv[:, li[c]]
            else:
                data[c] = self._base_values(self._spec[c][0])
        return pd.DataFrame(data, index=self.index, columns=self._cols)

    @_lazy
    def to_numpy(self, dtype=None, copy=False, na_value=None):
        a = self.to_pandas().to_numpy(dtype=dtype)
        return a

    @property
    def values(self):
        return super().values if self._mat is not None else self.to_numpy()

    @_lazy
    def __array__(self, dtype=None, copy=None):
        a = self.to_numpy()
        return a if dtype is None else a.astype(dtype)

    @_lazy
    def head(self, n=5):
        return self._take(np.arange(min(n, self._nrows()))).to_pandas()

    @_lazy
    def tail(self, n=5):
        k = self._nrows()
        return self._take(np.arange(max(0, k - n), k)).to_pandas()

    @_lazy
    def __repr__(self):
        k, m = self.shape
        if k <= 10:
            return repr(self.to_pandas())
        ht = self._take(np.r_[np.arange(5), np.arange(k - 5, k)]).to_pandas()
        with pd.option_context("display.max_rows", 9, "display.min_rows", 9,
                               "display.show_dimensions", False):
            body = repr(ht)
        return f"{body}\n\n[{k} rows x {m} columns]"

    def __getattr__(self, name):
        # only names that normal lookup did not find (pandas' methods are class attributes):
        # a column as an attribute, as DataFrame.__getattr__ gives it
        if name.startswith("_"):
            raise AttributeError(name)
        if self._mat is not None:
            return pd.DataFrame.__getattr__(self, name)
        if name in self._spec or name in self._overlay:
            return self._col_series(name)
        raise AttributeError(f"'LagFrame' object has no attribute {name!r}")

    # ------------------------------------------------------------------ device design
    def design(self):
        """engine.Design of this frame's values (every column numeric, no NaN cell), built from
        the device sources: lag and base columns alike are (source, shift) pairs; a column
        assigned to this frame (an overlay, e.g. the trial constants of
        sglm_cb_concat_make_design_mat.py:275) becomes a device source row holding its values at
        the frame's base rows (shift 0)."""
        if self._design is not None:
            return self._design
        from .engine import Design
        if self._mat is not None:
            # materialised (pandas code may have changed the values): the values as they are
            self._design = Design.from_host(self.to_numpy(dtype=np.float64))
            return self._design
        pos = self.positions()
        n = int(pos.size)
        ov = [c for c in self._cols if c in self._overlay]
        if ov and not self._inc and np.unique(pos).size != n:
            # repeated base rows: an assigned column's values have no one base row each
            self._design = Design.from_host(self.to_numpy(dtype=np.float64))
            return self._design
        if self._any_nan():
            raise ValueError("Input X contains NaN.")
        srcs = [self._spec[c][0] for c in self._cols if c not in self._overlay]
        names = sorted(set(srcs), key=str)
        at = {nm: i for i, nm in enumerate(names)}
        at.update({("__overlay__", c): len(names) + j for j, c in enumerate(ov)})
        cols = np.array([at[("__overlay__", c)] if c in self._overlay else at[self._spec[c][0]]
                         for c in self._cols], dtype=np.int64)
        shifts = np.array([0 if c in self._overlay else self._spec[c][1] for c in self._cols],
                          dtype=np.int64)
        sp = self._span()
        contiguous = n and (sp is not None or (pos[-1] - pos[0] == n - 1
                                               and np.all(np.diff(pos) == 1)))
        if contiguous and not ov:
            # every source 0/1 and the canonical lag layout: the design straight from the
            # uploaded bit rows (no float64 copy of the sources)
            B = self._src.bits(names)
            if B is not None:
                ones = np.array([self._src.ones(nm) for nm in names], dtype=np.int64)
                d = Design.from_lagged_bits(B, self._src.N, cols, shifts, int(pos[0]), n, ones)
                if d is not None:
                    self._design = d
                    return d
        import torch
        if names:
            E, idx = self._src.device(names)
            Esub = E[idx]
            if any(self._src.has_nan(nm) for nm in names):
                Esub = Esub.nan_to_num(0.0)    # NaN source cells are never read (checked above)
        else:
            Esub = torch.zeros((0, self._src.N), dtype=torch.float64, device="cuda")
        ones = [self._src.ones(nm) for nm in names]
        ones = None if any(o is None for o in ones) else ones
        if ov:
            # assigned columns: device rows over the base rows, their values at this frame's
            # rows (0 elsewhere: never read, and a 0/1 column stays 0/1)
            vals = np.stack([pd.array(self._overlay[c]).to_numpy(dtype=np.float64,
                                                                  na_value=np.nan)
                             for c in ov])
            Eov = torch.zeros((len(ov), self._src.N), dtype=torch.float64, device="cuda")
            pos_d = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.int64)).to("cuda")
            Eov[:, pos_d] = torch.from_numpy(vals).to("cuda")
            Esub = torch.cat([Esub, Eov])
            ones = None
        if contiguous:
            d = Design.from_lagged(Esub, cols, shifts, int(pos[0]), n, ones=ones)
        else:
            rows_d = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.int64)).to("cuda")
            d = Design.from_lagged(Esub, cols, shifts, 0, n, rows=rows_d)
        self._design = d
        return d


class _LagNA:
    """``frame.isna()`` (``negate``: ``notna()``) answered from the NaN counts per row."""

    def __init__(self, frame: LagFrame, negate: bool = False):
        self.frame = frame
        self.negate = negate

    def sum(self, axis=0, **kw):
        if axis in (1, "columns") and not kw:
            c = self.frame.nan_counts()
            if self.negate:
                c = len(self.frame._cols) - c
            return pd.Series(c, index=self.frame.index)
        return getattr(self._real(), "sum")(axis=axis, **kw)

    def any(self, axis=0, **kw):
        if axis in (1, "columns") and not kw:
            c = self.frame.nan_counts()
            full = len(self.frame._cols)
            return pd.Series((c < full) if self.negate else (c > 0), index=self.frame.index)
        return getattr(self._real(), "any")(axis=axis, **kw)

    def all(self, axis=0, **kw):
        if axis in (1, "columns") and not kw:
            c = self.frame.nan_counts()
            full = len(self.frame._cols)
            return pd.Series((c == 0) if self.negate else (c == full), index=self.frame.index)
        return getattr(self._real(), "all")(axis=axis, **kw)

    def _real(self):
        df = self.frame.to_pandas()
        return df.notna() if self.negate else df.isna()

    def __getattr__(self, name):
        return getattr(self._real(), name)

    def __repr__(self):
        return repr(self._real())


class _Loc:
    def __init__(self, frame):
        self.f = frame

    def __getitem__(self, key):
        f = self.f
        if isinstance(key, tuple):
            rk, ck = key
            out = self[rk] if not (isinstance(rk, slice) and rk == slice(None)) else f
            if isinstance(out, LagFrame):
                return out[ck]
            return out.loc[:, ck]
        arr = key if isinstance(key, (pd.Series, np.ndarray, pd.Index)) else None
        if arr is not None and pd.api.types.is_bool_dtype(arr.dtype):
            return f._bool_rows(key)
        if isinstance(key, slice):
            sl = f.index.slice_indexer(key.start, key.stop, key.step)
            return f._take(np.arange(len(f))[sl])
        labels = [key] if np.isscalar(key) else list(key)
        pos = f.index.get_indexer(labels)
        if (pos < 0).any():
            raise KeyError(f"{[l for l, q in zip(labels, pos) if q < 0]} not in index")
        out = f._take(pos)
        return out.to_pandas().iloc[0] if np.isscalar(key) else out


class _ILoc:
    def __init__(self, frame):
        self.f = frame

    def __getitem__(self, key):
        f = self.f
        if isinstance(key, tuple):
            rk, ck = key
            out = self[rk] if not (isinstance(rk, slice) and rk == slice(None)) else f
            cols = np.asarray(f._cols, dtype=object)[ck]
            if isinstance(out, LagFrame):
                return out[list(np.atleast_1d(cols))] if not np.isscalar(cols) else out[cols]
            return out.iloc[:, ck]
        if np.isscalar(key):
            return f._take(np.array([int(key)])).to_pandas().iloc[0]
        return f._take(np.arange(len(f))[key])
