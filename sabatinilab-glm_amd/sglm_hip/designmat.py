"""Event design matrix on the MI355X: host driver of the sglm_group_rows / sglm_dm_* kernels.

Restates /root/reference/pp_design_mat.py:6-205 (make_design_mat and its helpers).  The
pandas work of the reference -- per-row lick products, groupby('nTrial') cumcount / nth /
first / sum, Series.map lookups into the trial table, dummy interactions -- runs on float64
device columns (csrc/designmat.hip); the host keeps the bookkeeping that pandas does on
column NAMES (which columns a regex picks, get_dummies labels, output order and dtypes) and
the small trial table (10^2-10^4 rows).

Output dtypes follow pandas in this image where pandas yields a numpy dtype (int64 for the
cue / pulled-lick / flag columns and for counters whose values are all integral, float64
elsewhere).  Where pandas yields an object column (a dummy or isna map with unmapped trial
ids: mixed numbers and NaN) or a nullable extension column (the maps of the convert_dtypes'd
trial table: Int64 / Float64), the same numbers are returned as float64 -- numerically
identical, and the numeric consumers of the matrix (timeshift, fit) need float64 anyway.
"""
from __future__ import annotations

import ctypes
import re
import warnings
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from . import _lib

try:
    import torch
except ImportError as e:  # pragma: no cover
    raise _lib.HipEngineUnavailable("PyTorch-ROCm is required for device memory") from e

MAX_COLS = 32
MAX_PULL = 16


def _require_gpu():
    _lib.load()
    if not torch.cuda.is_available():
        raise _lib.HipEngineUnavailable(
            "no ROCm GPU visible: the sglm HIP engine has no CPU fallback")


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _ptrs(tensors):
    arr = (ctypes.c_void_p * max(len(tensors), 1))(*[t.data_ptr() for t in tensors])
    return ctypes.cast(arr, ctypes.c_void_p), arr


class _Stage:
    """The small host inputs of one design matrix (trial ids, mapped per-trial values, index
    lists) in ONE asynchronous copy from pinned memory: a pageable ``.to('cuda')`` waits for
    every kernel queued before it, a host round trip per upload.  A ring of pinned buffers;
    a buffer is rewritten only after the copy out of it (event) has run."""

    SLOTS = 4

    def __init__(self):
        self.h = [None] * self.SLOTS
        self.d = [None] * self.SLOTS
        self.ev = [None] * self.SLOTS
        self.i = 0

    def upload(self, arrays, dev):
        arrs = [np.ascontiguousarray(a) for a in arrays]
        offs, o = [], 0
        for a in arrs:
            offs.append(o)
            o += (a.nbytes + 255) // 256 * 256
        k = self.i
        self.i = (k + 1) % self.SLOTS
        if self.ev[k] is not None:
            self.ev[k].synchronize()
        if self.h[k] is None or self.h[k].numel() < o:
            # every slot at once (page-locking is slow: not once per call of the first few)
            size = max(o, 256) * 2
            for j in range(self.SLOTS):
                if self.ev[j] is not None:
                    self.ev[j].synchronize()
                self.h[j] = torch.empty(size, dtype=torch.uint8).pin_memory()
                self.d[j] = torch.empty(size, dtype=torch.uint8, device=dev)
        hb = self.h[k].numpy()
        for a, off in zip(arrs, offs):
            hb[off:off + a.nbytes] = a.reshape(-1).view(np.uint8)
        self.d[k][:o].copy_(self.h[k][:o], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.ev[k] = ev
        out = []
        for a, off in zip(arrs, offs):
            t = self.d[k][off:off + a.nbytes].view(_TORCH_DT[a.dtype])
            out.append(t.view(a.shape))
        return out


_TORCH_DT = {np.dtype(np.float64): torch.float64, np.dtype(np.int32): torch.int32,
             np.dtype(np.uint8): torch.uint8}
_STAGE = _Stage()


@dataclass
class Grouping:
    """A pandas groupby over float keys on the device: perm[:m] = the rows with non-NaN keys,
    grouped by key (row order within a group), seg = group starts (+ m), counts = {m, nseg,
    ordered} (device).  ``sorted``: the keys were already ordered (no sort was needed) -- a
    readback, so only asked for by tests."""
    perm: "torch.Tensor"
    seg: "torch.Tensor"
    counts: "torch.Tensor"

    @property
    def sorted(self) -> bool:
        return bool(self.counts[2].item())


class Workspace:
    """Grow-only device scratch of the grouping (one per session size)."""

    def __init__(self):
        self.buf = None

    def get(self, n, dev):
        nb = _lib.query("sglm_group_rows_work_bytes", int(n))
        if self.buf is None or self.buf.numel() < nb:
            self.buf = torch.empty(nb, dtype=torch.uint8, device=dev)
        return self.buf


_WS = Workspace()


def group_rows(key, key2=None, ws: Optional[Workspace] = None) -> Grouping:
    n = int(key.numel())
    dev = key.device
    perm = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    seg = torch.empty(n + 1, dtype=torch.int64, device=dev)
    counts = torch.empty(3, dtype=torch.int64, device=dev)
    _lib.call("sglm_group_rows", _p(key), _p(key2), n, _p(perm), _p(seg), _p(counts), None,
              _p((ws or _WS).get(n, dev)), _stream())
    return Grouping(perm, seg, counts)


class TrialTable:
    """The trial table indexed by nTrial (trials.set_index('nTrial'), :152) on the device:
    ascending unique ids and, per mapped quantity, one float64 row in that order (NaN for
    missing values)."""

    def __init__(self, index_values, dev):
        ids = np.asarray(index_values, dtype=np.float64)
        if ids.size and np.isnan(ids).any():
            ids = ids.copy()
        self.order = np.argsort(ids, kind="stable")
        sid = ids[self.order]
        self.keys = torch.from_numpy(np.ascontiguousarray(sid)).to(dev)
        self.n = int(sid.size)
        self.dev = dev

    def values(self, per_trial):
        """Device float64 [k][n] of host per-trial rows (trial-table order)."""
        v = np.atleast_2d(np.asarray(per_trial, dtype=np.float64))[:, self.order]
        return torch.from_numpy(np.ascontiguousarray(v)).to(self.dev)

    def lookup(self, key):
        tidx = torch.empty(int(key.numel()), dtype=torch.int32, device=key.device)
        _lib.call("sglm_trial_lookup", _p(key), int(key.numel()), _p(self.keys), self.n,
                  _p(tidx), _stream())
        return tidx


def heatmap(cols: Dict[str, "torch.Tensor"], g: Grouping, tidx, tsel):
    """add_heatmap_columns (:108-126): device [5][n] in the reference's column order."""
    n = int(cols["nTrial"].numel())
    out = torch.empty((5, max(n, 1)), dtype=torch.float64, device=cols["nTrial"].device)
    _lib.call("sglm_dm_heatmap", _p(cols["trial_clock"]), _p(cols["Cue"]),
              _p(cols["Consumption"]), _p(cols["stateConsumption"]), n, _p(g.perm), _p(g.seg),
              _p(g.counts), _p(tidx), _p(tsel), _p(out), out.shape[1], _stream())
    return out


HM_COLUMNS = ["hm_t_cue_offset_to_sel", "hm_t_from_cue_onset", "hm_t_from_cons_onset",
              "hm_t_sel_to_cons", "hm_t_cue_offset_to_cons"]


def licks(lick_src, from_spout: bool, states: List["torch.Tensor"], want_lick=False):
    """classify_lick_state (:6-23) (and Lick = ~isnan(iSpout), :160): device columns."""
    if len(states) > MAX_COLS:
        raise ValueError(f"at most {MAX_COLS} lick states")
    n = int(lick_src.numel())
    outs = [torch.empty(n, dtype=torch.float64, device=lick_src.device) for _ in states]
    lk = torch.empty(n, dtype=torch.float64, device=lick_src.device) if want_lick else None
    sp, keep1 = _ptrs(states)
    op, keep2 = _ptrs(outs)
    _lib.call("sglm_dm_licks", _p(lick_src), int(from_spout), sp, len(states), n, op, _p(lk),
              _stream())
    return outs, lk


def counters(cols, g: Grouping, g2: Grouping):
    """The cumcount**2 counters and the cue onset column (:167-183)."""
    n = int(cols["nTrial"].numel())
    dev = cols["nTrial"].device
    tenl, tenlp, cue = (torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3))
    _lib.call("sglm_dm_counters", _p(cols["ENL"]), _p(cols["Cue"]), _p(cols["state_ENLP"]), n,
              _p(g.perm), _p(g.seg), _p(g.counts), _p(g2.perm), _p(g2.seg), _p(g2.counts),
              _p(tenl), _p(tenlp), _p(cue), _stream())
    return tenl, tenlp, cue


def pull(bout, g: Grouping, nth_order: List[int], cols: List["torch.Tensor"], key=None):
    """pull_lick_from_bout (:44-53) over positions in processing order (bout updated in
    place).  ``key``: the grouping's key (the zero pass then skips the group rows)."""
    if len(nth_order) > MAX_PULL:
        raise ValueError(f"at most {MAX_PULL} lick positions")
    if not nth_order:
        return
    nth = (ctypes.c_int32 * len(nth_order))(*[int(v) for v in nth_order])
    cp, keep = _ptrs(cols)
    _lib.call("sglm_dm_pull_k", _p(bout), _p(key), int(bout.numel()), _p(g.perm), _p(g.seg),
              _p(g.counts), ctypes.cast(nth, ctypes.c_void_p), len(nth_order), cp, _stream())


def trial_map(tidx, block, src_cols, vals, val_cols, out_block, dst_cols):
    """out_block[dst] = (block[src] or 1) * vals[val][trial of row] (NaN when unmapped)."""
    n = int(tidx.numel())
    if not dst_cols:
        return
    dev = tidx.device
    sc = torch.tensor(src_cols, dtype=torch.int32, device=dev)
    vc = torch.tensor(val_cols, dtype=torch.int32, device=dev)
    dc = torch.tensor(dst_cols, dtype=torch.int32, device=dev)
    _lib.call("sglm_trial_map", n, _p(tidx), _p(block), 0 if block is None else block.shape[1],
              _p(sc), _p(vals), vals.shape[1], _p(vc), len(dst_cols), _p(out_block),
              out_block.shape[1], _p(dc), _stream())


def zero_groups_flag(g: Grouping, block, cols: List[int], flag):
    n = int(flag.numel())
    cd = torch.tensor(cols if cols else [0], dtype=torch.int32, device=flag.device)
    _lib.call("sglm_zero_groups_flag", n, _p(g.perm), _p(g.seg), _p(g.counts), _p(block),
              block.shape[1], _p(cd), len(cols), _p(flag), None, _stream())


# ----------------------------------------------------------------------------- the wrapper
DEVICE_INPUTS = ["nTrial", "nENL", "iSpout", "Cue", "ENL", "state_ENLP", "Consumption",
                 "stateConsumption", "trial_clock"]


def _masked(series):
    """(values, NA mask) of a numeric numpy or nullable (masked) trial-table column, else
    None: the plain arrays, without pandas' per-call conversions."""
    arr = series.array
    data, mask = getattr(arr, "_data", None), getattr(arr, "_mask", None)
    if isinstance(data, np.ndarray) and isinstance(mask, np.ndarray) and data.dtype.kind in "iufb":
        return data, mask
    v = series.to_numpy()
    if isinstance(v, np.ndarray) and v.dtype.kind in "iub":
        return v, np.zeros(v.shape, dtype=bool)
    if isinstance(v, np.ndarray) and v.dtype.kind == "f":
        return v, np.isnan(v)
    return None


def _f64(series):
    """series.to_numpy(float64, na_value=nan)."""
    dm = _masked(series)
    if dm is None:
        return series.to_numpy(dtype=np.float64, na_value=np.nan)
    data, mask = dm
    out = data.astype(np.float64)
    out[mask] = np.nan
    return out


def _na_mask(series):
    """series.isna() as a bool array."""
    dm = _masked(series)
    return series.isna().to_numpy(dtype=bool) if dm is None else dm[1]


def _isna(series):
    """series.isna() as float64 0/1."""
    return _na_mask(series).astype(np.float64)


def _dummy_rows(series, trial_type):
    """pd.get_dummies(trials[trial_type], prefix=trial_type) (:88) on the host (a trial-table
    column): the labels the reference puts in the new names (dummy_col.split('_')[-1], :96)
    and the 0/1 indicator of each level as uint8 rows [level][trial].  Numeric / nullable
    numeric columns: the sorted distinct non-NA values (get_dummies' categories:
    factorize(sort=True)), formatted as pandas formats the column names; other dtypes
    through pandas."""
    dm = _masked(series)
    if dm is not None:
        data, mask = dm
        anyna = bool(mask.any())
        v = data[~mask] if anyna else data
        levels = None
        if v.dtype.kind in "iu" and v.size:
            lo, hi = int(v.min()), int(v.max())
            if hi - lo < 65536:                      # small integer codes: a count, no sort
                cnt = np.bincount(v if lo == 0 else v - lo, minlength=hi - lo + 1)
                levels = (np.flatnonzero(cnt) + lo).astype(v.dtype)
        if levels is None:
            levels = np.unique(v)
        if not (levels.dtype.kind == "f" and np.isnan(levels).any()):
            rows = np.empty((levels.size, data.size), dtype=np.uint8)
            for d, lv in enumerate(levels):
                eq = data == lv
                if anyna:
                    eq &= ~mask
                rows[d] = eq
            return [str(f"{trial_type}_{x}").split("_")[-1] for x in levels.tolist()], rows
    import pandas as pd
    d = pd.get_dummies(series, prefix=trial_type)
    return ([str(c).split("_")[-1] for c in d.columns],
            np.ascontiguousarray(d.to_numpy(dtype=np.uint8).T))


def _dummy_labels(series, trial_type):
    """_dummy_rows with float64 values [trial][level] (get_dummies' frame layout)."""
    labels, rows = _dummy_rows(series, trial_type)
    return labels, rows.T.astype(np.float64)


@dataclass
class DesignResult:
    names: List[str]
    block: "torch.Tensor"          # [len(names)][n] float64 device, in `names` order
    base_dtypes: List[object]      # per column, before the mapped-NaN rule below
    factored: List[bool]           # the column is a product with mapped trial dummies
    mapped_nan: object = False     # device bool: some row maps to no trial (dummies -> NaN)
    lick: Optional["torch.Tensor"] = None          # the Lick column (:160)
    without: Optional[np.ndarray] = None           # trials_without_dummies (:201)

    @property
    def dtypes(self) -> List[object]:
        """pandas' dtypes: a dummy product is float64 (object in pandas) when some row's trial
        is unmapped.  Resolving it reads one flag back (after the block's download in
        to_frame, so it costs nothing there)."""
        if not isinstance(self.mapped_nan, bool):
            self.mapped_nan = bool(self.mapped_nan.item())
        return [np.dtype(np.float64) if (self.mapped_nan and f) else dt
                for dt, f in zip(self.base_dtypes, self.factored)]


@dataclass
class _Recipe:
    """A design-matrix column: a base column times the mapped dummies of ``factors``
    ((trial_type, dummy index) pairs, applied in order by event_interactions_dummies)."""
    base: str
    factors: tuple
    dtype: object


def upload(timeseries, states):
    """One host->device copy of every session column the device path reads (float64 block);
    returns ({name: device row}, {name: source dtype})."""
    _require_gpu()
    orig = list(timeseries.columns)
    photo = [c for c in orig if "z_grn" in c]
    pre_lick = [c for c in orig if "_lick" in c]
    needed = list(dict.fromkeys(DEVICE_INPUTS + list(states) + ["iBlock"] + photo + pre_lick))
    for c in needed:
        if c not in timeseries.columns:
            raise KeyError(c)
    n = len(timeseries)
    host = np.empty((len(needed), n), dtype=np.float64)
    src_dtypes = {}
    for j, c in enumerate(needed):
        sr = timeseries[c]
        src_dtypes[c] = sr.dtype
        host[j] = sr.to_numpy(dtype=np.float64, na_value=np.nan)
    blk = torch.from_numpy(host).to("cuda")
    cols = {c: blk[j] for j, c in enumerate(needed)}
    cols["__order__"] = orig
    return cols, src_dtypes


def design_matrix(timeseries, trials_idx, states, nth_licks, interactions, verbose=True):
    """make_design_mat (:128-205) over a host DataFrame; ``trials_idx`` is the trial table
    after set_index('nTrial').convert_dtypes() (:152-153)."""
    cols, src_dtypes = upload(timeseries, states)
    return design_matrix_device(cols, src_dtypes, len(timeseries), trials_idx, states,
                                nth_licks, interactions, verbose)


def _plan(orig, src_dtypes, states, nth_licks, interactions, trials_idx):
    """The reference's column-name flow (:155-196) on names only: the final column list with
    one recipe per column, and the per-interaction dummy tables."""
    bout = "con_lick"
    photo = [c for c in orig if "z_grn" in c]
    pre_lick = [c for c in orig if "_lick" in c]
    rec: Dict[str, _Recipe] = {c: _Recipe("in:" + c, (), src_dtypes[c]) for c in pre_lick}
    names = list(pre_lick)
    for st in states:                     # classify_lick_state: a repeated name is overwritten
        nm = f"{st[:3].lower()}_lick"
        if nm not in names:
            names.append(nm)
        rec[nm] = _Recipe("lick:" + nm, (), np.result_type(src_dtypes[st], np.int64))
    names += ["nTrial", "iBlock", "time_from_enl_onset", "time_from_enlp_onset"] + photo + ["cue"]
    rec["nTrial"] = _Recipe("in:nTrial", (), src_dtypes["nTrial"])
    rec["iBlock"] = _Recipe("in:iBlock", (), src_dtypes["iBlock"])
    rec["time_from_enl_onset"] = _Recipe("tenl", (), "counter")
    rec["time_from_enlp_onset"] = _Recipe("tenlp", (), "counter")
    for c in photo:
        rec[c] = _Recipe("in:" + c, (), src_dtypes[c])
    rec["cue"] = _Recipe("cue", (), np.dtype(np.int64))
    if bout not in names:
        raise KeyError(bout)
    order = sorted(nth_licks)[::-1] if len(nth_licks) > 1 else list(nth_licks)
    pulls = []
    for nth in order:
        nm = f"{bout}_{nth}"
        if nm not in pulls:
            pulls.append(nm)
        if nm not in names:
            names.append(nm)
        rec[nm] = _Recipe("pull:" + nm, (), np.dtype(np.int64))
    bout_base = rec[bout].base
    names.remove(bout)
    dummies = {}
    if interactions:
        names.append("flag")
        rec["flag"] = _Recipe("flag", (), "flag")
        for trial_type, st_ in interactions.items():
            pat = "|".join(x.lower()[:3] for x in st_)
            picked = [c for c in names if re.search(pat, str(c))]
            if "flag" in picked or "nTrial" in picked:
                raise NotImplementedError(
                    f"interaction pattern {pat!r} picks the 'flag' / 'nTrial' column, which the "
                    "reference then fails to update (KeyError at pp_design_mat.py:192)")
            later = [c for c in names if c not in picked]
            labels, drows = _dummy_rows(trials_idx[trial_type], trial_type)
            dummies[trial_type] = drows
            new = []
            for d, lab in enumerate(labels):
                for c in picked:
                    nm = f"{trial_type.lower()[:3]}_{lab}_{c}"
                    new.append(nm)
                    r = rec[c]
                    dt = r.dtype if isinstance(r.dtype, str) else \
                        np.result_type(r.dtype, np.bool_)
                    rec[nm] = _Recipe(r.base, r.factors + ((trial_type, d),), dt)
            names = new + later
    else:
        names.append("flag")                       # reference: KeyError('flag') (:196), fixed
        rec["flag"] = _Recipe("flag", (), np.dtype(np.int64))
    names += HM_COLUMNS
    for j, c in enumerate(HM_COLUMNS):
        rec[c] = _Recipe(f"hm:{j}", (), np.dtype(np.float64))
    return names, rec, pulls, order, bout_base, dummies


def design_matrix_device(cols, src_dtypes, n, trials_idx, states, nth_licks, interactions,
                         verbose=True) -> DesignResult:
    """make_design_mat on session columns already in HBM (``upload``).  Every kernel writes
    its final slot of ONE output block (no intermediate copies): the column plan comes first
    (host, names only), then the grouping, the row / group kernels, one trial-map launch for
    all interaction columns, the flag."""
    import pandas as pd
    _require_gpu()
    dev = "cuda"
    if not trials_idx.index.is_unique:
        raise pd.errors.InvalidIndexError(
            "Reindexing only valid with uniquely valued Index objects")
    orig = cols["__order__"]
    names, rec, pulls, order, bout_base, dummies = _plan(orig, src_dtypes, states, nth_licks,
                                                         interactions, trials_idx)
    K = len(names)
    # slots: final columns first, then scratch rows for bases used only through factors
    slot = {}
    for q, c in enumerate(names):
        if not rec[c].factors:
            slot[rec[c].base] = q
    scratch = []
    for c in names:
        b = rec[c].base
        if b not in slot and b not in scratch:
            scratch.append(b)
    if bout_base not in slot and bout_base not in scratch:
        scratch.append(bout_base)                 # the pull's working column (:185, dropped)
    for b in ["lick:" + f"{st[:3].lower()}_lick" for st in states] + ["tenl", "tenlp", "cue"] \
            + ["pull:" + p for p in pulls]:
        if b not in slot and b not in scratch:
            scratch.append(b)                     # computed anyway (one kernel writes them)
    for b in scratch:
        slot[b] = K + scratch.index(b)
    blk = torch.empty((K + len(scratch), max(n, 1)), dtype=torch.float64, device=dev)
    row = lambda b: blk[slot[b]]                  # noqa: E731
    # every host input of the kernels below (the trial table's ids in ascending order and its
    # mapped rows, the trial-map index lists, the cue-like columns) in ONE staged copy,
    # enqueued before the first kernel: no host round trip in the whole matrix
    ids = trials_idx.index.to_numpy(dtype=np.float64, na_value=np.nan)
    nt = int(ids.size)
    # the trial table in ascending id order (usually it already is: no gather then)
    if nt < 2 or bool(np.all(ids[1:] > ids[:-1])):
        asc = lambda a: a                                           # noqa: E731
    else:
        torder = np.argsort(ids, kind="stable")
        asc = lambda a: np.ascontiguousarray(a[..., torder])        # noqa: E731
    inter = [c for c in names if rec[c].factors]
    fq = names.index("flag")
    cue_like = [names.index(c) for c in names if str(c).endswith("cue")]
    # per interaction column its per-trial factor, the product of its 0/1 dummies (uint8:
    # exact, an eighth of the float64 upload)
    fv = np.ones((len(inter), nt), dtype=np.uint8)
    for j, c in enumerate(inter):
        for tt_name, d in rec[c].factors:
            fv[j] &= dummies[tt_name][d]
    isna = np.zeros(nt, dtype=bool)
    for trial_type in (interactions or {}):
        isna |= _na_mask(trials_idx[trial_type])
    i32 = lambda v: np.asarray(v, dtype=np.int32)          # noqa: E731
    (tkeys, tsel, fvd, isnad, isrc, ival, idst, fsrc, fval, fdst, cd) = _STAGE.upload([
        asc(ids), asc(_f64(trials_idx["tSelection"])), asc(fv),
        asc(isna.view(np.uint8))[None, :],
        i32([slot[rec[c].base] for c in inter]), i32(range(len(inter))),
        i32([names.index(c) for c in inter]), i32([-1]), i32([0]), i32([fq]),
        i32(cue_like if cue_like else [0])], dev)
    g = group_rows(cols["nTrial"])
    g2 = group_rows(cols["nTrial"], cols["nENL"])
    tidx = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    _lib.call("sglm_trial_lookup", _p(cols["nTrial"]), n, _p(tkeys), nt, _p(tidx), _stream())
    # add_heatmap_columns: the five hm rows are consecutive at the end of the block
    # (the _k entries: the per-row default passes write only the rows outside every group)
    _lib.call("sglm_dm_heatmap_k", _p(cols["trial_clock"]), _p(cols["Cue"]),
              _p(cols["Consumption"]), _p(cols["stateConsumption"]), _p(cols["nTrial"]), n,
              _p(g.perm), _p(g.seg), _p(g.counts), _p(tidx), _p(tsel), _p(row("hm:0")),
              blk.shape[1], _stream())
    lick_col = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    st_src = [cols[st] for st in states]
    st_dst = [row("lick:" + f"{st[:3].lower()}_lick") for st in states]
    sp, k1 = _ptrs(st_src)
    dp, k2 = _ptrs(st_dst)
    _lib.call("sglm_dm_licks", _p(cols["iSpout"]), 1, sp, len(states), n, dp, _p(lick_col),
              _stream())
    _lib.call("sglm_dm_counters_k", _p(cols["ENL"]), _p(cols["Cue"]), _p(cols["state_ENLP"]),
              _p(cols["nTrial"]), _p(cols["nENL"]), n, _p(g.perm), _p(g.seg), _p(g.counts),
              _p(g2.perm), _p(g2.seg), _p(g2.counts), _p(row("tenl")), _p(row("tenlp")),
              _p(row("cue")), _stream())
    # inputs that are columns of the matrix (or sources of interactions) are copied in
    for b, q in slot.items():
        if b.startswith("in:"):
            blk[q, :n].copy_(cols[b[3:]][:n])
    pull(row(bout_base), g, order, [row("pull:" + f"con_lick_{nth}") for nth in order],
         key=cols["nTrial"])
    # interactions: every column with factors in one trial-map launch, the per-trial factor
    # the product of its dummies (0/1 exact, in any order)
    ld = blk.shape[1]
    if inter:
        _lib.call("sglm_trial_map_u8", n, _p(tidx), _p(blk), ld, _p(isrc), _p(fvd), nt,
                  _p(ival), len(inter), _p(blk), ld, _p(idst), _stream())
    # flag (:189-203): the mapped isna sums, clipped
    if interactions:
        _lib.call("sglm_trial_map_u8", n, _p(tidx), None, 0, _p(fsrc), _p(isnad), nt, _p(fval),
                  1, _p(blk), ld, _p(fdst), _stream())
    else:
        blk[fq].zero_()
    gz = torch.zeros(max(n, 1), dtype=torch.uint8, device=dev) if verbose else None
    _lib.call("sglm_zero_groups_flag", n, _p(g.perm), _p(g.seg), _p(g.counts), _p(blk), ld,
              _p(cd), len(cue_like), _p(blk[fq]), _p(gz), _stream())
    mapped_nan = (tidx[:n] < 0).any() if (interactions and n) else False
    res = DesignResult(names, blk[:K, :n], [rec[c].dtype for c in names],
                       [bool(rec[c].factors) for c in names], mapped_nan, lick_col[:n])
    if verbose:
        res.without = _without(g, gz, cols["nTrial"])
        print(f"trials_without_dummies = {res.without!r}")
    return res


def _without(g: Grouping, gz, key):
    """The keys of the groups flagged for having no cue dummy (one small readback)."""
    m, ns = (int(v) for v in g.counts[:2].cpu().tolist())
    if ns == 0:
        return np.array([], dtype=np.float64)
    z = gz[:ns].cpu().numpy().astype(bool)
    heads = g.perm[g.seg[:ns]]
    keys = key[heads].cpu().numpy()
    return keys[z]


def to_frame(res: DesignResult, index):
    """Download the device block (one copy) and build the DataFrame with pandas' dtypes."""
    import pandas as pd
    host = res.block.cpu().numpy()
    data = {}
    for j, (c, dt) in enumerate(zip(res.names, res.dtypes)):
        v = host[j]
        if isinstance(dt, str):                     # "counter" / "flag": int64 when integral
            integral = bool(np.all(np.isfinite(v))) and bool(np.all(v == np.round(v)))
            data[c] = v.astype(np.int64) if integral else v
        elif isinstance(dt, np.dtype) and dt.kind in "iub":
            data[c] = v.astype(dt) if np.all(np.isfinite(v)) else v
        elif isinstance(dt, np.dtype):
            data[c] = v.astype(dt)
        else:                                        # extension / object source dtypes
            data[c] = v
    return pd.DataFrame(data, index=index, columns=res.names)
