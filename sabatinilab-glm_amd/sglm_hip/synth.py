"""Synthetic inputs of the shape BASELINE.json's configs name.

Base events ``E in {0,1}^{N_raw x m}`` i.i.d. Bernoulli(rho) from ``default_rng(seed)``;
lags ``[-L, ..., L-1]`` expanded in the shift-major layout of
``sglm_ez.timeshift_cols`` (backend/sglm_ez.py:102-123: shifts ``[0] + [-L..-1] + [1..L-1]``);
the first ``L-1`` and last ``L`` rows of the expansion hold the NaN fill and are dropped, so
``N_raw = N + 2L - 1`` leaves exactly ``N`` rows.  ``beta_true ~ N(0, 0.1^2)`` (rng 1);
Poisson ``y ~ Poisson(exp(X beta + b))`` with ``b = -1`` (rng 2); Gaussian
``y = X beta + 0.5 + N(0, 1)``.  Trial ids ``t // 100``.

The linear predictor is computed by per-event convolution of E with the lag kernel, so the
1M x 2000 design never has to exist on the host.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Synthetic:
    E: np.ndarray            # (N_raw, m) float32 0/1 events
    L: int                   # lags -L..L-1
    shifts: list             # shift-major shift list
    N: int                   # rows after the NaN drop
    beta: np.ndarray         # (p,) true coefficients, shift-major column order
    intercept: float
    y: np.ndarray            # (N,) response
    trial: np.ndarray        # (N,) trial ids
    family: str

    @property
    def p(self):
        return len(self.shifts) * self.E.shape[1]

    def dense_X(self, dtype=np.float64):
        """Materialise X (N x p) on the host — small configs / tests only."""
        Nr, m = self.E.shape
        X = np.empty((self.N, self.p), dtype=dtype)
        r0 = self.L - 1
        for bi, s in enumerate(self.shifts):
            X[:, bi * m:(bi + 1) * m] = self.E[r0 - s:r0 - s + self.N]
        return X


def shift_list(L):
    return [0] + list(range(-L, 0)) + list(range(1, L))


def make(N, m, L, family="poisson", rho=0.02, seed=0, beta_scale=0.1, intercept=None):
    rng = np.random.default_rng(seed)
    N_raw = N + 2 * L - 1
    E = (rng.random((N_raw, m)) < rho).astype(np.float32)
    shifts = shift_list(L)
    p = len(shifts) * m
    beta = np.random.default_rng(seed + 1).normal(0.0, beta_scale, size=p)
    b = (-1.0 if family == "poisson" else 0.5) if intercept is None else intercept
    # eta[t] = sum_{shift s, event a} E[t + r0 - s, a] * beta[s, a]  (r0 = L-1)
    eta = np.full(N, b, dtype=np.float64)
    r0 = L - 1
    B = beta.reshape(len(shifts), m)
    for bi, s in enumerate(shifts):
        eta += E[r0 - s:r0 - s + N].astype(np.float64) @ B[bi]
    rng2 = np.random.default_rng(seed + 2)
    if family == "poisson":
        y = rng2.poisson(np.exp(eta)).astype(np.float64)
    elif family == "gamma":
        mu = np.exp(eta)
        y = rng2.gamma(2.0, mu / 2.0)
    else:
        y = eta + rng2.normal(0.0, 1.0, size=N)
    trial = np.arange(N) // 100
    return Synthetic(E=E, L=L, shifts=shifts, N=N, beta=beta, intercept=b, y=y,
                     trial=trial, family=family)


SESSION_LONG_NAMES = {"cpn": "centerIn", "lpx": "leftOut", "rpx": "rightOut", "lpn": "leftIn",
                      "rpn": "rightIn", "r": "reward", "nr": "noreward", "rl": "rightLick",
                      "ll": "leftLick"}


def session(n: int, seed: int, rate: float = 0.02, with_extra: bool = True):
    """Seeded behaviour session with the long column names of the acquisition files: sparse
    0/1 port entries/exits, licks and reward outcomes, a photometry trace and an 'Unnamed'
    index column; center entries precede side exits so trials form."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    cols = {}
    for short in ("cpn", "lpx", "rpx", "lpn", "rpn", "rl", "ll"):
        cols[short] = (rng.random(n) < rate).astype(np.int64)
    cols["r"] = (rng.random(n) < rate / 2).astype(np.int64)
    cols["nr"] = (rng.random(n) < rate / 2).astype(np.int64)
    df = pd.DataFrame({SESSION_LONG_NAMES[k]: v for k, v in cols.items()})
    if with_extra:
        df.insert(0, "Unnamed: 0", np.arange(n))
        df["zscored green"] = rng.standard_normal(n)
        df["centerOcc"] = (rng.random(n) < 0.3).astype(np.int64)
    return df, cols


def _ab_words(rew, left, right):
    """The 'word' the acquisition pipeline stores per trial: previous trial rewarded 'A' / 'a'
    (the first trial counts as rewarded), then this trial rewarded on the same side 'A', on
    the other 'B', unrewarded same 'a', other 'b'."""
    prev = lambda x: np.r_[True, x[:-1].astype(bool)]              # noqa: E731
    same = (left == prev(left)) & (right == prev(right))
    rw = rew.astype(bool)
    first = np.where(prev(rew), "A", "a")
    second = np.where(rw, np.where(same, "A", "B"), np.where(same, "a", "b"))
    return np.char.add(first, second).astype(object)


def signal_session(n_trials: int, seed: int, *, short_gap=0.3, missed_co=0.05,
                   no_photometry=0.05, no_lick=0.1, nan_rows=0.03, past_end=2, signal_tail=40,
                   channels=3):
    """(signal_df, table_df) in the layout gen_signal_df.generate_signal_df reads: a behaviour
    table of ``n_trials`` trials (MATLAB 1-based sample indices of center in/out, side in/out,
    first lick; reward, choice, 'word') over a photometry signal.  A fraction of inter-trial
    gaps is shorter than the default trial bounds (trials overlap, rows get duplicated), some
    center outs are carried into the next trial's sample (the repair loop), some trials lack
    photometry or a lick, some table rows carry NaN (dropped), and the last ``past_end``
    trials lie beyond the recording (their indices match no signal row)."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    # per trial: center in, +1..5 center out, +2..10 side in, +0..3 first lick, +5..30 side out
    d = np.stack([rng.integers(1, 6, n_trials), rng.integers(2, 11, n_trials),
                  rng.integers(5, 31, n_trials), rng.integers(0, 4, n_trials)], axis=1)
    gap = np.where(rng.random(n_trials) < short_gap, rng.integers(3, 18, n_trials),
                   rng.integers(18, 80, n_trials))
    span = d[:, 0] + d[:, 1] + d[:, 2] + gap
    ci = 30 + np.r_[0, np.cumsum(span)[:-1]]
    co = ci + d[:, 0]
    si = co + d[:, 1]
    so = si + d[:, 2]
    fl = si + d[:, 3]
    idx = np.stack([ci, co, si, so, fl], axis=1).astype(np.float64) + 1.0   # MATLAB 1-based
    n_sig = int(idx[max(0, n_trials - past_end - 1), 3]) + signal_tail if n_trials else 50
    carried = np.flatnonzero(rng.random(max(n_trials - 1, 0)) < missed_co)
    idx[carried, 1] = idx[carried + 1, 1]
    idx[rng.random(n_trials) < no_lick, 4] = 0.0
    left = (rng.random(n_trials) < 0.5).astype(np.int64)
    right = 1 - left
    right[rng.random(n_trials) < 0.03] = 0                                  # no choice
    rew = (rng.random(n_trials) < 0.6).astype(np.int64)
    table = pd.DataFrame({c: idx[:, j] for j, c in enumerate(
        ["photometryCenterInIndex", "photometryCenterOutIndex", "photometrySideInIndex",
         "photometrySideOutIndex", "photometryFirstLickIndex"])})
    table["hasAllPhotometryData"] = (rng.random(n_trials) >= no_photometry).astype(np.int64)
    table["wasRewarded"] = rew
    table["choseLeft"] = left
    table["choseRight"] = right
    table["word"] = _ab_words(rew, left, right)
    rt = rng.random(n_trials)
    rt[rng.random(n_trials) < nan_rows] = np.nan
    table["reactionTime"] = rt
    sig = pd.DataFrame({f"Ch{c + 1}": rng.standard_normal(n_sig) for c in range(channels)})
    sig["timestamp"] = np.arange(n_sig) / 20.0
    return sig, table


def designmat_session(n_trials: int, seed: int, *, lead=7, no_cue=0.03, timeout=0.08,
                      missing_trials=2, enlp_rate=0.25, lick_rate=0.06, cons_lick_rate=0.5,
                      nan_clock=0.01, photo=("z_grnR", "z_grnL")):
    """(timeseries, trials) in the layout pp_design_mat.make_design_mat reads, 50 Hz rows.

    Per trial, in order: Cue (4 rows), ENL (8-40 rows; with probability ``enlp_rate`` a
    penalised ENL repeated 1-3 times: ENLP / state_ENLP rows, nENL counting the ENL periods of
    the trial), Select (5-30 rows), Consumption (10-60 rows, stateConsumption spanning Select
    and Consumption), an ITI (5-20 rows).  iSpout is a spout id on lick rows (denser in
    Consumption), NaN elsewhere; trial_clock is ms since the trial start (a few NaN).  ``lead``
    rows before the first trial have NaN nTrial / nENL.  A fraction of trials lacks its cue
    rows (``no_cue``; flagged by make_design_mat), timeouts carry NaN Reward and tSelection,
    and the last ``missing_trials`` trial ids of the session are absent from the trial table
    (unmapped keys).  Vectorised: sizes of millions of rows are cheap."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    T = int(n_trials)
    L_cue = np.where(rng.random(T) < no_cue, 0, 4)
    L_enl = rng.integers(8, 41, T)
    n_enlp = np.where(rng.random(T) < enlp_rate, rng.integers(1, 4, T), 0)
    L_enlp = n_enlp * rng.integers(6, 15, T)
    L_sel = rng.integers(5, 31, T)
    L_con = rng.integers(10, 61, T)
    L_iti = rng.integers(5, 21, T)
    phases = np.stack([L_cue, L_enl, L_enlp, L_sel, L_con, L_iti], 1)    # T x 6 row counts
    per_trial = phases.sum(1)
    n = int(lead + per_trial.sum())
    trial_of_row = np.repeat(np.arange(T), per_trial)
    start = np.r_[0, np.cumsum(per_trial)[:-1]]
    pos = np.arange(n - lead) - np.repeat(start, per_trial)              # row within trial
    bounds = np.cumsum(phases, 1)
    b = bounds[trial_of_row]
    phase = (pos[:, None] >= b).sum(1)                                    # 0..5
    z = np.zeros(n)

    def col(mask):
        c = z.copy()
        c[lead:] = mask.astype(np.float64)
        return c
    ts = {}
    nt = np.full(n, np.nan)
    nt[lead:] = trial_of_row + 1.0
    ts["nTrial"] = nt
    blk = np.full(n, np.nan)
    blk[lead:] = (trial_of_row // 40).astype(np.float64)
    ts["iBlock"] = blk
    ts["Cue"] = col(phase == 0)
    ts["ENL"] = col(phase == 1)
    ts["ENLP"] = col(phase == 2)
    ts["state_ENLP"] = col(phase == 2)
    ts["Select"] = col(phase == 3)
    ts["Consumption"] = col(phase == 4)
    ts["stateConsumption"] = col((phase == 3) | (phase == 4))
    # nENL: 1 in the first ENL, then one more per penalised repeat (equal-length chunks)
    chunk = np.maximum(L_enlp // np.maximum(n_enlp, 1), 1)[trial_of_row]
    rep = np.where(phase == 2, (pos - bounds[trial_of_row, 1]) // chunk + 2, 1)
    ne = np.full(n, np.nan)
    ne[lead:] = np.where(phase >= 3, 1 + n_enlp[trial_of_row], rep).astype(np.float64)
    ts["nENL"] = ne
    clock = np.full(n, np.nan)
    clock[lead:] = pos * 20.0
    clock[rng.random(n) < nan_clock] = np.nan
    ts["trial_clock"] = clock
    lick_p = np.full(n, lick_rate)
    lick_p[lead:][phase == 4] = cons_lick_rate
    sp = np.where(rng.random(n) < lick_p, rng.integers(1, 3, n).astype(np.float64), np.nan)
    ts["iSpout"] = sp
    for p in photo:
        ts[p] = rng.standard_normal(n)
    timeseries = pd.DataFrame(ts)
    tsel = (L_cue + L_enl + L_enlp) * 20.0 + rng.integers(0, 200, T)
    to = rng.random(T) < timeout
    reward = np.where(to, np.nan, (rng.random(T) < 0.6).astype(np.float64))
    tsel = np.where(to, np.nan, tsel)
    h2 = rng.integers(0, 2, T).astype(np.float64)
    keep = T - int(missing_trials)
    trials = pd.DataFrame({"nTrial": np.arange(1, T + 1)[:keep], "tSelection": tsel[:keep],
                           "Reward": reward[:keep], "h2": h2[:keep]})
    return timeseries, trials


def prod_counters(trial: np.ndarray, seed: int = 0) -> np.ndarray:
    """The two unshifted continuous counters of the production design (pp_design_mat.py:167-172,
    sglm_cb_concat_make_design_mat.py:224, 310) over design rows with trial ids ``trial`` (rows of
    a trial contiguous): per trial a cue row and an ENL run (20-60 rows) from the trial's second
    row -- time_from_enl_onset = cumcount over the cue + ENL rows, squared / (50*100) -- and with
    probability 0.4 an ENLP run (8-20 rows) right after it -- time_from_enlp_onset likewise;
    0 elsewhere.  Returns float64 (2, N)."""
    rng = np.random.default_rng(seed)
    trial = np.asarray(trial)
    N = trial.size
    start = np.r_[0, np.flatnonzero(np.diff(trial) != 0) + 1]
    lens = np.diff(np.r_[start, N])
    T = start.size
    le = rng.integers(20, 61, T)
    lp = np.where(rng.random(T) < 0.4, rng.integers(8, 21, T), 0)
    pos = np.arange(N) - np.repeat(start, lens)                  # row within its trial
    ti = np.repeat(np.arange(T), lens)
    enl = pos <= le[ti]                                          # cue row 0 + ENL rows 1..le
    enlp = (pos > le[ti]) & (pos <= le[ti] + lp[ti])
    out = np.zeros((2, N))
    out[0] = np.where(enl, pos.astype(np.float64) ** 2 / 5000.0, 0.0)
    out[1] = np.where(enlp, (pos - le[ti] - 1).astype(np.float64) ** 2 / 5000.0, 0.0)
    return out


def ols_frame(N: int, m: int, neg: int, pos: int, seed: int = 0, rate=(0.005, 0.03),
              trial_len=(120, 360)):
    """A host session frame in the layout the reference's OLS drivers start from
    (er_refactored_from_scratch_cleanup.py:421-452; 02-create_features-lynne.ipynb): ``nTrial``
    (trials of ``trial_len`` rows), m float64 0/1 event columns ``e0 ..`` (Bernoulli per row at
    rates spread over ``rate``), and a Gaussian response ``y`` = the lag design (shifts 0,
    neg..-1, 1..pos, as sglm_ez.timeshift_cols) times random coefficients + intercept + noise,
    NaN on the first |neg| and last pos rows (where a lag leaves the recording).  Returns
    (DataFrame, event names, coefficient table [K][m] in timeshift_cols' shift order, intercept)."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    rates = np.linspace(rate[0], rate[1], m)
    E = (rng.random((N, m)) < rates[None, :]).astype(np.float64)
    lens = rng.integers(trial_len[0], trial_len[1] + 1, N // trial_len[0] + 2)
    trial = np.repeat(np.arange(1, lens.size + 1), lens)[:N].astype(np.float64)
    shifts = [0] + list(range(neg, 0)) + list(range(1, pos + 1))
    beta = rng.normal(0, 0.3, (len(shifts), m))
    b0 = 0.7
    y = np.full(N, b0)
    for bi, s in enumerate(shifts):
        contrib = E @ beta[bi]
        if s >= 0:
            y[s:] += contrib[:N - s]
        else:
            y[:N + s] += contrib[-s:]
    y += rng.normal(0, 1.0, N)
    y[:max(0, pos)] = np.nan
    if neg < 0:
        y[N + neg:] = np.nan
    ev = [f"e{a}" for a in range(m)]
    df = pd.DataFrame(E, columns=ev)
    df.insert(0, "nTrial", trial)
    df["y"] = y
    return df, ev, beta, b0


def cb_frame(N: int, m: int, neg: int, pos: int, sessions: int = 4, seed: int = 0,
             rate=(0.005, 0.03), trial_len=(120, 360), nan_frac=0.02):
    """A concatenated multi-session host frame in the layout sglm_cb_concat_make_design_mat.py
    starts from (:219-244: ``load_sessions.read_in_multi_sessions`` output): ``nTrial``,
    ``iBlock`` (trial-wide constants), ``session`` (a label per session), ``flag`` (1 on every row
    of ~10 % of the trials: timeouts, dropped after the shifts, :268), m float64 0/1 event
    columns ``e0 ..``, the two unshifted counters ``time_from_enl_onset`` /
    ``time_from_enlp_onset`` (prod_counters) and a photometry response ``grn`` that is NaN on
    short runs of rows (lost signal, dropped before the shifts, :251).  Over the rows that keep
    their signal, ``grn`` = the lag design (shifts 0, neg..-1, 1..pos of the compacted rows,
    sglm_ez.timeshift_cols' order) x coefficients + counters x gamma + a per-session offset
    + noise.  Returns (DataFrame, event names, coefficient table [K][m], gamma, session offsets)."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    rates = np.linspace(rate[0], rate[1], m)
    E = (rng.random((N, m)) < rates[None, :]).astype(np.float64)
    lens = rng.integers(trial_len[0], trial_len[1] + 1, N // trial_len[0] + 2)
    trial = np.repeat(np.arange(1, lens.size + 1), lens)[:N]
    ntr = int(trial.max())
    block = (trial - 1) // 20
    sess_of_trial = np.minimum((np.arange(1, ntr + 1) - 1) * sessions // ntr, sessions - 1)
    sess = sess_of_trial[trial - 1]
    flag_tr = (rng.random(ntr + 1) < 0.1).astype(np.int64)
    flag = flag_tr[trial]
    cnt = prod_counters(trial, seed=seed + 1)
    # lost-signal runs (NaN photometry), dropped before the shifts
    keep = np.ones(N, dtype=bool)
    nrun = max(1, int(N * nan_frac / 50))
    for s0 in rng.integers(0, max(1, N - 50), nrun):
        keep[s0:s0 + rng.integers(10, 50)] = False
    rows = np.flatnonzero(keep)
    Ek = E[rows]
    n = rows.size
    shifts = [0] + list(range(neg, 0)) + list(range(1, pos + 1))
    beta = rng.normal(0, 0.3, (len(shifts), m))
    gamma = np.array([0.8, -0.5])
    offs = rng.normal(0.5, 0.3, sessions)
    y = offs[sess[rows]] + gamma @ cnt[:, rows]
    for bi, s in enumerate(shifts):
        contrib = Ek @ beta[bi]
        if s >= 0:
            y[s:] += contrib[:n - s]
        else:
            y[:n + s] += contrib[-s:]
    y += rng.normal(0, 1.0, n)
    grn = np.full(N, np.nan)
    grn[rows] = y
    ev = [f"e{a}" for a in range(m)]
    df = pd.DataFrame(E, columns=ev)
    df.insert(0, "nTrial", trial.astype(np.int64))
    df.insert(1, "iBlock", block.astype(np.int64))
    df.insert(2, "session", np.array([f"2024-0{1 + q}-1{q}" for q in range(sessions)])[sess])
    df.insert(3, "flag", flag)
    df["time_from_enl_onset"] = cnt[0]
    df["time_from_enlp_onset"] = cnt[1]
    df["grn"] = grn
    return df, ev, beta, gamma, offs
