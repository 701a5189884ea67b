"""Host-side figures of the event-structured Gram (engine._lagw_exec_flop): the MFMA work the
launch issues covers the structured products (the H entries' own terms) and does not shrink with the fit
count; no GPU needed."""
import numpy as np


class _Lag:
    def __init__(self, m, K, cnt):
        self.m, self.K, self.cnt = m, K, np.asarray(cnt)


def test_exec_flop_covers_the_algorithmic_products():
    from sglm_hip import engine as E
    rng = np.random.default_rng(0)
    for m, K in ((50, 40), (13, 10), (7, 41), (40, 12)):
        lg = _Lag(m, K, rng.integers(100, 30000, m))
        prev = 0.0
        for nact in (1, 2, 5, 14):
            ex = E._lagw_exec_flop(lg, nact)
            alg = E._lagw_alg_flop1(m, K, lg.cnt) * nact
            assert ex >= alg, (m, K, nact, ex, alg)   # the kernel's own decomposition, padded
            # every H entry of the upper triangle once: (mK(mK+1)/2 + mK) entries, each summing
            # the occurrences of one of its two events (equal counts: exactly that many terms)
            flat = E._lagw_alg_flop1(m, K, np.full(m, 7))
            pl = m * K
            assert flat == 2.0 * 7 * (pl * (pl + 1) // 2 + pl)
            assert ex >= prev                                    # 32-column tiles: flat inside one
            prev = ex
        assert E._lagw_exec_flop(lg, 5) == lg.exec_flop[5]    # memoised per launch size
