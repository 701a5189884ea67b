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
            alg = 2.0 * sum(int(c) * ((m - a) * K + 1) for a, c in enumerate(lg.cnt)) * K * nact
            assert ex >= 0.5 * alg, (m, K, nact, ex, alg)     # both count each H entry once
            assert ex >= prev                                    # 32-column tiles: flat inside one
            prev = ex
        assert E._lagw_exec_flop(lg, 5) == lg.exec_flop[5]    # memoised per launch size
