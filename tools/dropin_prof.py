"""Profile the drop-in production flow (bench.py dropin_grid) at a config: phases and the top
host functions (cProfile).  Usage on the box: python tools/dropin_prof.py [c4|c3]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sabatinilab-glm_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    from sglm_hip import synth
    N, m, L, K, nlam = bench.CONFIGS[cfg]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    df, ev = bench.dropin_frame(s)
    lams = np.logspace(-4, 1, nlam)
    for _ in range(2):
        bench.dropin_grid(df, ev, L, K, lams)
    for _ in range(2):
        t = time.perf_counter()
        _, ph = bench.dropin_grid(df, ev, L, K, lams)
        print(f"wall {1e3 * (time.perf_counter() - t):.1f} ms", {k: round(v * 1e3, 1) for k, v in ph.items()})
    pr = cProfile.Profile()
    pr.enable()
    bench.dropin_grid(df, ev, L, K, lams)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    pstats.Stats(pr).sort_stats("cumtime").print_stats(45)
    st = pstats.Stats(pr).sort_stats("cumtime")
    for fn in ("nan_counts", "_lag_nan_counts", "device", "design", "from_events",
               "trial_keys_codes", "group_shuffle_split", "_run", "run_multi"):
        st.print_callees(fn)


if __name__ == "__main__":
    main()
