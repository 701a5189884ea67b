"""Interleaved in-process A/B of engine knobs on the C4 grid (development tool).

python tools/grid_ab.py ROUNDS VARIANT [VARIANT ...]
  VARIANT = name:attr=value[,attr=value]   (attributes of sglm_hip.engine, grid.attr, or
            env.NAME for an environment switch the library reads per launch)
e.g.  python tools/grid_ab.py 6 base: split1:CHOL_SPLIT=1
Box-to-box clocks differ by 20 %+, so variants are compared inside one process on one
design, alternating grid by grid; prints the median and all wall times per variant.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def parse(v):
    name, _, kv = v.partition(":")
    out = []
    for item in filter(None, kv.split(",")):
        k, _, val = item.partition("=")
        out.append((k, type_of(val)))
    return name, out


def type_of(val):
    if val in ("True", "False"):
        return val == "True"
    for t in (int, float):
        try:
            return t(val)
        except ValueError:
            pass
    return val


def main():
    import pandas as pd
    import torch
    import bench
    from sglm_hip import engine as E, folds, grid, synth
    from sglm_hip.estimators import Objective
    rounds = int(sys.argv[1])
    variants = [parse(v) for v in sys.argv[2:]]
    N, m, L, K, nlam = bench.CONFIGS[os.environ.get("AB_CONFIG", "c4")]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    codes = folds.trial_keys_codes(pd.DataFrame({"nTrial": s.trial}), ["nTrial"]).values
    np.random.seed(3)
    cv_idx = folds.cv_idx_from_bucket_ids(codes, num_folds=K)
    objs = [Objective("irls", E.FAM_TWEEDIE_LOG, 1.0, float(al), "n", True, 100)
            for al in np.logspace(-4, 1, nlam)]
    mods = {"grid": grid}
    base = {}
    envs = set()
    for _, kv in variants:
        for k, _ in kv:
            if k.startswith("env."):
                envs.add(k[4:])
                continue
            mod, attr = (mods[k.split(".")[0]], k.split(".")[1]) if "." in k else (E, k)
            base.setdefault((mod, attr), getattr(mod, attr))
    env0 = {k: os.environ.get(k) for k in envs}

    def apply(kv):
        for (mod, attr), v in base.items():
            setattr(mod, attr, v)
        for k, v in env0.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for k, v in kv:
            if k.startswith("env."):
                os.environ[k[4:]] = str(v)
                continue
            mod, attr = (mods[k.split(".")[0]], k.split(".")[1]) if "." in k else (E, k)
            setattr(mod, attr, v)

    times = {name: [] for name, _ in variants}
    iters = {}
    for _, kv in variants:              # warm every variant (graph caches, allocator)
        apply(kv)
        for _ in range(2):
            grid.run(d, s.y, cv_idx, objs, [0] * nlam)
    for r in range(rounds):
        for name, kv in (variants if r % 2 == 0 else variants[::-1]):
            apply(kv)
            st = E.IrlsStats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            grid.run(d, s.y, cv_idx, objs, [0] * nlam, stats=st)
            torch.cuda.synchronize()
            times[name].append(round((time.perf_counter() - t0) * 1e3, 2))
            iters[name] = (st.fit_iters, st.gram_fits, st.newton_iters,
                           round(st.chain_host_s * 1e3, 2), round(st.sync_wait_s * 1e3, 2))
        print(json.dumps({"round": r, **{k: v[-1] for k, v in times.items()}}), flush=True)
    print(json.dumps({"median_ms": {k: float(np.median(v)) for k, v in times.items()},
                      "all_ms": times,
                      "fit_iters_grams_newton_chainhostms_syncwaitms": iters}))


if __name__ == "__main__":
    main()
