"""Where LagSource.upload's time goes on the box (development tool): the column views, the
threaded bit pack, the copy; and nan_counts' host parts."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    import bench
    import sglm_ez
    from sglm_hip import _lib, synth, lagframe
    from sglm_hip.engine import HOST_THREADS, _pinned
    N, m, L, K, nlam = bench.CONFIGS["c4"]
    s = synth.make(N=N, m=m, L=L, family="poisson", rho=0.02, seed=0)
    df, ev = bench.dropin_frame(s)
    print("HOST_THREADS", HOST_THREADS, "cpu_count", os.cpu_count(),
          "affinity", len(os.sched_getaffinity(0)))
    for rep in range(4):
        src = lagframe.LagSource(df)
        t0 = time.perf_counter()
        arrs = [src._f64(c) for c in ev]
        t1 = time.perf_counter()
        Nn = src.N
        nw = (Nn + 31) // 32
        bits = _pinned("lagbits_prof", max(1, m * nw), torch.int32)
        binary = np.zeros(m, dtype=np.uint8)
        ones = np.zeros(m, dtype=np.int64)
        ptrs = (ctypes.c_void_p * m)(*[a.ctypes.data for a in arrs])
        strides = np.array([a.strides[0] // 8 for a in arrs], dtype=np.int64)
        res = {}
        for th in (HOST_THREADS, 8, 32):
            t2 = time.perf_counter()
            _lib.call("sglm_host_pack_bits_cols", ctypes.cast(ptrs, ctypes.c_void_p),
                      strides.ctypes.data, m, Nn, bits.data_ptr(), binary.ctypes.data,
                      ones.ctypes.data, th)
            res[f"pack_t{th}"] = round(1e3 * (time.perf_counter() - t2), 2)
        t3 = time.perf_counter()
        bd = bits[: m * nw].view(m, nw).to("cuda", non_blocking=True)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        src2 = lagframe.LagSource(df)
        t5 = time.perf_counter()
        src2.upload(ev)
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        y = df["y"].to_numpy()
        t7 = time.perf_counter()
        na = np.isnan(y)
        t8 = time.perf_counter()
        print({"views": round(1e3 * (t1 - t0), 2), **res, "h2d": round(1e3 * (t4 - t3), 2),
               "upload": round(1e3 * (t6 - t5), 2), "isnan_y": round(1e3 * (t8 - t7), 2),
               "strides": int(strides[0])})


if __name__ == "__main__":
    main()
