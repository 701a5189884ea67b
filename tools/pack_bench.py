"""Host bit-pack bandwidth on the box (development tool): sglm_host_pack_bits_cols over the
drop-in frame's 1M x 50 float64 event block at several thread counts, plus a plain memcpy and
a numpy sum of the same bytes for scale."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]
from sglm_hip import _lib
_lib.load()
n, m = 1_000_039, 52
A = (np.random.default_rng(0).random((n, m)) < 0.02).astype(np.float64)
nw = (n + 31) // 32
bits = np.zeros(m * nw, np.uint32); binary = np.zeros(m, np.uint8); ones = np.zeros(m, np.int64)
ptrs = (ctypes.c_void_p * m)(*[A.ctypes.data + 8 * c for c in range(m)])
strides = np.full(m, m, np.int64)
out = {}
for nt in (4, 8, 16, 32, 64):
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        _lib.call("sglm_host_pack_bits_cols", ctypes.cast(ptrs, ctypes.c_void_p), strides.ctypes.data,
                  m, n, bits.ctypes.data, binary.ctypes.data, ones.ctypes.data, nt)
        ts.append(time.perf_counter() - t)
    out[f"pack_t{nt}_ms"] = round(1e3 * min(ts), 2)
dst = np.empty_like(A)
for nt in (8, 16, 32):
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        _lib.call("sglm_host_copy", dst.ctypes.data, A.ctypes.data, A.nbytes, nt)
        ts.append(time.perf_counter() - t)
    out[f"copy_t{nt}_ms"] = round(1e3 * min(ts), 2)
t = time.perf_counter(); A.sum(); out["numpy_sum_ms"] = round(1e3 * (time.perf_counter() - t), 2)
out["bytes"] = A.nbytes
out["affinity_cpus"] = len(os.sched_getaffinity(0))
print(out)
